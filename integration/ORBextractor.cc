// integration/ORBextractor.cc -- drop-in replacement for src/ORBextractor.cc of
// ORB_SLAM2 (yg838457845/ORB_SLAM2-Chinese-annotation): every member of
// include/ORBextractor.h:45-114 forwards to the MI355X C ABI
// (include/orb_abi.h, lib/liborb_amd.so).
//
// Header change: include/ORBextractor.h gains
//   #include "orb_abi.h"
//   public:  orb_extractor_t* gpu() const { return mpGpu; }
//   protected: orb_extractor_t* mpGpu = nullptr;
// and its inline destructor becomes `~ORBextractor(){ orb_extractor_destroy(mpGpu); }`.
// Frame.cc and Tracking.cc compile unchanged.
//
// mvImagePyramid (public, read by Frame::ComputeStereoMatches,
// src/Frame.cc:524,619,633,639) points at the library's pinned host mirror of
// the call's levels after each call (orb_extractor_host_pyramid).
// With ORB_AMD_GPU_STEREO defined (and integration/FrameStereo.cc replacing
// Frame::ComputeStereoMatches) nothing reads it on the host, and the copy is
// skipped: keypoints, descriptors and pyramids then stay in HBM for stereo.
#include "ORBextractor.h"

#include <cassert>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>
#include <opencv2/imgproc/imgproc.hpp>

#include "orb_abi.h"

using namespace cv;
using namespace std;

namespace ORB_SLAM2 {

static_assert(sizeof(cv::KeyPoint) == sizeof(orb_keypoint_t), "cv::KeyPoint is 28 bytes");

static void check(orb_status_t st, const char* what) {
  if (st != ORB_OK)
    throw std::runtime_error(std::string("ORBextractor::") + what + ": " + orb_status_string(st));
}

// src/ORBextractor.cc:428-489: the scale tables, per-level quotas and umax are
// computed by the library with the reference's float/double expressions and
// read back through the getters.
ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST,
                           int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels),
      iniThFAST(_iniThFAST), minThFAST(_minThFAST) {
  const char* dev = getenv("ORB_AMD_DEVICE");
  check(orb_extractor_create(nfeatures, (float)scaleFactor, nlevels, iniThFAST, minThFAST,
                             dev ? atoi(dev) : 0, &mpGpu),
        "ORBextractor");
  mvScaleFactor.resize(nlevels);
  orb_extractor_get_scale_factors(mpGpu, mvScaleFactor.data());
  mvInvScaleFactor.resize(nlevels);
  orb_extractor_get_inverse_scale_factors(mpGpu, mvInvScaleFactor.data());
  mvLevelSigma2.resize(nlevels);
  orb_extractor_get_scale_sigma_squares(mpGpu, mvLevelSigma2.data());
  mvInvLevelSigma2.resize(nlevels);
  orb_extractor_get_inverse_scale_sigma_squares(mpGpu, mvInvLevelSigma2.data());
  mnFeaturesPerLevel.resize(nlevels);
  orb_extractor_get_features_per_level(mpGpu, mnFeaturesPerLevel.data());
  mvImagePyramid.resize(nlevels);
}

// src/ORBextractor.cc:1091-1169.  The mask is ignored, as in the reference.
void ORBextractor::operator()(InputArray _image, InputArray _mask, vector<KeyPoint>& _keypoints,
                              OutputArray _descriptors) {
  (void)_mask;
  if (_image.empty()) return;  // :1095-1096, outputs untouched
  Mat image = _image.getMat();
  assert(image.type() == CV_8UC1);  // :1100
  const int cap = orb_extractor_capacity(mpGpu, image.cols, image.rows);
  if (cap < 0) throw std::runtime_error("ORBextractor::operator(): unsupported image size");
  // the library writes up to `cap` records; they land in per-thread scratch kept
  // across calls (sizing the caller's vector to `cap` first value-initialised
  // thousands of KeyPoints per frame, and a fresh descriptor Mat each call)
  thread_local std::vector<KeyPoint> kpScratch;
  thread_local std::vector<uint8_t> descScratch;
  if ((int)kpScratch.size() < cap) kpScratch.resize(cap);
  if (descScratch.size() < (size_t)cap * 32) descScratch.resize((size_t)cap * 32);
  int n = 0;
  check(orb_extractor_extract(mpGpu, image.ptr<uint8_t>(), image.cols, image.rows, image.step,
                              reinterpret_cast<orb_keypoint_t*>(kpScratch.data()),
                              descScratch.data(), cap, &n),
        "operator()");
  _keypoints.assign(kpScratch.begin(), kpScratch.begin() + n);  // :1127-1128 clears and refills
  if (n == 0)
    _descriptors.release();  // :1118-1121
  else
    Mat(n, 32, CV_8U, descScratch.data(), 32).copyTo(_descriptors);
#ifndef ORB_AMD_GPU_STEREO
  // mvImagePyramid aliases the library's pinned host mirror of this call's
  // levels (one DMA in the call's graph, no copy here), valid until the next
  // call, as the reference's own levels are rebuilt on every call
  for (int l = 0; l < nlevels; ++l) {
    const uint8_t* p = nullptr;
    int w = 0, h = 0;
    size_t step = 0;
    check(orb_extractor_host_pyramid(mpGpu, l, &p, &w, &h, &step), "mvImagePyramid");
    mvImagePyramid[l] = Mat(h, w, CV_8U, const_cast<uint8_t*>(p), step);
  }
#endif
}

}  // namespace ORB_SLAM2
