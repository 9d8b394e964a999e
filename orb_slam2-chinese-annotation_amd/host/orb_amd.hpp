// orb_amd.hpp -- C++ host mirror of ORB_SLAM2::ORBextractor / ORB_SLAM2::ORBmatcher
// over the C ABI (include/orb_abi.h).  Header-only, C++17, no OpenCV.
//
// Same member names, argument meaning and error behaviour as the reference
// classes (include/ORBextractor.h:45-114, include/ORBmatcher.h:37-102), with
// cv::Mat / cv::KeyPoint replaced by plain views:
//   cv::KeyPoint            -> orb_keypoint_t  (identical 28-byte layout)
//   cv::Mat N x 32 CV_8U    -> Descriptors      (row-major N x 32 bytes)
//   cv::Mat 8UC1 image      -> ImageView        (pointer, width, height, stride)
// The OpenCV-typed drop-in a maintainer compiles into the reference tree is in
// INTEGRATION.md; it forwards to these calls.
#pragma once

#include <cassert>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/orb_abi.h"

namespace orb_amd {

struct Error : std::runtime_error {
  orb_status_t status;
  Error(orb_status_t s, const std::string& what)
      : std::runtime_error(what + ": " + orb_status_string(s)), status(s) {}
};

inline void check(orb_status_t s, const char* what) {
  if (s != ORB_OK) throw Error(s, what);
}

using KeyPoint = orb_keypoint_t;

struct ImageView {
  const uint8_t* data = nullptr;
  int width = 0, height = 0;
  size_t stride = 0;  // bytes between rows
  bool empty() const { return !data || width <= 0 || height <= 0; }
};

struct Descriptors {
  int rows = 0;
  std::vector<uint8_t> data;  // rows x 32
  const uint8_t* row(int i) const { return data.data() + (size_t)i * ORB_DESC_BYTES; }
  bool empty() const { return rows == 0; }
};

struct Image {
  int width = 0, height = 0;
  std::vector<uint8_t> data;
  ImageView view() const { return {data.data(), width, height, (size_t)width}; }
};

// ---------------------------------------------------------------- extractor
class ORBextractor {
 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
               int device = 0) {
    check(orb_extractor_create(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device,
                               &h_),
          "ORBextractor");
  }
  ~ORBextractor() { orb_extractor_destroy(h_); }
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // operator()(image, mask, keypoints, descriptors) -- src/ORBextractor.cc:1091-1169.
  // Empty image: returns with the outputs untouched (:1095-1096).  The mask is
  // ignored, as in the reference (include/ORBextractor.h:58).
  void operator()(const ImageView& image, const ImageView& /*mask*/,
                  std::vector<KeyPoint>& keypoints, Descriptors& descriptors) {
    if (image.empty()) return;
    const int cap = orb_extractor_capacity(h_, image.width, image.height);
    assert(cap >= 0 && "image too small/large for this pyramid");  // reference: assert (:1100)
    if (cap < 0) throw Error(ORB_EINVAL, "ORBextractor::operator()");
    keypoints.resize(cap);
    descriptors.data.resize((size_t)cap * ORB_DESC_BYTES);
    int n = 0;
    check(orb_extractor_extract(h_, image.data, image.width, image.height, image.stride,
                                keypoints.data(), descriptors.data.data(), cap, &n),
          "ORBextractor::operator()");
    keypoints.resize(n);
    descriptors.data.resize((size_t)n * ORB_DESC_BYTES);
    descriptors.rows = n;
  }

  int GetLevels() { return orb_extractor_get_levels(h_); }
  float GetScaleFactor() { return orb_extractor_get_scale_factor(h_); }
  std::vector<float> GetScaleFactors() { return floats(orb_extractor_get_scale_factors); }
  std::vector<float> GetInverseScaleFactors() {
    return floats(orb_extractor_get_inverse_scale_factors);
  }
  std::vector<float> GetScaleSigmaSquares() { return floats(orb_extractor_get_scale_sigma_squares); }
  std::vector<float> GetInverseScaleSigmaSquares() {
    return floats(orb_extractor_get_inverse_scale_sigma_squares);
  }

  // mvImagePyramid (include/ORBextractor.h:85): host copies of the last image's levels.
  std::vector<Image> ImagePyramid() {
    std::vector<Image> out(GetLevels());
    for (int l = 0; l < (int)out.size(); ++l) {
      check(orb_extractor_pyramid_level(h_, l, nullptr, 0, &out[l].width, &out[l].height),
            "mvImagePyramid");
      out[l].data.resize((size_t)out[l].width * out[l].height);
      check(orb_extractor_pyramid_level(h_, l, out[l].data.data(), out[l].width, nullptr, nullptr),
            "mvImagePyramid");
    }
    return out;
  }

  orb_extractor_t* handle() { return h_; }

 private:
  std::vector<float> floats(void (*fn)(const orb_extractor_t*, float*)) {
    std::vector<float> v(GetLevels());
    fn(h_, v.data());
    return v;
  }
  orb_extractor_t* h_ = nullptr;
};

// ------------------------------------------------------------------ matcher
// The matcher-side Frame / MapPoint state, flattened (what ORBmatcher reads).
struct FrameView {
  std::vector<KeyPoint> mvKeysUn;
  Descriptors mDescriptors;
  std::vector<float> mvuRight;  // empty = monocular
  float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
  std::vector<float> mvScaleFactors;
  int N() const { return (int)mvKeysUn.size(); }
  orb_frame_t c() const {
    orb_frame_t f;
    f.n = N();
    f.keys = mvKeysUn.data();
    f.descriptors = mDescriptors.data.data();
    f.u_right = mvuRight.empty() ? nullptr : mvuRight.data();
    f.min_x = mnMinX;
    f.max_x = mnMaxX;
    f.min_y = mnMinY;
    f.max_y = mnMaxY;
    f.n_levels = (int)mvScaleFactors.size();
    f.scale_factors = mvScaleFactors.data();
    return f;
  }
};

class ORBmatcher {
 public:
  static const int TH_LOW = 50;
  static const int TH_HIGH = 100;
  static const int HISTO_LENGTH = 30;

  explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, int device = 0)
      : mfNNratio(nnratio), mbCheckOrientation(checkOri) {
    check(orb_matcher_create(device, &h_), "ORBmatcher");
  }
  ~ORBmatcher() { orb_matcher_destroy(h_); }
  ORBmatcher(const ORBmatcher&) = delete;
  ORBmatcher& operator=(const ORBmatcher&) = delete;

  // static int DescriptorDistance(const cv::Mat&, const cv::Mat&) -- src/ORBmatcher.cc:1814-1830
  static int DescriptorDistance(const uint8_t* a, const uint8_t* b) {
    return orb_descriptor_distance(a, b);
  }

  // SearchByProjection(Frame&, const vector<MapPoint*>&, th) -- src/ORBmatcher.cc:47-133.
  // mvpMapPoints[i] is the map-point index assigned to keypoint i (-1 = NULL);
  // on entry locked[i] = (mvpMapPoints[i] && Observations() > 0).  Returns nmatches.
  int SearchByProjection(const FrameView& F, const std::vector<orb_mp_track_t>& mps,
                         const std::vector<uint8_t>& mpDescriptors, float th,
                         std::vector<int32_t>& mvpMapPoints,
                         const std::vector<uint8_t>& locked = {}) {
    const orb_frame_t f = F.c();
    std::vector<int32_t> km(F.N(), -1);
    int32_t n = 0;
    check(orb_match_projection_local(h_, &f, locked.empty() ? nullptr : locked.data(),
                                     (int)mps.size(), mps.data(), mpDescriptors.data(), th,
                                     mfNNratio, km.data(), &n),
          "SearchByProjection");
    if ((int)mvpMapPoints.size() != F.N()) mvpMapPoints.assign(F.N(), -1);
    for (int i = 0; i < F.N(); ++i)
      if (km[i] >= 0) mvpMapPoints[i] = km[i];
    return n;
  }

  // SearchByProjection(CurrentFrame, LastFrame, th, bMono) -- src/ORBmatcher.cc:1460-1619.
  int SearchByProjection(const FrameView& current, const std::vector<orb_last_mp_t>& last,
                         const std::vector<uint8_t>& lastDescriptors, const orb_camera_t& cam,
                         float tlc_z, float th, bool bMono, std::vector<int32_t>& mvpMapPoints,
                         const std::vector<uint8_t>& locked = {}) {
    const orb_frame_t f = current.c();
    std::vector<int32_t> km(current.N(), -1);
    int32_t n = 0;
    check(orb_match_projection_frame(h_, &f, locked.empty() ? nullptr : locked.data(),
                                     (int)last.size(), last.data(), lastDescriptors.data(), &cam,
                                     tlc_z, th, bMono ? 1 : 0, mbCheckOrientation ? 1 : 0,
                                     km.data(), &n),
          "SearchByProjection(F, LastFrame)");
    if ((int)mvpMapPoints.size() != current.N()) mvpMapPoints.assign(current.N(), -1);
    for (int i = 0; i < current.N(); ++i) {
      if (km[i] >= 0) mvpMapPoints[i] = km[i];
      else if (km[i] == -2) mvpMapPoints[i] = -1;  // rotation filter reset
    }
    return n;
  }

  // Frame::ComputeStereoMatches -- src/Frame.cc:516-704 (mvuRight, mvDepth).
  void ComputeStereoMatches(const FrameView& left, const std::vector<KeyPoint>& rightKeys,
                            const Descriptors& rightDesc, const std::vector<Image>& leftPyr,
                            const std::vector<Image>& rightPyr,
                            const std::vector<float>& invScale, float bf, float fx,
                            std::vector<float>& mvuRight, std::vector<float>& mvDepth) {
    const int L = (int)leftPyr.size();
    std::vector<const uint8_t*> lp(L), rp(L);
    std::vector<int32_t> w(L), hh(L);
    std::vector<int64_t> st(L);
    for (int l = 0; l < L; ++l) {
      lp[l] = leftPyr[l].data.data();
      rp[l] = rightPyr[l].data.data();
      w[l] = leftPyr[l].width;
      hh[l] = leftPyr[l].height;
      st[l] = leftPyr[l].width;
    }
    const orb_frame_t f = left.c();
    orb_stereo_input_t in;
    in.left = &f;
    in.n_right = (int)rightKeys.size();
    in.right_keys = rightKeys.data();
    in.right_desc = rightDesc.data.data();
    in.n_levels = L;
    in.left_levels = lp.data();
    in.right_levels = rp.data();
    in.level_width = w.data();
    in.level_height = hh.data();
    in.level_stride = st.data();
    in.inv_scale_factors = invScale.data();
    in.bf = bf;
    in.fx = fx;
    mvuRight.assign(left.N(), -1.0f);
    mvDepth.assign(left.N(), -1.0f);
    check(orb_stereo_match(h_, &in, mvuRight.data(), mvDepth.data()), "ComputeStereoMatches");
  }

  float mfNNratio;
  bool mbCheckOrientation;
  orb_matcher_t* handle() { return h_; }

 private:
  orb_matcher_t* h_ = nullptr;
};

}  // namespace orb_amd
