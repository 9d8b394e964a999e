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
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
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

// --------------------------------------------------------------- DBoW2 types
// DBoW2::BowVector (std::map<WordId, WordValue>, Thirdparty/DBoW2/DBoW2/BowVector.h)
// and DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>,
// FeatureVector.h): the same containers, so Frame::mBowVec / mFeatVec keep their
// types.  CsrFeatureVector is the flat form the C ABI takes.
using WordId = uint32_t;
using NodeId = uint32_t;
using BowVector = std::map<WordId, double>;
using FeatureVector = std::map<NodeId, std::vector<unsigned int>>;

struct CsrFeatureVector {
  std::vector<uint32_t> nodes;
  std::vector<int32_t> offs{0};
  std::vector<uint32_t> feats;
  int size() const { return (int)nodes.size(); }
};

inline CsrFeatureVector flatten(const FeatureVector& fv) {
  CsrFeatureVector c;
  c.nodes.reserve(fv.size());
  c.offs.reserve(fv.size() + 1);
  for (const auto& it : fv) {
    c.nodes.push_back(it.first);
    c.feats.insert(c.feats.end(), it.second.begin(), it.second.end());
    c.offs.push_back((int32_t)c.feats.size());
  }
  return c;
}

// ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
// (include/ORBVocabulary.h), device-resident.  loadFromTextFile as
// TemplatedVocabulary.h:1362-1448 (returns false on a malformed header);
// transform as Frame::ComputeBoW calls it (src/Frame.cc:439-449:
// transform(vCurrentDesc, mBowVec, mFeatVec, 4)).
class ORBVocabulary {
 public:
  explicit ORBVocabulary(int device = 0) : device_(device) {}
  ~ORBVocabulary() { orb_vocabulary_destroy(h_); }
  ORBVocabulary(const ORBVocabulary&) = delete;
  ORBVocabulary& operator=(const ORBVocabulary&) = delete;

  bool loadFromTextFile(const std::string& filename) {
    orb_vocabulary_t* h = nullptr;
    if (orb_vocabulary_load_text(device_, filename.c_str(), &h) != ORB_OK) return false;
    orb_vocabulary_destroy(h_);
    h_ = h;
    return true;
  }
  // Node table form (node 0 = root; parent[i] < i; entry 0 ignored).
  void create(int k, int L, int scoring, int weighting, const std::vector<int32_t>& parent,
              const std::vector<uint8_t>& leaf, const std::vector<uint8_t>& descriptors,
              const std::vector<double>& weights) {
    orb_vocabulary_t* h = nullptr;
    check(orb_vocabulary_create(device_, k, L, scoring, weighting, (int)parent.size(),
                                parent.data(), leaf.data(), descriptors.data(), weights.data(),
                                &h),
          "ORBVocabulary::create");
    orb_vocabulary_destroy(h_);
    h_ = h;
  }
  unsigned int size() const { return (unsigned)info()[5]; }
  bool empty() const { return size() == 0; }
  unsigned int getBranchingFactor() const { return (unsigned)info()[0]; }
  unsigned int getDepthLevels() const { return (unsigned)info()[1]; }

  // transform(const vector<cv::Mat>& features, BowVector&, FeatureVector&, levelsup),
  // TemplatedVocabulary.h:1128-1210; desc rows are the features in order.
  void transform(const Descriptors& desc, BowVector& v, FeatureVector& fv, int levelsup) const {
    v.clear();
    fv.clear();
    if (!h_ || desc.rows == 0) return;
    const int n = desc.rows;
    std::vector<uint32_t> bw(n), fvn(n), fvf(n);
    std::vector<double> bv(n);
    std::vector<int32_t> fvo(n + 1);
    int32_t nw = 0, nf = 0;
    check(orb_vocabulary_transform(h_, n, desc.data.data(), levelsup, bw.data(), bv.data(), &nw,
                                   fvn.data(), fvo.data(), fvf.data(), &nf, nullptr, nullptr),
          "ORBVocabulary::transform");
    for (int i = 0; i < nw; ++i) v.emplace_hint(v.end(), bw[i], bv[i]);
    for (int j = 0; j < nf; ++j)
      fv.emplace_hint(fv.end(), fvn[j],
                      std::vector<unsigned int>(fvf.begin() + fvo[j], fvf.begin() + fvo[j + 1]));
  }
  orb_vocabulary_t* handle() { return h_; }

 private:
  std::vector<int32_t> info() const {
    std::vector<int32_t> i(6, 0);
    if (h_) orb_vocabulary_info(h_, i.data());
    return i;
  }
  int device_;
  orb_vocabulary_t* h_ = nullptr;
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

  // SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches),
  // src/ORBmatcher.cc:164-306.  kfMapPoints[i] = MapPoint id of KF keypoint i or
  // -1; kfBad[i] = isBad().  vpMapPointMatches (out) = MapPoint id per F keypoint.
  int SearchByBoW(const FrameView& KF, const std::vector<int32_t>& kfMapPoints,
                  const std::vector<uint8_t>& kfBad, const FeatureVector& kfFeatVec,
                  const FrameView& F, const FeatureVector& fFeatVec,
                  std::vector<int32_t>& vpMapPointMatches) {
    const CsrFeatureVector a = flatten(kfFeatVec), b = flatten(fFeatVec);
    const std::vector<float> ka = angles(KF), fa = angles(F);
    vpMapPointMatches.assign(F.N(), -1);
    int32_t n = 0;
    check(orb_match_bow(h_, KF.N(), KF.mDescriptors.data.data(), ka.data(), kfMapPoints.data(),
                        kfBad.empty() ? nullptr : kfBad.data(), a.size(), a.nodes.data(),
                        a.offs.data(), a.feats.data(), F.N(), F.mDescriptors.data.data(),
                        fa.data(), b.size(), b.nodes.data(), b.offs.data(), b.feats.data(),
                        mfNNratio, mbCheckOrientation ? 1 : 0, vpMapPointMatches.data(), &n),
          "SearchByBoW(KF, F)");
    return n;
  }

  // SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12),
  // src/ORBmatcher.cc:581-716.  vpMatches12 (out) = KF2 MapPoint id per KF1 keypoint.
  int SearchByBoW(const FrameView& KF1, const std::vector<int32_t>& mp1,
                  const std::vector<uint8_t>& bad1, const FeatureVector& fv1,
                  const FrameView& KF2, const std::vector<int32_t>& mp2,
                  const std::vector<uint8_t>& bad2, const FeatureVector& fv2,
                  std::vector<int32_t>& vpMatches12) {
    const CsrFeatureVector a = flatten(fv1), b = flatten(fv2);
    const std::vector<float> a1 = angles(KF1), a2 = angles(KF2);
    vpMatches12.assign(KF1.N(), -1);
    int32_t n = 0;
    check(orb_match_bow_kf(h_, KF1.N(), KF1.mDescriptors.data.data(), a1.data(), mp1.data(),
                           bad1.empty() ? nullptr : bad1.data(), a.size(), a.nodes.data(),
                           a.offs.data(), a.feats.data(), KF2.N(), KF2.mDescriptors.data.data(),
                           a2.data(), mp2.data(), bad2.empty() ? nullptr : bad2.data(), b.size(),
                           b.nodes.data(), b.offs.data(), b.feats.data(), mfNNratio,
                           mbCheckOrientation ? 1 : 0, vpMatches12.data(), &n),
          "SearchByBoW(KF, KF)");
    return n;
  }

  // SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize),
  // src/ORBmatcher.cc:429-577.  vbPrevMatched as (x, y) pairs, updated in place.
  int SearchForInitialization(const FrameView& F1, const FrameView& F2,
                              std::vector<float>& vbPrevMatched, std::vector<int>& vnMatches12,
                              int windowSize = 10) {
    const orb_frame_t f1 = F1.c(), f2 = F2.c();
    std::vector<int32_t> m(F1.N(), -1);
    int32_t n = 0;
    check(orb_search_for_initialization(h_, &f1, &f2, vbPrevMatched.data(), windowSize,
                                        mfNNratio, mbCheckOrientation ? 1 : 0, m.data(), &n),
          "SearchForInitialization");
    vnMatches12.assign(m.begin(), m.end());
    return n;
  }

  // Tracking::SearchLocalPoints' isInFrustum pass (src/Tracking.cc:1360-1377,
  // src/Frame.cc:303-366); returns nToMatch, tracks feed SearchByProjection.
  int isInFrustum(const std::vector<orb_map_point_t>& mps, const orb_pose_t& pose,
                  const orb_camera_t& cam, const FrameView& F, float viewingCosLimit,
                  float logScaleFactor, std::vector<orb_mp_track_t>& tracks) {
    tracks.assign(mps.size(), orb_mp_track_t{});
    int32_t n = 0;
    check(orb_frustum(h_, (int)mps.size(), mps.data(), &pose, &cam, F.mnMinX, F.mnMaxX, F.mnMinY,
                      F.mnMaxY, viewingCosLimit, logScaleFactor, (int)F.mvScaleFactors.size(),
                      tracks.data(), &n),
          "isInFrustum");
    return n;
  }

  // MapPoint::ComputeDistinctiveDescriptors for many points (src/MapPoint.cc:250-326):
  // observation descriptors in CSR (obsOffs.size() = points + 1).  Returns BestIdx
  // per point (-1 for an empty list, whose descriptor row is left untouched).
  std::vector<int32_t> ComputeDistinctiveDescriptors(const std::vector<int32_t>& obsOffs,
                                                     const std::vector<uint8_t>& obsDesc,
                                                     std::vector<uint8_t>& descriptors) {
    const int n = (int)obsOffs.size() - 1;
    std::vector<int32_t> best(n > 0 ? n : 0, -1);
    if (n <= 0) return best;
    descriptors.resize((size_t)n * ORB_DESC_BYTES);
    check(orb_distinctive_descriptors(h_, n, obsOffs.data(),
                                      obsDesc.empty() ? nullptr : obsDesc.data(), best.data(),
                                      descriptors.data()),
          "ComputeDistinctiveDescriptors");
    return best;
  }

  // Fuse(KeyFrame* pKF, vpMapPoints, th), src/ORBmatcher.cc:903-1077 (match half):
  // fuseIdx[i] = keypoint point i fuses into, or -1.
  int Fuse(const FrameView& KF, const std::vector<float>& invLevelSigma2, const orb_pose_t& pose,
           const orb_camera_t& cam, float logScaleFactor,
           const std::vector<orb_map_point_t>& mps, const std::vector<uint8_t>& mpDesc, float th,
           std::vector<int32_t>& fuseIdx) {
    const orb_frame_t f = KF.c();
    fuseIdx.assign(mps.size(), -1);
    int32_t n = 0;
    check(orb_fuse(h_, &f, invLevelSigma2.data(), &pose, &cam, logScaleFactor, (int)mps.size(),
                   mps.data(), mpDesc.data(), th, fuseIdx.data(), &n),
          "Fuse");
    return n;
  }

  // Fuse(KeyFrame* pKF, Scw, vpPoints, th, vpReplacePoint), src/ORBmatcher.cc:1079-1210.
  int Fuse(const FrameView& KF, const float scw[12], const orb_camera_t& cam,
           float logScaleFactor, const std::vector<orb_map_point_t>& mps,
           const std::vector<uint8_t>& mpDesc, float th, std::vector<int32_t>& fuseIdx) {
    const orb_frame_t f = KF.c();
    fuseIdx.assign(mps.size(), -1);
    int32_t n = 0;
    check(orb_fuse_sim3(h_, &f, scw, &cam, logScaleFactor, (int)mps.size(), mps.data(),
                        mpDesc.data(), th, fuseIdx.data(), &n),
          "Fuse(KF, Scw)");
    return n;
  }

  // SearchByProjection(Frame& F, KeyFrame* pKF, sAlreadyFound, th, ORBdist),
  // src/ORBmatcher.cc:1622-1759: kpMatch[j] = point assigned, -1 none, -2 reset.
  int SearchByProjection(const FrameView& F, const std::vector<uint8_t>& locked,
                         const orb_pose_t& pose, const orb_camera_t& cam, float logScaleFactor,
                         const std::vector<orb_map_point_t>& mps,
                         const std::vector<uint8_t>& mpDesc, const std::vector<float>& kfAngle,
                         float th, int ORBdist, std::vector<int32_t>& kpMatch) {
    const orb_frame_t f = F.c();
    kpMatch.assign(F.N(), -1);
    int32_t n = 0;
    check(orb_search_by_projection_reloc(h_, &f, locked.empty() ? nullptr : locked.data(), &pose,
                                         &cam, logScaleFactor, (int)mps.size(), mps.data(),
                                         mpDesc.data(), kfAngle.data(), th, ORBdist,
                                         mbCheckOrientation ? 1 : 0, kpMatch.data(), &n),
          "SearchByProjection(F, KF)");
    return n;
  }

  // SearchByProjection(KeyFrame* pKF, Scw, vpPoints, vpMatched, th),
  // src/ORBmatcher.cc:311-425: vpMatched[j] = index into vpPoints or -1 (in/out).
  int SearchByProjection(const FrameView& KF, const float scw[12], const orb_camera_t& cam,
                         float logScaleFactor, const std::vector<orb_map_point_t>& mps,
                         const std::vector<uint8_t>& mpDesc, std::vector<int32_t>& vpMatched,
                         int th) {
    const orb_frame_t f = KF.c();
    if ((int)vpMatched.size() != KF.N()) vpMatched.assign(KF.N(), -1);
    int32_t n = 0;
    check(orb_search_by_projection_sim3(h_, &f, scw, &cam, logScaleFactor, (int)mps.size(),
                                        mps.data(), mpDesc.data(), (float)th, vpMatched.data(),
                                        &n),
          "SearchByProjection(KF, Scw)");
    return n;
  }

  // SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo),
  // src/ORBmatcher.cc:718-901.  hasMp[i] = GetMapPoint(i) != NULL; levelSigma2 =
  // pKF2->mvLevelSigma2; F12 row-major; Cw = pKF1 camera centre; R2w/t2w = pKF2
  // pose.  vMatchedPairs (out) = (i1, i2) in ascending i1.
  int SearchForTriangulation(const FrameView& KF1, const std::vector<uint8_t>& hasMp1,
                             const FeatureVector& fv1, const FrameView& KF2,
                             const std::vector<uint8_t>& hasMp2, const FeatureVector& fv2,
                             const std::vector<float>& levelSigma2, const float F12[9],
                             const orb_camera_t& cam, const float Cw[3], const float R2w[9],
                             const float t2w[3], bool bOnlyStereo,
                             std::vector<std::pair<size_t, size_t>>& vMatchedPairs) {
    const orb_frame_t f1 = KF1.c(), f2 = KF2.c();
    const CsrFeatureVector a = flatten(fv1), b = flatten(fv2);
    std::vector<int32_t> m12(KF1.N(), -1);
    int32_t n = 0;
    check(orb_search_for_triangulation(h_, &f1, hasMp1.data(), &f2, hasMp2.data(),
                                       levelSigma2.data(), F12, &cam, Cw, R2w, t2w, a.size(),
                                       a.nodes.data(), a.offs.data(), a.feats.data(), b.size(),
                                       b.nodes.data(), b.offs.data(), b.feats.data(),
                                       bOnlyStereo ? 1 : 0, mbCheckOrientation ? 1 : 0,
                                       m12.data(), &n),
          "SearchForTriangulation");
    vMatchedPairs.clear();
    vMatchedPairs.reserve(n);
    for (int i = 0; i < KF1.N(); ++i)
      if (m12[i] >= 0) vMatchedPairs.emplace_back((size_t)i, (size_t)m12[i]);
    return n;
  }

  // SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th), src/ORBmatcher.cc:1212-1458.
  // mpsX / mpDescX = the MapPoint of keypoint i of KF X (validX[i] = non-NULL),
  // alreadyX = vbAlreadyMatchedX.  vpMatches12 (out) = idx2 per KF1 keypoint, or -1.
  int SearchBySim3(const FrameView& KF1, const FrameView& KF2, float logScaleFactor,
                   const orb_camera_t& cam, const float R1w[9], const float t1w[3],
                   const float R2w[9], const float t2w[3],
                   const std::vector<orb_map_point_t>& mps1, const std::vector<uint8_t>& valid1,
                   const std::vector<uint8_t>& already1, const std::vector<uint8_t>& mpDesc1,
                   const std::vector<orb_map_point_t>& mps2, const std::vector<uint8_t>& valid2,
                   const std::vector<uint8_t>& already2, const std::vector<uint8_t>& mpDesc2,
                   float s12, const float R12[9], const float t12[3], float th,
                   std::vector<int32_t>& vpMatches12) {
    const orb_frame_t f1 = KF1.c(), f2 = KF2.c();
    vpMatches12.assign(KF1.N(), -1);
    int32_t n = 0;
    check(orb_search_by_sim3(h_, &f1, &f2, logScaleFactor, &cam, R1w, t1w, R2w, t2w, mps1.data(),
                             valid1.data(), already1.data(), mpDesc1.data(), mps2.data(),
                             valid2.data(), already2.data(), mpDesc2.data(), s12, R12, t12, th,
                             vpMatches12.data(), &n),
          "SearchBySim3");
    return n;
  }

  // Frame::UndistortKeyPoints (src/Frame.cc:452-482): mvKeysUn from mvKeys with
  // cv::undistortPoints(mat, mat, mK, mDistCoef, cv::Mat(), mK).  K = mK row-major.
  void UndistortKeyPoints(const std::vector<KeyPoint>& mvKeys, const float K[9],
                          const std::vector<float>& mDistCoef, std::vector<KeyPoint>& mvKeysUn) {
    mvKeysUn.resize(mvKeys.size());
    check(orb_undistort_keypoints(h_, (int)mvKeys.size(), mvKeys.data(), K, mDistCoef.data(),
                                  (int)mDistCoef.size(), mvKeysUn.data()),
          "UndistortKeyPoints");
  }

  // Frame::ComputeImageBounds (src/Frame.cc:484-514) -> F.mnMinX .. mnMaxY.
  void ComputeImageBounds(int cols, int rows, const float K[9],
                          const std::vector<float>& mDistCoef, FrameView& F) {
    float b[4];
    check(orb_compute_image_bounds(h_, cols, rows, K, mDistCoef.data(), (int)mDistCoef.size(), b),
          "ComputeImageBounds");
    F.mnMinX = b[0];
    F.mnMaxX = b[1];
    F.mnMinY = b[2];
    F.mnMaxY = b[3];
  }

  float mfNNratio;
  bool mbCheckOrientation;
  orb_matcher_t* handle() { return h_; }

 private:
  static std::vector<float> angles(const FrameView& F) {
    std::vector<float> a(F.N());
    for (int i = 0; i < F.N(); ++i) a[i] = F.mvKeysUn[i].angle;
    return a;
  }
  orb_matcher_t* h_ = nullptr;
};

}  // namespace orb_amd
