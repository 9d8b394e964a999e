// integration/ORBmatcher.cc -- drop-in replacement for src/ORBmatcher.cc of
// ORB_SLAM2 (yg838457845/ORB_SLAM2-Chinese-annotation).  Every member keeps the
// signature of include/ORBmatcher.h:41-83; each flattens the Frame / KeyFrame /
// MapPoint state its reference body reads into the C structs of
// include/orb_abi.h, runs the MI355X kernels (lib/liborb_amd.so), and applies
// the results to the caller's objects in the reference's order.
//
// Build: replace src/ORBmatcher.cc with this file, add three accessors to class
// MapPoint (include/MapPoint.h):
//   float GetMinDistance(){ unique_lock<mutex> lock(mMutexPos); return mfMinDistance; }
//   float GetMaxDistance(){ unique_lock<mutex> lock(mMutexPos); return mfMaxDistance; }
//   void CopyDescriptor(unsigned char* dst){ unique_lock<mutex> lock(mMutexFeatures);
//                                            memcpy(dst, mDescriptor.data, 32); }
// (the projection variants need the unscaled limits that PredictScale and
// Get{Min,Max}DistanceInvariance use), add -I<repo>/include and
// -L<repo>/orb_slam2-chinese-annotation_amd/lib -lorb_amd.  Tracking.cc, LocalMapping.cc and LoopClosing.cc
// compile unchanged.
//
// Errors: the reference has no error path; a failing kernel call throws
// std::runtime_error (no CPU fallback exists).
#include "ORBmatcher.h"

#include <limits.h>
#include <stdint.h>
#include <string.h>

#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>

#include "Thirdparty/DBoW2/DBoW2/FeatureVector.h"
#include "orb_abi.h"

using namespace std;

namespace ORB_SLAM2 {

const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

namespace {

void check(orb_status_t st, const char* what) {
  if (st != ORB_OK) throw std::runtime_error(std::string("ORBmatcher::") + what + ": " + orb_status_string(st));
}

// One matcher handle (stream + device scratch) per host thread: ORBmatcher
// objects are built per call site on the Tracking, LocalMapping and
// LoopClosing threads (src/Tracking.cc:698,913,1026,1381,1579,1621,
// src/LocalMapping.cc:255,576, src/LoopClosing.cc:259,641).
orb_matcher_t* gpu() {
  struct Handle {
    orb_matcher_t* h = nullptr;
    ~Handle() { orb_matcher_destroy(h); }
  };
  thread_local Handle t;
  if (!t.h) {
    const char* dev = getenv("ORB_AMD_DEVICE");
    check(orb_matcher_create(dev ? atoi(dev) : 0, &t.h), "create");
  }
  return t.h;
}

// Frame members ORBmatcher reads (mvKeysUn, mDescriptors, mvuRight, bounds, scales).
orb_frame_t frame_view(const Frame& F) {
  orb_frame_t f;
  f.n = F.N;
  f.keys = reinterpret_cast<const orb_keypoint_t*>(F.mvKeysUn.data());
  f.descriptors = F.mDescriptors.ptr<uint8_t>();
  f.u_right = F.mvuRight.empty() ? nullptr : F.mvuRight.data();
  f.min_x = Frame::mnMinX;
  f.max_x = Frame::mnMaxX;
  f.min_y = Frame::mnMinY;
  f.max_y = Frame::mnMaxY;
  f.n_levels = F.mnScaleLevels;
  f.scale_factors = F.mvScaleFactors.data();
  return f;
}

orb_frame_t keyframe_view(const KeyFrame* K) {
  orb_frame_t f;
  f.n = K->N;
  f.keys = reinterpret_cast<const orb_keypoint_t*>(K->mvKeysUn.data());
  f.descriptors = K->mDescriptors.ptr<uint8_t>();
  f.u_right = K->mvuRight.empty() ? nullptr : K->mvuRight.data();
  f.min_x = (float)K->mnMinX;
  f.max_x = (float)K->mnMaxX;
  f.min_y = (float)K->mnMinY;
  f.max_y = (float)K->mnMaxY;
  f.n_levels = K->mnScaleLevels;
  f.scale_factors = K->mvScaleFactors.data();
  return f;
}

orb_camera_t frame_camera(const Frame& F) {
  return orb_camera_t{Frame::fx, Frame::fy, Frame::cx, Frame::cy, F.mbf, F.mb};
}
orb_camera_t keyframe_camera(const KeyFrame* K) {
  return orb_camera_t{K->fx, K->fy, K->cx, K->cy, K->mbf, K->mb};
}

// Rcw (row-major), tcw and the camera centre Ow = -Rcw^T tcw, with the
// reference's cv::Mat float arithmetic (src/ORBmatcher.cc:1625-1627).
orb_pose_t pose_from_tcw(const cv::Mat& Tcw) {
  const cv::Mat Rcw = Tcw.rowRange(0, 3).colRange(0, 3);
  const cv::Mat tcw = Tcw.rowRange(0, 3).col(3);
  const cv::Mat Ow = -Rcw.t() * tcw;
  orb_pose_t p;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) p.rcw[3 * r + c] = Rcw.at<float>(r, c);
    p.tcw[r] = tcw.at<float>(r);
    p.ow[r] = Ow.at<float>(r);
  }
  return p;
}
orb_pose_t keyframe_pose(KeyFrame* K) {  // Fuse: GetRotation / GetTranslation / GetCameraCenter
  const cv::Mat R = K->GetRotation(), t = K->GetTranslation(), Ow = K->GetCameraCenter();
  orb_pose_t p;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) p.rcw[3 * r + c] = R.at<float>(r, c);
    p.tcw[r] = t.at<float>(r);
    p.ow[r] = Ow.at<float>(r);
  }
  return p;
}
void mat33(const cv::Mat& M, float* out) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) out[3 * r + c] = M.at<float>(r, c);
}
void vec3(const cv::Mat& v, float* out) {
  for (int r = 0; r < 3; ++r) out[r] = v.at<float>(r);
}

// MapPoint::CopyDescriptor (INTEGRATION CHANGE, include/MapPoint.h): the 32
// bytes under mMutexFeatures, as GetDescriptor reads them, without the cv::Mat
// clone (a heap allocation per map point per call: 0.13-0.16 ms of a 5,000-point
// SearchByProjection in the drop-in harness)
void copy_descriptor(MapPoint* pMP, uint8_t* dst) { pMP->CopyDescriptor(dst); }

// DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>, ascending ids) as CSR.
struct CsrFeatureVector {
  std::vector<uint32_t> nodes, feats;
  std::vector<int32_t> offs{0};
  explicit CsrFeatureVector(const DBoW2::FeatureVector& fv) {
    for (DBoW2::FeatureVector::const_iterator it = fv.begin(); it != fv.end(); ++it) {
      nodes.push_back(it->first);
      feats.insert(feats.end(), it->second.begin(), it->second.end());
      offs.push_back((int32_t)feats.size());
    }
  }
  int size() const { return (int)nodes.size(); }
};

}  // namespace

// A MapPoint as the projection kernels read it (GetWorldPos, GetNormal, the
// unscaled distance limits of Get{Min,Max}DistanceInvariance / PredictScale,
// isBad, Observations); `seen` is set per variant.
static orb_map_point_t map_point_record(MapPoint* pMP) {
  orb_map_point_t r;
  memset(&r, 0, sizeof(r));
  if (!pMP) {
    r.bad = 1;
    return r;
  }
  vec3(pMP->GetWorldPos(), r.pos);
  vec3(pMP->GetNormal(), r.normal);
  r.min_distance = pMP->GetMinDistance();
  r.max_distance = pMP->GetMaxDistance();
  r.bad = pMP->isBad() ? 1 : 0;
  r.has_obs = pMP->Observations() > 0 ? 1 : 0;
  return r;
}

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

// src/ORBmatcher.cc:47-133 (Tracking::SearchLocalPoints after the isInFrustum pass)
int ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, const float th) {
  const int N = F.N, M = (int)vpMapPoints.size();
  if (N == 0) return 0;
  // the frame and every map point flattened straight into the handle's pinned
  // input block (orb_match_projection_local_stage: one DMA in, no library-side
  // copy, no per-call heap buffers)
  orb_local_stage_t S;
  check(orb_match_projection_local_stage(gpu(), N, M, &S), "SearchByProjection(F, vpMapPoints) stage");
  memcpy(S.keys, F.mvKeysUn.data(), (size_t)N * sizeof(orb_keypoint_t));
  memcpy(S.descriptors, F.mDescriptors.ptr<uint8_t>(), (size_t)N * 32);
  const bool stereo = !F.mvuRight.empty();
  if (stereo) memcpy(S.u_right, F.mvuRight.data(), (size_t)N * 4);
  for (int i = 0; i < N; ++i)  // a claim by a point with observations locks the keypoint (:90-93)
    S.kp_locked[i] = F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0;
  const orb_frame_t f = frame_view(F);
  // the frame's part goes out and its keypoint grid is built while the map is flattened
  check(orb_match_projection_local_begin(gpu(), &f, stereo ? 1 : 0, 1),
        "SearchByProjection(F, vpMapPoints) begin");
  for (int i = 0; i < M; ++i) {
    MapPoint* p = vpMapPoints[i];
    orb_mp_track_t& t = S.mps[i];
    t.proj_x = p->mTrackProjX;
    t.proj_y = p->mTrackProjY;
    t.proj_xr = p->mTrackProjXR;
    t.view_cos = p->mTrackViewCos;
    t.level = p->mnTrackScaleLevel;
    t.in_view = p->mbTrackInView ? 1 : 0;
    t.bad = p->isBad() ? 1 : 0;
    t.has_obs = p->Observations() > 0 ? 1 : 0;
    t._pad = 0;
    // (a point skipped by :57-61 is never read: its descriptor is not copied)
    if (t.in_view && !t.bad) copy_descriptor(p, S.mp_desc + (size_t)i * 32);
  }
  thread_local vector<int32_t> kpMatch;
  kpMatch.resize(N);
  int32_t nmatches = 0;
  check(orb_match_projection_local_staged(gpu(), &f, M, stereo ? 1 : 0, 1, th, mfNNratio,
                                          kpMatch.data(), &nmatches),
        "SearchByProjection(F, vpMapPoints)");
  for (int i = 0; i < N; ++i)
    if (kpMatch[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[kpMatch[i]];  // :127
  return nmatches;
}

float ORBmatcher::RadiusByViewingCos(const float& viewCos) {  // :135-141
  if (viewCos > 0.998) return 2.5;
  return 4.0;
}

// src/ORBmatcher.cc:144-161 (SearchForTriangulation's filter; the kernel evaluates
// the same expression, this host copy serves callers of the protected member)
bool ORBmatcher::CheckDistEpipolarLine(const cv::KeyPoint& kp1, const cv::KeyPoint& kp2,
                                       const cv::Mat& F12, const KeyFrame* pKF2) {
  const float a = kp1.pt.x * F12.at<float>(0, 0) + kp1.pt.y * F12.at<float>(1, 0) + F12.at<float>(2, 0);
  const float b = kp1.pt.x * F12.at<float>(0, 1) + kp1.pt.y * F12.at<float>(1, 1) + F12.at<float>(2, 1);
  const float c = kp1.pt.x * F12.at<float>(0, 2) + kp1.pt.y * F12.at<float>(1, 2) + F12.at<float>(2, 2);
  const float num = a * kp2.pt.x + b * kp2.pt.y + c;
  const float den = a * a + b * b;
  if (den == 0) return false;
  const float dsqr = num * num / den;
  return dsqr < 3.84 * pKF2->mvLevelSigma2[kp2.octave];
}

// src/ORBmatcher.cc:164-306 (Tracking::TrackReferenceKeyFrame, Relocalization)
int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches) {
  const vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
  vpMapPointMatches = vector<MapPoint*>(F.N, static_cast<MapPoint*>(NULL));
  const int NK = pKF->N;
  vector<int32_t> kfMp(NK);
  vector<uint8_t> kfBad(NK);
  vector<float> kfAngle(NK), fAngle(F.N);
  for (int i = 0; i < NK; ++i) {
    MapPoint* p = vpMapPointsKF[i];
    kfMp[i] = p ? i : -1;
    kfBad[i] = p && p->isBad() ? 1 : 0;
    kfAngle[i] = pKF->mvKeysUn[i].angle;
  }
  for (int j = 0; j < F.N; ++j) fAngle[j] = F.mvKeys[j].angle;  // :258 reads mvKeys
  const CsrFeatureVector a(pKF->mFeatVec), b(F.mFeatVec);
  vector<int32_t> fMatch(F.N);
  int32_t nmatches = 0;
  check(orb_match_bow(gpu(), NK, pKF->mDescriptors.ptr<uint8_t>(), kfAngle.data(), kfMp.data(),
                      kfBad.data(), a.size(), a.nodes.data(), a.offs.data(), a.feats.data(), F.N,
                      F.mDescriptors.ptr<uint8_t>(), fAngle.data(), b.size(), b.nodes.data(),
                      b.offs.data(), b.feats.data(), mfNNratio, mbCheckOrientation ? 1 : 0,
                      fMatch.data(), &nmatches),
        "SearchByBoW(KF, F)");
  for (int j = 0; j < F.N; ++j)
    if (fMatch[j] >= 0) vpMapPointMatches[j] = vpMapPointsKF[fMatch[j]];
  return nmatches;
}

// src/ORBmatcher.cc:311-425 (LoopClosing::ComputeSim3)
int ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints,
                                   vector<MapPoint*>& vpMatched, int th) {
  float scw[12];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) scw[4 * r + c] = Scw.at<float>(r, c);
  set<MapPoint*> spAlreadyFound(vpMatched.begin(), vpMatched.end());
  spAlreadyFound.erase(static_cast<MapPoint*>(NULL));
  const int M = (int)vpPoints.size();
  vector<orb_map_point_t> mps(M);
  vector<uint8_t> mpDesc((size_t)M * 32);
  for (int i = 0; i < M; ++i) {
    mps[i] = map_point_record(vpPoints[i]);
    mps[i].seen = spAlreadyFound.count(vpPoints[i]) ? 1 : 0;
    if (!mps[i].bad) copy_descriptor(vpPoints[i], &mpDesc[(size_t)i * 32]);
  }
  // occupancy in, new claims out: an occupied slot only needs a value >= 0
  const int N = pKF->N;
  vector<int32_t> kp(N);
  for (int j = 0; j < N; ++j) kp[j] = vpMatched[j] ? INT_MAX : -1;
  const orb_frame_t f = keyframe_view(pKF);
  const orb_camera_t cam = keyframe_camera(pKF);
  int32_t nmatches = 0;
  check(orb_search_by_projection_sim3(gpu(), &f, scw, &cam, pKF->mfLogScaleFactor, M, mps.data(),
                                      mpDesc.data(), (float)th, kp.data(), &nmatches),
        "SearchByProjection(KF, Scw)");
  for (int j = 0; j < N; ++j)
    if (!vpMatched[j] && kp[j] >= 0 && kp[j] < M) vpMatched[j] = vpPoints[kp[j]];  // :416-420
  return nmatches;
}

// src/ORBmatcher.cc:429-577 (Tracking::MonocularInitialization)
int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
                                        vector<int>& vnMatches12, int windowSize) {
  const orb_frame_t f1 = frame_view(F1), f2 = frame_view(F2);
  vector<int32_t> m12(F1.mvKeysUn.size(), -1);
  int32_t nmatches = 0;
  // vbPrevMatched: one cv::Point2f (x, y floats) per F1 keypoint, updated in place (:571-574)
  check(orb_search_for_initialization(gpu(), &f1, &f2, reinterpret_cast<float*>(vbPrevMatched.data()),
                                      windowSize, mfNNratio, mbCheckOrientation ? 1 : 0,
                                      m12.data(), &nmatches),
        "SearchForInitialization");
  vnMatches12.assign(m12.begin(), m12.end());
  return nmatches;
}

// src/ORBmatcher.cc:581-716 (LoopClosing::ComputeSim3)
int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12) {
  const vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
  const vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
  const int N1 = (int)vpMapPoints1.size(), N2 = (int)vpMapPoints2.size();
  vpMatches12 = vector<MapPoint*>(N1, static_cast<MapPoint*>(NULL));
  vector<int32_t> mp1(N1), mp2(N2), match12(N1);
  vector<uint8_t> bad1(N1), bad2(N2);
  vector<float> a1(N1), a2(N2);
  for (int i = 0; i < N1; ++i) {
    mp1[i] = vpMapPoints1[i] ? i : -1;
    bad1[i] = vpMapPoints1[i] && vpMapPoints1[i]->isBad() ? 1 : 0;
    a1[i] = pKF1->mvKeysUn[i].angle;
  }
  for (int i = 0; i < N2; ++i) {
    mp2[i] = vpMapPoints2[i] ? i : -1;
    bad2[i] = vpMapPoints2[i] && vpMapPoints2[i]->isBad() ? 1 : 0;
    a2[i] = pKF2->mvKeysUn[i].angle;
  }
  const CsrFeatureVector f1(pKF1->mFeatVec), f2(pKF2->mFeatVec);
  int32_t nmatches = 0;
  check(orb_match_bow_kf(gpu(), N1, pKF1->mDescriptors.ptr<uint8_t>(), a1.data(), mp1.data(),
                         bad1.data(), f1.size(), f1.nodes.data(), f1.offs.data(), f1.feats.data(),
                         N2, pKF2->mDescriptors.ptr<uint8_t>(), a2.data(), mp2.data(), bad2.data(),
                         f2.size(), f2.nodes.data(), f2.offs.data(), f2.feats.data(), mfNNratio,
                         mbCheckOrientation ? 1 : 0, match12.data(), &nmatches),
        "SearchByBoW(KF, KF)");
  for (int i = 0; i < N1; ++i)
    if (match12[i] >= 0) vpMatches12[i] = vpMapPoints2[match12[i]];
  return nmatches;
}

// src/ORBmatcher.cc:718-901 (LocalMapping::CreateNewMapPoints)
int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                                       vector<pair<size_t, size_t> >& vMatchedPairs,
                                       const bool bOnlyStereo) {
  const int N1 = pKF1->N, N2 = pKF2->N;
  vector<uint8_t> has1(N1), has2(N2);
  for (int i = 0; i < N1; ++i) has1[i] = pKF1->GetMapPoint(i) ? 1 : 0;
  for (int i = 0; i < N2; ++i) has2[i] = pKF2->GetMapPoint(i) ? 1 : 0;
  float f12[9], cw[3], r2w[9], t2w[3];
  mat33(F12, f12);
  vec3(pKF1->GetCameraCenter(), cw);
  mat33(pKF2->GetRotation(), r2w);
  vec3(pKF2->GetTranslation(), t2w);
  const orb_frame_t k1 = keyframe_view(pKF1), k2 = keyframe_view(pKF2);
  const orb_camera_t cam = keyframe_camera(pKF2);  // the epipole is projected with pKF2's intrinsics
  const CsrFeatureVector a(pKF1->mFeatVec), b(pKF2->mFeatVec);
  vector<int32_t> match12(N1);
  int32_t n = 0;
  check(orb_search_for_triangulation(gpu(), &k1, has1.data(), &k2, has2.data(),
                                     pKF2->mvLevelSigma2.data(), f12, &cam, cw, r2w, t2w, a.size(),
                                     a.nodes.data(), a.offs.data(), a.feats.data(), b.size(),
                                     b.nodes.data(), b.offs.data(), b.feats.data(),
                                     bOnlyStereo ? 1 : 0, mbCheckOrientation ? 1 : 0,
                                     match12.data(), &n),
        "SearchForTriangulation");
  vMatchedPairs.clear();
  vMatchedPairs.reserve(n);
  for (int i = 0; i < N1; ++i)  // :890-897, ascending i1
    if (match12[i] >= 0) vMatchedPairs.push_back(make_pair((size_t)i, (size_t)match12[i]));
  return n;
}

// src/ORBmatcher.cc:903-1077 (LocalMapping::SearchInNeighbors).  The kernels
// find every point's target keypoint from the entry state; the side effects
// then run in point order against the live state, re-checking what the
// reference re-checks (a point made bad, or put into pKF, by an earlier
// Replace is skipped, and the keypoint's current MapPoint is re-read).
int ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, const float th) {
  const int M = (int)vpMapPoints.size();
  vector<orb_map_point_t> mps(M);
  vector<uint8_t> mpDesc((size_t)M * 32);
  for (int i = 0; i < M; ++i) {
    MapPoint* p = vpMapPoints[i];
    mps[i] = map_point_record(p);
    if (p) mps[i].seen = p->IsInKeyFrame(pKF) ? 1 : 0;
    if (p && !mps[i].bad && !mps[i].seen) copy_descriptor(p, &mpDesc[(size_t)i * 32]);
  }
  const orb_frame_t f = keyframe_view(pKF);
  const orb_pose_t pose = keyframe_pose(pKF);
  const orb_camera_t cam = keyframe_camera(pKF);
  vector<int32_t> fuseIdx(M);
  int32_t nMatched = 0;
  check(orb_fuse(gpu(), &f, pKF->mvInvLevelSigma2.data(), &pose, &cam, pKF->mfLogScaleFactor, M,
                 mps.data(), mpDesc.data(), th, fuseIdx.data(), &nMatched),
        "Fuse");
  int nFused = 0;
  for (int i = 0; i < M; ++i) {
    if (fuseIdx[i] < 0) continue;
    MapPoint* pMP = vpMapPoints[i];
    if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;  // :919-923, live
    const int bestIdx = fuseIdx[i];
    MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);  // :1044-1070
    if (pMPinKF) {
      if (!pMPinKF->isBad()) {
        if (pMPinKF->Observations() > pMP->Observations())
          pMP->Replace(pMPinKF);
        else
          pMPinKF->Replace(pMP);
      }
    } else {
      pMP->AddObservation(pKF, bestIdx);
      pKF->AddMapPoint(pMP, bestIdx);
    }
    nFused++;
  }
  return nFused;
}

// src/ORBmatcher.cc:1079-1210 (LoopClosing::SearchAndFuse)
int ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, float th,
                     vector<MapPoint*>& vpReplacePoint) {
  float scw[12];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) scw[4 * r + c] = Scw.at<float>(r, c);
  const set<MapPoint*> spAlreadyFound = pKF->GetMapPoints();  // :1092, entry copy
  const int M = (int)vpPoints.size();
  vector<orb_map_point_t> mps(M);
  vector<uint8_t> mpDesc((size_t)M * 32);
  for (int i = 0; i < M; ++i) {
    mps[i] = map_point_record(vpPoints[i]);
    mps[i].seen = spAlreadyFound.count(vpPoints[i]) ? 1 : 0;
    if (!mps[i].bad && !mps[i].seen) copy_descriptor(vpPoints[i], &mpDesc[(size_t)i * 32]);
  }
  const orb_frame_t f = keyframe_view(pKF);
  const orb_camera_t cam = keyframe_camera(pKF);
  vector<int32_t> fuseIdx(M);
  int32_t nMatched = 0;
  check(orb_fuse_sim3(gpu(), &f, scw, &cam, pKF->mfLogScaleFactor, M, mps.data(), mpDesc.data(), th,
                      fuseIdx.data(), &nMatched),
        "Fuse(KF, Scw)");
  int nFused = 0;
  for (int i = 0; i < M; ++i) {
    if (fuseIdx[i] < 0) continue;
    MapPoint* pMP = vpPoints[i];
    const int bestIdx = fuseIdx[i];
    MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);  // :1187-1199, live
    if (pMPinKF) {
      if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
    } else {
      pMP->AddObservation(pKF, bestIdx);
      pKF->AddMapPoint(pMP, bestIdx);
    }
    nFused++;
  }
  return nFused;
}

// src/ORBmatcher.cc:1212-1458 (LoopClosing::ComputeSim3)
int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12,
                             const float& s12, const cv::Mat& R12, const cv::Mat& t12,
                             const float th) {
  const vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
  const vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
  const int N1 = (int)vpMapPoints1.size(), N2 = (int)vpMapPoints2.size();
  vector<uint8_t> already1(N1, 0), already2(N2, 0), valid1(N1), valid2(N2);
  for (int i = 0; i < N1; ++i) {  // :1240-1252
    MapPoint* pMP = vpMatches12[i];
    if (pMP) {
      already1[i] = 1;
      const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
      if (idx2 >= 0 && idx2 < N2) already2[idx2] = 1;
    }
  }
  vector<orb_map_point_t> mps1(N1), mps2(N2);
  vector<uint8_t> d1((size_t)N1 * 32), d2((size_t)N2 * 32);
  for (int i = 0; i < N1; ++i) {
    MapPoint* p = vpMapPoints1[i];
    valid1[i] = p ? 1 : 0;
    mps1[i] = map_point_record(p);
    if (p && !mps1[i].bad) copy_descriptor(p, &d1[(size_t)i * 32]);
  }
  for (int i = 0; i < N2; ++i) {
    MapPoint* p = vpMapPoints2[i];
    valid2[i] = p ? 1 : 0;
    mps2[i] = map_point_record(p);
    if (p && !mps2[i].bad) copy_descriptor(p, &d2[(size_t)i * 32]);
  }
  float r1w[9], t1w[3], r2w[9], t2w[3], r12[9], tt12[3];
  mat33(pKF1->GetRotation(), r1w);
  vec3(pKF1->GetTranslation(), t1w);
  mat33(pKF2->GetRotation(), r2w);
  vec3(pKF2->GetTranslation(), t2w);
  mat33(R12, r12);
  vec3(t12, tt12);
  const orb_frame_t k1 = keyframe_view(pKF1), k2 = keyframe_view(pKF2);
  const orb_camera_t cam = keyframe_camera(pKF1);  // :1215-1218
  vector<int32_t> match12(N1);
  int32_t nFound = 0;
  check(orb_search_by_sim3(gpu(), &k1, &k2, pKF1->mfLogScaleFactor, &cam, r1w, t1w, r2w, t2w,
                           mps1.data(), valid1.data(), already1.data(), d1.data(), mps2.data(),
                           valid2.data(), already2.data(), d2.data(), s12, r12, tt12, th,
                           match12.data(), &nFound),
        "SearchBySim3");
  for (int i = 0; i < N1; ++i)
    if (match12[i] >= 0) vpMatches12[i] = vpMapPoints2[match12[i]];  // :1450-1453
  return nFound;
}

// src/ORBmatcher.cc:1460-1619 (Tracking::TrackWithMotionModel)
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th,
                                   const bool bMono) {
  const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);  // :1472-1480
  const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
  const cv::Mat twc = -Rcw.t() * tcw;
  const cv::Mat Rlw = LastFrame.mTcw.rowRange(0, 3).colRange(0, 3);
  const cv::Mat tlw = LastFrame.mTcw.rowRange(0, 3).col(3);
  const cv::Mat tlc = Rlw * twc + tlw;
  const int NL = LastFrame.N, N = CurrentFrame.N;
  vector<orb_last_mp_t> last(NL);
  vector<uint8_t> lastDesc((size_t)NL * 32);
  unordered_map<MapPoint*, int32_t> id;  // a MapPoint's id = its first index in LastFrame
  for (int i = 0; i < NL; ++i) {
    MapPoint* pMP = LastFrame.mvpMapPoints[i];
    orb_last_mp_t& r = last[i];
    memset(&r, 0, sizeof(r));
    r.mp_id = -1;
    if (!pMP || LastFrame.mvbOutlier[i]) continue;
    const cv::Mat x3Dw = pMP->GetWorldPos();  // :1500-1505
    const cv::Mat x3Dc = Rcw * x3Dw + tcw;
    r.xc = x3Dc.at<float>(0);
    r.yc = x3Dc.at<float>(1);
    r.invzc = 1.0 / x3Dc.at<float>(2);
    r.last_octave = LastFrame.mvKeys[i].octave;
    r.last_angle = LastFrame.mvKeysUn[i].angle;
    r.valid = 1;
    r.has_obs = pMP->Observations() > 0 ? 1 : 0;
    r.mp_id = id.emplace(pMP, i).first->second;
    copy_descriptor(pMP, &lastDesc[(size_t)i * 32]);
  }
  vector<uint8_t> locked(N);
  for (int j = 0; j < N; ++j)
    locked[j] = CurrentFrame.mvpMapPoints[j] && CurrentFrame.mvpMapPoints[j]->Observations() > 0;
  const orb_frame_t f = frame_view(CurrentFrame);
  const orb_camera_t cam = frame_camera(CurrentFrame);
  vector<int32_t> kpMatch(N);
  int32_t nmatches = 0;
  check(orb_match_projection_frame(gpu(), &f, locked.data(), NL, last.data(), lastDesc.data(), &cam,
                                   tlc.at<float>(2), th, bMono ? 1 : 0, mbCheckOrientation ? 1 : 0,
                                   kpMatch.data(), &nmatches),
        "SearchByProjection(F, LastFrame)");
  for (int j = 0; j < N; ++j) {
    if (kpMatch[j] >= 0) CurrentFrame.mvpMapPoints[j] = LastFrame.mvpMapPoints[kpMatch[j]];  // :1576
    else if (kpMatch[j] == -2) CurrentFrame.mvpMapPoints[j] = static_cast<MapPoint*>(NULL);  // :1611
  }
  return nmatches;
}

// src/ORBmatcher.cc:1622-1759 (Tracking::Relocalization)
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF,
                                   const set<MapPoint*>& sAlreadyFound, const float th,
                                   const int ORBdist) {
  const vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
  const int M = (int)vpMPs.size(), N = CurrentFrame.N;
  vector<orb_map_point_t> mps(M);
  vector<uint8_t> mpDesc((size_t)M * 32);
  vector<float> kfAngle(M);
  for (int i = 0; i < M; ++i) {
    MapPoint* p = vpMPs[i];
    mps[i] = map_point_record(p);
    if (p) mps[i].seen = sAlreadyFound.count(p) ? 1 : 0;
    if (p && !mps[i].bad && !mps[i].seen) copy_descriptor(p, &mpDesc[(size_t)i * 32]);
    kfAngle[i] = pKF->mvKeysUn[i].angle;
  }
  vector<uint8_t> locked(N);
  for (int j = 0; j < N; ++j) locked[j] = CurrentFrame.mvpMapPoints[j] ? 1 : 0;  // :1683-1684
  const orb_frame_t f = frame_view(CurrentFrame);
  const orb_pose_t pose = pose_from_tcw(CurrentFrame.mTcw);
  const orb_camera_t cam = frame_camera(CurrentFrame);
  vector<int32_t> kpMatch(N);
  int32_t nmatches = 0;
  check(orb_search_by_projection_reloc(gpu(), &f, locked.data(), &pose, &cam,
                                       CurrentFrame.mfLogScaleFactor, M, mps.data(), mpDesc.data(),
                                       kfAngle.data(), th, ORBdist, mbCheckOrientation ? 1 : 0,
                                       kpMatch.data(), &nmatches),
        "SearchByProjection(F, KF, sAlreadyFound)");
  for (int j = 0; j < N; ++j) {
    if (kpMatch[j] >= 0) CurrentFrame.mvpMapPoints[j] = vpMPs[kpMatch[j]];  // :1703
    else if (kpMatch[j] == -2) CurrentFrame.mvpMapPoints[j] = NULL;      // :1750
  }
  return nmatches;
}

// src/ORBmatcher.cc:1765-1809 (the kernels apply it; host copy for the protected member)
void ORBmatcher::ComputeThreeMaxima(vector<int>* histo, const int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = histo[i].size();
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}

// src/ORBmatcher.cc:1814-1830: popcount of the XOR of the two 256-bit rows
int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return orb_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

}  // namespace ORB_SLAM2
