// harness.cc -- TEST HARNESS (tests/test_gpu_dropin.py; built by
// tests/integration_run/Makefile, never part of the product).
//
// Runs the reference-typed drop-ins (integration/ORBextractor.cc,
// ORBmatcher.cc, FrameStereo.cc) as ORB-SLAM2 would call them, on the GPU
// through lib/liborb_amd.so.  OpenCV and the ORB-SLAM2 classes are absent
// from this image, so this file gives the declarations of
// tests/integration_stub/orb_slam2_decls.h minimal definitions of its own:
// a reference-counted cv::Mat (CV_8U / CV_32F, row/column views, the float
// products the drop-ins form), and Frame / KeyFrame / MapPoint holding just
// the state the drop-ins read and write.  MapPoint::Replace moves a point's
// observations and keyframe slots to the other point and marks it bad, as the
// reference's MapPoint::Replace does to the state the matcher later reads;
// descriptor recomputation and covisibility updates are left out (nothing
// in a Fuse loop reads them for a point processed later: DESIGN.md §1).
//
// Scenarios read raw little-endian arrays written by the Python test from a
// directory and write their results back there:
//   harness extract DIR   ORBextractor::operator() + mvImagePyramid + empty image
//   harness stereo  DIR   two extractors + Frame::ComputeStereoMatches (GPU drop-in)
//   harness local   DIR   SearchByProjection(F, vpMapPoints, th): F.mvpMapPoints
//   harness fuse    DIR   Fuse(pKF, vpMapPoints, th) against a sequential loop
//                         over the oracle's targets (Replace / AddObservation order)
//   harness sim3    DIR   SearchBySim3(pKF1, pKF2, vpMatches12, ...)
//   harness time    DIR   per-frame wall times of the drop-ins (bench.py `dropin`)
#include <assert.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <thread>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

#include "Frame.h"
#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "orb_abi.h"

#define CV_32F 5

namespace cv {
static size_t elem(int t) { return t == CV_32F ? 4 : 1; }
Mat::Mat() : rows(0), cols(0), step(0), data(nullptr) {}
Mat::Mat(int r, int c, int t) : Mat() { create(r, c, t); }
Mat::Mat(int r, int c, int t, void* d, size_t st) : rows(r), cols(c), step(st), data((unsigned char*)d) {
  typ = t;
}
void Mat::create(int r, int c, int t) {
  if (data && rows == r && cols == c && typ == t) return;
  rows = r;
  cols = c;
  typ = t;
  step = (size_t)c * elem(t);
  mem.reset(new unsigned char[std::max<size_t>(step * r, 1)](), std::default_delete<unsigned char[]>());
  data = mem.get();
}
template <typename T> T* Mat::ptr(int r) { return reinterpret_cast<T*>(data + (size_t)r * step); }
template <typename T> const T* Mat::ptr(int r) const {
  return reinterpret_cast<const T*>(data + (size_t)r * step);
}
template <typename T> T& Mat::at(int r, int c) { return ptr<T>(r)[c]; }
template <typename T> const T& Mat::at(int r, int c) const { return ptr<T>(r)[c]; }
template <typename T> T& Mat::at(int i) { return cols == 1 ? at<T>(i, 0) : at<T>(0, i); }
template <typename T> const T& Mat::at(int i) const { return cols == 1 ? at<T>(i, 0) : at<T>(0, i); }
template unsigned char* Mat::ptr<unsigned char>(int);
template const unsigned char* Mat::ptr<unsigned char>(int) const;
template float& Mat::at<float>(int, int);
template const float& Mat::at<float>(int, int) const;
template float& Mat::at<float>(int);
template const float& Mat::at<float>(int) const;
Mat Mat::rowRange(int a, int b) const {
  Mat m(*this);
  m.rows = b - a;
  m.data = data + (size_t)a * step;
  return m;
}
Mat Mat::colRange(int a, int b) const {
  Mat m(*this);
  m.cols = b - a;
  m.data = data + (size_t)a * elem(typ);
  return m;
}
Mat Mat::row(int r) const { return rowRange(r, r + 1); }
Mat Mat::col(int c) const { return colRange(c, c + 1); }
Mat Mat::clone() const {
  Mat m(rows, cols, typ);
  for (int r = 0; r < rows; ++r) memcpy(m.data + r * m.step, data + r * step, m.step);
  return m;
}
Mat Mat::t() const {  // float matrices only (poses, vectors)
  Mat m(cols, rows, typ);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) m.at<float>(c, r) = at<float>(r, c);
  return m;
}
void Mat::copyTo(OutputArray dst) const {
  Mat& d = *dst.m;
  d.create(rows, cols, typ);
  for (int r = 0; r < rows; ++r) memcpy(d.data + r * d.step, data + r * step, (size_t)cols * elem(typ));
}
bool Mat::empty() const { return !data || rows * cols == 0; }
int Mat::type() const { return typ; }
double Mat::dot(const Mat& o) const {
  double s = 0;
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) s += (double)at<float>(r, c) * o.at<float>(r, c);
  return s;
}
// Float products accumulate in float, left to right (the oracle's pinning of
// the reference's small cv::Mat expressions; OpenCV's gemm may differ).
Mat operator*(const Mat& a, const Mat& b) {
  Mat m(a.rows, b.cols, CV_32F);
  for (int i = 0; i < a.rows; ++i)
    for (int j = 0; j < b.cols; ++j) {
      float s = 0.f;
      for (int k = 0; k < a.cols; ++k) s += a.at<float>(i, k) * b.at<float>(k, j);
      m.at<float>(i, j) = s;
    }
  return m;
}
Mat operator+(const Mat& a, const Mat& b) {
  Mat m(a.rows, a.cols, CV_32F);
  for (int i = 0; i < a.rows; ++i)
    for (int j = 0; j < a.cols; ++j) m.at<float>(i, j) = a.at<float>(i, j) + b.at<float>(i, j);
  return m;
}
Mat operator-(const Mat& a) {
  Mat m(a.rows, a.cols, CV_32F);
  for (int i = 0; i < a.rows; ++i)
    for (int j = 0; j < a.cols; ++j) m.at<float>(i, j) = -a.at<float>(i, j);
  return m;
}
Mat operator/(const Mat& a, double s) {
  Mat m(a.rows, a.cols, CV_32F);
  for (int i = 0; i < a.rows; ++i)
    for (int j = 0; j < a.cols; ++j) m.at<float>(i, j) = (float)(a.at<float>(i, j) / s);
  return m;
}
_InputArray::_InputArray(const Mat& mm) : m(&mm) {}
Mat _InputArray::getMat() const { return *m; }
bool _InputArray::empty() const { return m->empty(); }
_OutputArray::_OutputArray(Mat& mm) : m(&mm) {}
void _OutputArray::release() const { *m = Mat(); }
}  // namespace cv

namespace ORB_SLAM2 {
ORBextractor::~ORBextractor() { orb_extractor_destroy(mpGpu); }  // INTEGRATION CHANGE

float Frame::fx, Frame::fy, Frame::cx, Frame::cy;
float Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;

KeyFrame::KeyFrame(const Frame& F, const cv::Mat& R, const cv::Mat& t, const cv::Mat& Ow,
                   const std::vector<float>& sigma2, const std::vector<float>& invSigma2)
    : fx(Frame::fx), fy(Frame::fy), cx(Frame::cx), cy(Frame::cy), invfx(1.f / Frame::fx),
      invfy(1.f / Frame::fy), mbf(F.mbf), mb(F.mb), mThDepth(0.f), N(F.N), mvKeysUn(F.mvKeysUn),
      mvuRight(F.mvuRight), mDescriptors(F.mDescriptors.clone()), mnScaleLevels(F.mnScaleLevels),
      mfLogScaleFactor(F.mfLogScaleFactor), mvScaleFactors(F.mvScaleFactors),
      mvLevelSigma2(sigma2), mvInvLevelSigma2(invSigma2), mnMinX((int)Frame::mnMinX),
      mnMinY((int)Frame::mnMinY), mnMaxX((int)Frame::mnMaxX), mnMaxY((int)Frame::mnMaxY),
      Rcw_(R.clone()), tcw_(t.clone()), Ow_(Ow.clone()), mvpMapPoints_(F.N, nullptr) {}
cv::Mat KeyFrame::GetCameraCenter() { return Ow_.clone(); }
cv::Mat KeyFrame::GetRotation() { return Rcw_.clone(); }
cv::Mat KeyFrame::GetTranslation() { return tcw_.clone(); }
void KeyFrame::AddMapPoint(MapPoint* pMP, const size_t& idx) { mvpMapPoints_[idx] = pMP; }
std::set<MapPoint*> KeyFrame::GetMapPoints() {  // the non-NULL, non-bad points
  std::set<MapPoint*> s;
  for (MapPoint* p : mvpMapPoints_)
    if (p && !p->isBad()) s.insert(p);
  return s;
}
std::vector<MapPoint*> KeyFrame::GetMapPointMatches() { return mvpMapPoints_; }
MapPoint* KeyFrame::GetMapPoint(const size_t& idx) { return mvpMapPoints_[idx]; }
void KeyFrame::ReplaceMapPointMatch(size_t idx, MapPoint* p) { mvpMapPoints_[idx] = p; }
void KeyFrame::EraseMapPointMatch(size_t idx) { mvpMapPoints_[idx] = nullptr; }

static cv::Mat vec3(const float* v) {
  cv::Mat m(3, 1, CV_32F);
  for (int i = 0; i < 3; ++i) m.at<float>(i) = v ? v[i] : 0.f;
  return m;
}
MapPoint::MapPoint(const float* pos, const float* normal, float minDist, float maxDist,
                   const unsigned char* desc, int extraObservations, bool bad)
    : mfMinDistance(minDist), mfMaxDistance(maxDist), pos_(vec3(pos)), normal_(vec3(normal)),
      desc_(1, 32, CV_8U), extraObs_(extraObservations), bad_(bad) {
  if (desc) memcpy(desc_.data, desc, 32);
}
cv::Mat MapPoint::GetWorldPos() { return pos_.clone(); }
cv::Mat MapPoint::GetNormal() { return normal_.clone(); }
int MapPoint::Observations() { return (int)obs_.size() + extraObs_; }
void MapPoint::AddObservation(KeyFrame* pKF, size_t idx) { obs_.emplace(pKF, idx); }
int MapPoint::GetIndexInKeyFrame(KeyFrame* pKF) {
  auto it = obs_.find(pKF);
  return it == obs_.end() ? -1 : (int)it->second;
}
bool MapPoint::IsInKeyFrame(KeyFrame* pKF) { return obs_.count(pKF) > 0; }
bool MapPoint::isBad() { return bad_; }
void MapPoint::Replace(MapPoint* pMP) {
  if (pMP == this) return;
  std::map<KeyFrame*, size_t> obs;
  obs.swap(obs_);
  bad_ = true;
  for (auto& o : obs) {
    if (!pMP->IsInKeyFrame(o.first)) {
      o.first->ReplaceMapPointMatch(o.second, pMP);
      pMP->AddObservation(o.first, o.second);
    } else {
      o.first->EraseMapPointMatch(o.second);
    }
  }
  pMP->extraObs_ += extraObs_;
  extraObs_ = 0;
}
cv::Mat MapPoint::GetDescriptor() { return desc_.clone(); }
void MapPoint::CopyDescriptor(unsigned char* dst) { memcpy(dst, desc_.data, 32); }  // INTEGRATION CHANGE
float MapPoint::GetMinDistance() { return mfMinDistance; }
float MapPoint::GetMaxDistance() { return mfMaxDistance; }
}  // namespace ORB_SLAM2

using namespace ORB_SLAM2;

// ------------------------------------------------------------ scenario I/O
static std::string g_dir;
static std::vector<char> rd(const char* name) {
  std::ifstream f(g_dir + "/" + name, std::ios::binary);
  if (!f) {
    fprintf(stderr, "harness: missing %s\n", name);
    exit(2);
  }
  return std::vector<char>(std::istreambuf_iterator<char>(f), {});
}
template <typename T> static std::vector<T> rdv(const char* name) {
  std::vector<char> b = rd(name);
  std::vector<T> v(b.size() / sizeof(T));
  memcpy(v.data(), b.data(), v.size() * sizeof(T));
  return v;
}
static std::vector<double> meta() {
  std::vector<char> b = rd("meta.txt");
  std::istringstream s(std::string(b.begin(), b.end()));
  std::vector<double> v;
  double x;
  while (s >> x) v.push_back(x);
  return v;
}
static void wr(const char* name, const void* p, size_t n) {
  std::ofstream f(g_dir + "/" + name, std::ios::binary);
  f.write(static_cast<const char*>(p), (std::streamsize)n);
}
template <typename T> static void wrv(const char* name, const std::vector<T>& v) {
  wr(name, v.data(), v.size() * sizeof(T));
}
static cv::Mat mat_u8(const std::vector<uint8_t>& v, int rows, int cols) {
  cv::Mat m(rows, cols, CV_8U);
  memcpy(m.data, v.data(), (size_t)rows * cols);
  return m;
}
static cv::Mat mat_f32(const float* v, int rows, int cols) {
  cv::Mat m(rows, cols, CV_32F);
  memcpy(m.data, v, sizeof(float) * rows * cols);
  return m;
}
static std::vector<cv::KeyPoint> keys_of(const std::vector<orb_keypoint_t>& k) {
  std::vector<cv::KeyPoint> out(k.size());
  memcpy(out.data(), k.data(), k.size() * sizeof(orb_keypoint_t));
  return out;
}

// A Frame from keypoints (used as mvKeys and mvKeysUn), descriptors and scales.
static void fill_frame(Frame& F, const char* prefix) {
  const std::string p(prefix);
  auto keys = rdv<orb_keypoint_t>((p + "keys.bin").c_str());
  auto desc = rdv<uint8_t>((p + "desc.bin").c_str());
  auto scale = rdv<float>((p + "scale.bin").c_str());
  F.N = (int)keys.size();
  F.mvKeys = keys_of(keys);
  F.mvKeysUn = F.mvKeys;
  F.mDescriptors = mat_u8(desc, F.N, 32);
  F.mvScaleFactors = scale;
  F.mnScaleLevels = (int)scale.size();
  F.mvpMapPoints.assign(F.N, nullptr);
  F.mvbOutlier.assign(F.N, false);
}

struct MpRec {  // orb_map_point_t
  float pos[3], normal[3], min_distance, max_distance;
  uint8_t bad, seen, has_obs, pad;
};
static_assert(sizeof(MpRec) == 36, "orb_map_point_t");

static int run_extract() {
  const std::vector<double> m = meta();
  const int W = (int)m[0], H = (int)m[1], NF = (int)m[2];
  ORBextractor ext(NF, 1.2f, 8, 20, 7);
  const cv::Mat img = mat_u8(rdv<uint8_t>("img.bin"), H, W);
  std::vector<cv::KeyPoint> kps;
  cv::Mat desc;
  ext(img, cv::Mat(), kps, desc);
  wr("kps.bin", kps.data(), kps.size() * sizeof(cv::KeyPoint));
  std::vector<uint8_t> d((size_t)kps.size() * 32);
  for (int r = 0; r < (int)kps.size(); ++r) memcpy(&d[(size_t)r * 32], desc.ptr<uint8_t>(r), 32);
  wrv("desc.bin", d);
  std::ostringstream sizes;
  for (size_t l = 0; l < ext.mvImagePyramid.size(); ++l) {
    const cv::Mat& L = ext.mvImagePyramid[l];
    std::vector<uint8_t> px((size_t)L.rows * L.cols);
    for (int r = 0; r < L.rows; ++r) memcpy(&px[(size_t)r * L.cols], L.ptr<uint8_t>(r), L.cols);
    wrv(("pyr_" + std::to_string(l) + ".bin").c_str(), px);
    sizes << L.cols << " " << L.rows << "\n";
  }
  const std::string sz = sizes.str();
  wr("pyr_sizes.txt", sz.data(), sz.size());
  // an empty image returns with the outputs untouched (src/ORBextractor.cc:1095-1096)
  std::vector<cv::KeyPoint> k2(3);
  k2[0].pt.x = 7.f;
  cv::Mat d2(2, 32, CV_8U);
  memset(d2.data, 0xAB, 64);
  ext(cv::Mat(), cv::Mat(), k2, d2);
  const bool untouched = k2.size() == 3 && k2[0].pt.x == 7.f && d2.rows == 2 && d2.data[63] == 0xAB;
  wr("empty_ok.txt", untouched ? "1" : "0", 1);
  return 0;
}

static int run_stereo() {
  const std::vector<double> m = meta();
  const int W = (int)m[0], H = (int)m[1], NF = (int)m[2];
  ORBextractor L(NF, 1.2f, 8, 20, 7), R(NF, 1.2f, 8, 20, 7);
  Frame F;
  F.mpORBextractorLeft = &L;
  F.mpORBextractorRight = &R;
  F.mbf = (float)m[3];
  Frame::fx = (float)m[4];
  const cv::Mat il = mat_u8(rdv<uint8_t>("imgL.bin"), H, W), ir = mat_u8(rdv<uint8_t>("imgR.bin"), H, W);
  L(il, cv::Mat(), F.mvKeys, F.mDescriptors);  // src/Frame.cc:81-84 (one thread each there)
  R(ir, cv::Mat(), F.mvKeysRight, F.mDescriptorsRight);
  F.N = (int)F.mvKeys.size();
  F.ComputeStereoMatches();  // integration/FrameStereo.cc
  wrv("ur.bin", F.mvuRight);
  wrv("depth.bin", F.mvDepth);
  return 0;
}

static int run_local() {
  const std::vector<double> m = meta();
  const float th = (float)m[2], nnratio = (float)m[3];
  Frame F;
  fill_frame(F, "");
  Frame::mnMinX = 0.f;
  Frame::mnMaxX = (float)m[0];
  Frame::mnMinY = 0.f;
  Frame::mnMaxY = (float)m[1];
  auto trk = rdv<orb_mp_track_t>("tracks.bin");
  auto mpd = rdv<uint8_t>("mpdesc.bin");
  auto pre = rdv<uint8_t>("pre.bin");  // 0: NULL, 1: a point with observations, 2: one without
  std::vector<MapPoint*> own;
  for (int i = 0; i < F.N; ++i)
    if (pre[i]) {
      own.push_back(new MapPoint(nullptr, nullptr, 0, 0, nullptr, pre[i] == 1 ? 1 : 0, false));
      own.back()->id_ = -2;
      F.mvpMapPoints[i] = own.back();
    }
  std::vector<MapPoint*> vp(trk.size());
  for (size_t i = 0; i < trk.size(); ++i) {
    MapPoint* p = new MapPoint(nullptr, nullptr, 0, 0, &mpd[i * 32], trk[i].has_obs, trk[i].bad);
    p->mTrackProjX = trk[i].proj_x;
    p->mTrackProjY = trk[i].proj_y;
    p->mTrackProjXR = trk[i].proj_xr;
    p->mTrackViewCos = trk[i].view_cos;
    p->mnTrackScaleLevel = trk[i].level;
    p->mbTrackInView = trk[i].in_view != 0;
    p->id_ = (int)i;
    vp[i] = p;
    own.push_back(p);
  }
  ORBmatcher matcher(nnratio, true);
  const int n = matcher.SearchByProjection(F, vp, th);  // Tracking::SearchLocalPoints
  std::vector<int32_t> res(F.N);
  for (int i = 0; i < F.N; ++i) res[i] = F.mvpMapPoints[i] ? F.mvpMapPoints[i]->id_ : -1;
  wrv("res.bin", res);
  wr("count.txt", std::to_string(n).data(), std::to_string(n).size());
  for (MapPoint* p : own) delete p;
  return 0;
}

// A KeyFrame read from files with a prefix: keys, desc, scale, sigma2,
// invsigma2, uright, R, t, ow; camera and bounds from the shared meta.
static KeyFrame* read_keyframe(const std::string& p, const std::vector<double>& m) {
  Frame F;
  fill_frame(F, p.c_str());
  F.mvuRight = rdv<float>((p + "uright.bin").c_str());
  F.mfLogScaleFactor = (float)m[3];
  F.mbf = (float)m[8];
  F.mb = (float)m[9];
  auto R = rdv<float>((p + "R.bin").c_str()), t = rdv<float>((p + "t.bin").c_str()),
       ow = rdv<float>((p + "ow.bin").c_str());
  return new KeyFrame(F, mat_f32(R.data(), 3, 3), mat_f32(t.data(), 3, 1), mat_f32(ow.data(), 3, 1),
                      rdv<float>((p + "sigma2.bin").c_str()),
                      rdv<float>((p + "invsigma2.bin").c_str()));
}
static void set_camera_bounds(const std::vector<double>& m) {
  Frame::mnMinX = 0.f;
  Frame::mnMaxX = (float)m[0];
  Frame::mnMinY = 0.f;
  Frame::mnMaxY = (float)m[1];
  Frame::fx = (float)m[4];
  Frame::fy = (float)m[5];
  Frame::cx = (float)m[6];
  Frame::cy = (float)m[7];
}

// Fuse scenario state: the keyframe, its existing points, the points to fuse.
struct FuseWorld {
  KeyFrame* kf = nullptr;
  std::vector<MapPoint*> existing, points, vp;  // vp: the call's vpMapPoints
  ~FuseWorld() {
    for (MapPoint* p : existing) delete p;
    for (MapPoint* p : points) delete p;
    delete kf;
  }
};
static void build_fuse(FuseWorld& w, const std::vector<double>& m) {
  w.kf = read_keyframe("kf_", m);
  auto ex = rdv<MpRec>("ex_mps.bin");
  auto exd = rdv<uint8_t>("ex_desc.bin");
  auto exo = rdv<int32_t>("ex_obs.bin");    // observations by other keyframes
  auto exs = rdv<int32_t>("ex_slot.bin");   // the keyframe slot of existing point e
  for (size_t e = 0; e < ex.size(); ++e) {
    MapPoint* p = new MapPoint(ex[e].pos, ex[e].normal, ex[e].min_distance, ex[e].max_distance,
                               &exd[e * 32], exo[e], ex[e].bad != 0);
    p->id_ = (int)e;
    p->AddObservation(w.kf, (size_t)exs[e]);
    w.kf->AddMapPoint(p, (size_t)exs[e]);
    w.existing.push_back(p);
  }
  auto mp = rdv<MpRec>("mps.bin");
  auto mpd = rdv<uint8_t>("mpdesc.bin");
  auto mpo = rdv<int32_t>("mp_obs.bin");
  auto ref = rdv<int32_t>("mp_ref.bin");  // -1: a point of its own, e: existing point e, -2: NULL
  for (size_t i = 0; i < mp.size(); ++i) {
    if (ref[i] >= 0) {
      w.vp.push_back(w.existing[ref[i]]);
    } else if (ref[i] == -2) {
      w.vp.push_back(nullptr);
    } else {
      MapPoint* p = new MapPoint(mp[i].pos, mp[i].normal, mp[i].min_distance, mp[i].max_distance,
                                 &mpd[i * 32], mpo[i], mp[i].bad != 0);
      p->id_ = 100000 + (int)i;
      w.points.push_back(p);
      w.vp.push_back(p);
    }
  }
}
// Final state: per keyframe slot the id of its point (-1 NULL); per scenario
// point (existing, then own) its bad flag, observation count and slot index.
static std::vector<int32_t> fuse_state(FuseWorld& w) {
  std::vector<int32_t> s;
  for (MapPoint* p : w.kf->GetMapPointMatches()) s.push_back(p ? p->id_ : -1);
  for (auto* list : {&w.existing, &w.points})
    for (MapPoint* p : *list) {
      s.push_back(p->isBad());
      s.push_back(p->Observations());
      s.push_back(p->GetIndexInKeyFrame(w.kf));
    }
  return s;
}

static int run_fuse() {
  const std::vector<double> m = meta();
  set_camera_bounds(m);
  const float th = (float)m[2];
  // the drop-in
  FuseWorld a;
  build_fuse(a, m);
  ORBmatcher matcher;
  const int n = matcher.Fuse(a.kf, a.vp, th);
  // the reference's loop (src/ORBmatcher.cc:903-1077) on a second copy, with
  // the oracle's entry-state target per point: skip NULL / bad / in-KF points
  // as they stand when the loop reaches them, then Replace or AddObservation
  FuseWorld b;
  build_fuse(b, m);
  auto best = rdv<int32_t>("oracle_best.bin");
  int nref = 0;
  for (size_t i = 0; i < b.vp.size(); ++i) {
    MapPoint* pMP = b.vp[i];
    if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(b.kf)) continue;  // :916-923
    if (best[i] < 0) continue;                                       // :1042 bestDist > TH_LOW
    MapPoint* pMPinKF = b.kf->GetMapPoint((size_t)best[i]);          // :1044-1070
    if (pMPinKF) {
      if (!pMPinKF->isBad()) {
        if (pMPinKF->Observations() > pMP->Observations())
          pMP->Replace(pMPinKF);
        else
          pMPinKF->Replace(pMP);
      }
    } else {
      pMP->AddObservation(b.kf, (size_t)best[i]);
      b.kf->AddMapPoint(pMP, (size_t)best[i]);
    }
    nref++;
  }
  wrv("state_dropin.bin", fuse_state(a));
  wrv("state_ref.bin", fuse_state(b));
  const std::string c = std::to_string(n) + " " + std::to_string(nref);
  wr("count.txt", c.data(), c.size());
  return 0;
}

static int run_sim3() {
  const std::vector<double> m = meta();
  set_camera_bounds(m);
  const float s12 = (float)m[2], th = (float)m[10];
  KeyFrame* k[2] = {read_keyframe("k1_", m), read_keyframe("k2_", m)};
  std::vector<MapPoint*> own;
  for (int j = 0; j < 2; ++j) {
    const std::string p = j ? "k2_" : "k1_";
    auto rec = rdv<MpRec>((p + "mps.bin").c_str());
    auto d = rdv<uint8_t>((p + "mpdesc.bin").c_str());
    auto valid = rdv<uint8_t>((p + "valid.bin").c_str());
    for (size_t i = 0; i < rec.size(); ++i) {
      if (!valid[i]) continue;
      MapPoint* q = new MapPoint(rec[i].pos, rec[i].normal, rec[i].min_distance,
                                 rec[i].max_distance, &d[i * 32], 0, rec[i].bad != 0);
      q->id_ = j ? (int)i : -10;
      q->AddObservation(k[j], i);
      k[j]->AddMapPoint(q, i);
      own.push_back(q);
    }
  }
  // vpMatches12 on entry: -1 NULL, j >= 0 a point observed by pKF2 at j
  // (already matched on both sides), -2 a point pKF2 does not observe
  auto init = rdv<int32_t>("init12.bin");
  std::vector<MapPoint*> vpMatches12(init.size(), nullptr);
  for (size_t i = 0; i < init.size(); ++i) {
    if (init[i] == -1) continue;
    MapPoint* q = new MapPoint(nullptr, nullptr, 0, 0, nullptr, 0, false);
    q->id_ = -3;
    if (init[i] >= 0) q->AddObservation(k[1], (size_t)init[i]);
    own.push_back(q);
    vpMatches12[i] = q;
  }
  auto R12 = rdv<float>("R12.bin"), t12 = rdv<float>("t12.bin");
  ORBmatcher matcher;
  const int n = matcher.SearchBySim3(k[0], k[1], vpMatches12, s12, mat_f32(R12.data(), 3, 3),
                                     mat_f32(t12.data(), 3, 1), th);
  std::vector<int32_t> res(init.size());
  for (size_t i = 0; i < init.size(); ++i) res[i] = vpMatches12[i] ? vpMatches12[i]->id_ : -1;
  wrv("res.bin", res);
  wr("count.txt", std::to_string(n).data(), std::to_string(n).size());
  for (MapPoint* p : own) delete p;
  delete k[0];
  delete k[1];
  return 0;
}


// ------------------------------------------------------------- timing
// harness time DIR: the drop-ins at ORB-SLAM2's own call granularity, one
// frame per call (bench.py's `dropin` key).  Mono: Frame::ExtractORB
// (src/Frame.cc:278-285) through ORBextractor::operator(), then
// Tracking::SearchLocalPoints' SearchByProjection(F, vpMapPoints, th)
// (src/Tracking.cc:1381-1390) over MapPoint objects (the flatten of every point
// -- mutexed getters, GetDescriptor -- included).  Stereo: the two extractions
// on two threads as the stereo Frame constructor runs them (src/Frame.cc:81-84),
// then Frame::ComputeStereoMatches.  Median wall times of ITERS frames.
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}
static int run_time() {
  const std::vector<double> m = meta();
  const int W = (int)m[0], H = (int)m[1], NF = (int)m[2], NMP = (int)m[3], NFR = (int)m[4],
            ITERS = (int)m[5];
  const float bf = (float)m[6], fx = (float)m[7];
  auto imgs = rdv<uint8_t>("imgs.bin"), imgsR = rdv<uint8_t>("imgsR.bin");
  auto trk = rdv<orb_mp_track_t>("tracks.bin");
  auto mpd = rdv<uint8_t>("mpdesc.bin");
  auto scale = rdv<float>("scale.bin");
  Frame::mnMinX = 0.f;
  Frame::mnMaxX = (float)W;
  Frame::mnMinY = 0.f;
  Frame::mnMaxY = (float)H;
  Frame::fx = fx;
  std::vector<cv::Mat> fr(NFR), frR(NFR);
  for (int f = 0; f < NFR; ++f) {
    fr[f] = cv::Mat(H, W, CV_8U);
    frR[f] = cv::Mat(H, W, CV_8U);
    memcpy(fr[f].data, &imgs[(size_t)f * W * H], (size_t)W * H);
    memcpy(frR[f].data, &imgsR[(size_t)f * W * H], (size_t)W * H);
  }
  // each frame's local map as MapPoint objects (built once: the map exists
  // before tracking runs)
  std::vector<std::vector<MapPoint*>> maps(NFR);
  for (int f = 0; f < NFR; ++f)
    for (int i = 0; i < NMP; ++i) {
      const orb_mp_track_t& t = trk[(size_t)f * NMP + i];
      MapPoint* p = new MapPoint(nullptr, nullptr, 0, 0, &mpd[((size_t)f * NMP + i) * 32], t.has_obs,
                                 t.bad);
      p->mTrackProjX = t.proj_x;
      p->mTrackProjY = t.proj_y;
      p->mTrackProjXR = t.proj_xr;
      p->mTrackViewCos = t.view_cos;
      p->mnTrackScaleLevel = t.level;
      p->mbTrackInView = t.in_view != 0;
      p->id_ = i;
      maps[f].push_back(p);
    }
  ORBextractor ext(NF, 1.2f, 8, 20, 7);
  ORBmatcher matcher(0.8f, true);
  std::vector<double> tExt, tMatch, tTot;
  long matches = 0;
  for (int it = -3; it < ITERS; ++it) {
    const int f = (it + 3) % NFR;
    Frame F;
    const double t0 = now_ms();
    ext(fr[f], cv::Mat(), F.mvKeys, F.mDescriptors);
    const double t1 = now_ms();
    F.N = (int)F.mvKeys.size();
    F.mvKeysUn = F.mvKeys;
    F.mvScaleFactors = scale;
    F.mnScaleLevels = (int)scale.size();
    F.mvpMapPoints.assign(F.N, nullptr);
    const int n = matcher.SearchByProjection(F, maps[f], 1.0f);
    const double t2 = now_ms();
    if (it >= 0) {
      tExt.push_back(t1 - t0);
      tMatch.push_back(t2 - t1);
      tTot.push_back(t2 - t0);
      matches += n;
    }
  }
  // the flatten alone (the calls integration/ORBmatcher.cc makes per point
  // before the kernels: track fields, isBad, Observations, CopyDescriptor)
  std::vector<double> tFl;
  {
    std::vector<orb_mp_track_t> trk2(NMP);
    std::vector<uint8_t> dsc(NMP * 32);
    for (int it = 0; it < std::min(ITERS, 100); ++it) {
      const std::vector<MapPoint*>& vp = maps[it % NFR];
      const double t0 = now_ms();
      for (int i = 0; i < NMP; ++i) {
        MapPoint* q = vp[i];
        orb_mp_track_t& t = trk2[i];
        t.proj_x = q->mTrackProjX;
        t.proj_y = q->mTrackProjY;
        t.proj_xr = q->mTrackProjXR;
        t.view_cos = q->mTrackViewCos;
        t.level = q->mnTrackScaleLevel;
        t.in_view = q->mbTrackInView ? 1 : 0;
        t.bad = q->isBad() ? 1 : 0;
        t.has_obs = q->Observations() > 0 ? 1 : 0;
        if (t.in_view && !t.bad) q->CopyDescriptor(&dsc[(size_t)i * 32]);
      }
      tFl.push_back(now_ms() - t0);
    }
  }
  ORBextractor L(2 * NF, 1.2f, 8, 20, 7), R(2 * NF, 1.2f, 8, 20, 7);
  std::vector<double> tSt;
  for (int it = -3; it < ITERS; ++it) {
    const int f = (it + 3) % NFR;
    Frame F;
    F.mpORBextractorLeft = &L;
    F.mpORBextractorRight = &R;
    F.mbf = bf;
    const double t0 = now_ms();
    std::thread tl([&] { L(fr[f], cv::Mat(), F.mvKeys, F.mDescriptors); });
    R(frR[f], cv::Mat(), F.mvKeysRight, F.mDescriptorsRight);
    tl.join();
    F.N = (int)F.mvKeys.size();
    F.ComputeStereoMatches();
    const double t1 = now_ms();
    if (it >= 0) tSt.push_back(t1 - t0);
  }
  char buf[512];
  snprintf(buf, sizeof buf,
           "{\"mono_extract_ms\": %.5f, \"mono_search_by_projection_ms\": %.5f, "
           "\"mono_frame_ms\": %.5f, \"stereo_pair_ms\": %.5f, \"frames\": %d, "
           "\"mean_matches\": %.2f, \"map_flatten_ms\": %.5f}\n",
           median(tExt), median(tMatch), median(tTot), median(tSt), ITERS, (double)matches / ITERS,
           median(tFl));
  wr("time.json", buf, strlen(buf));
  for (auto& v : maps)
    for (MapPoint* p : v) delete p;
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: harness extract|stereo|local|fuse|sim3|time DIR\n");
    return 2;
  }
  g_dir = argv[2];
  const std::string cmd = argv[1];
  try {
    if (cmd == "extract") return run_extract();
    if (cmd == "stereo") return run_stereo();
    if (cmd == "local") return run_local();
    if (cmd == "fuse") return run_fuse();
    if (cmd == "sim3") return run_sim3();
    if (cmd == "time") return run_time();
  } catch (const std::exception& e) {
    fprintf(stderr, "harness: %s\n", e.what());
    return 1;
  }
  fprintf(stderr, "harness: unknown scenario %s\n", cmd.c_str());
  return 2;
}
