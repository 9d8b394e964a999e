// orb_slam2_decls.h -- TEST FIXTURE (tests/test_integration_compile.py only).
//
// Declarations a compiler needs to syntax-check integration/*.cc: a minimal
// cv:: surface (the OpenCV 3 members the drop-ins call, declared, never
// defined), DBoW2::FeatureVector, and the ORB_SLAM2 classes with only the
// members the drop-ins touch.  Nothing here is built or linked, and no
// reference source is compiled against it.  test_integration_compile.py checks
// that every ORB_SLAM2 declaration below also appears (whitespace- and
// std::-normalised) in the reference headers, and that ORBmatcher's and
// ORBextractor's public/protected methods are exactly the reference's, so the
// drop-ins compile against the unchanged reference headers plus the two
// documented additions (marked INTEGRATION CHANGE).
//
// With ORB_RUN_HARNESS defined (tests/integration_run/harness.cc only) the
// classes also carry the storage and test constructors of the runnable
// harness; those #ifdef blocks are not part of the checked declarations.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <list>
#include <map>
#ifdef ORB_RUN_HARNESS
#include <memory>
#endif
#include <mutex>
#include <set>
#include <utility>
#include <vector>

using namespace std;

// ------------------------------------------------------------------- cv
namespace cv {
enum { CV_8U_ = 0 };
struct Point2f { float x, y; };
struct Point { int x, y; };
typedef Point Point2i;
struct KeyPoint {
  Point2f pt;
  float size, angle, response;
  int octave, class_id;
};
class _OutputArray;
typedef const _OutputArray& OutputArray;
class Mat {
 public:
  Mat();
  Mat(int rows, int cols, int type);
  Mat(int rows, int cols, int type, void* data, size_t step);  // external data, not owned
  int rows, cols;
  size_t step;
  unsigned char* data;
  template <typename T> T* ptr(int row = 0);
  template <typename T> const T* ptr(int row = 0) const;
  template <typename T> T& at(int r, int c);
  template <typename T> const T& at(int r, int c) const;
  template <typename T> T& at(int i);
  template <typename T> const T& at(int i) const;
  Mat rowRange(int a, int b) const;
  Mat colRange(int a, int b) const;
  Mat row(int r) const;
  Mat col(int c) const;
  Mat t() const;
  Mat clone() const;
  void create(int rows, int cols, int type);
  void copyTo(OutputArray dst) const;
  bool empty() const;
  int type() const;
  double dot(const Mat& m) const;
#ifdef ORB_RUN_HARNESS
  std::shared_ptr<unsigned char> mem;  // owner of data
  int typ = 0;                         // CV_8U or CV_32F
#endif
};
Mat operator*(const Mat& a, const Mat& b);
Mat operator+(const Mat& a, const Mat& b);
Mat operator-(const Mat& a);
Mat operator/(const Mat& a, double s);
class _InputArray {
 public:
  _InputArray(const Mat& m);
  Mat getMat() const;
  bool empty() const;
#ifdef ORB_RUN_HARNESS
  const Mat* m = nullptr;
#endif
};
class _OutputArray {
 public:
  _OutputArray(Mat& m);
  void release() const;
#ifdef ORB_RUN_HARNESS
  Mat* m = nullptr;
#endif
};
typedef const _InputArray& InputArray;
}  // namespace cv
#define CV_8U 0
#define CV_8UC1 0

// ------------------------------------------------------------ DBoW2
namespace DBoW2 {
typedef unsigned int NodeId;
class FeatureVector : public std::map<NodeId, std::vector<unsigned int> > {};
class BowVector : public std::map<unsigned int, double> {};
}  // namespace DBoW2

// -------------------------------------------------------- ORB_SLAM2
struct orb_extractor;  // include/orb_abi.h

namespace ORB_SLAM2 {
class MapPoint;
class KeyFrame;
class Frame;

class ORBextractor {
 public:
  enum {HARRIS_SCORE=0, FAST_SCORE=1 };
  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
  ~ORBextractor();  // INTEGRATION CHANGE: destroys mpGpu
  void operator()( cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints, cv::OutputArray descriptors);
  std::vector<cv::Mat> mvImagePyramid;
  orb_extractor* gpu() const { return mpGpu; }  // INTEGRATION CHANGE
 protected:
  void ComputePyramid(cv::Mat image);
  std::vector<cv::Point> pattern;
  int nfeatures;
  double scaleFactor;
  int nlevels;
  int iniThFAST;
  int minThFAST;
  std::vector<int> mnFeaturesPerLevel;
  std::vector<int> umax;
  std::vector<float> mvScaleFactor;
  std::vector<float> mvInvScaleFactor;
  std::vector<float> mvLevelSigma2;
  std::vector<float> mvInvLevelSigma2;
  orb_extractor* mpGpu = nullptr;  // INTEGRATION CHANGE
};

class Frame {
 public:
  static float fx;
  static float fy;
  static float cx;
  static float cy;
  float mbf;
  float mb;
  int N;
  std::vector<cv::KeyPoint> mvKeys, mvKeysRight;
  std::vector<cv::KeyPoint> mvKeysUn;
  std::vector<float> mvuRight;
  std::vector<float> mvDepth;
  DBoW2::FeatureVector mFeatVec;
  cv::Mat mDescriptors, mDescriptorsRight;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<bool> mvbOutlier;
  cv::Mat mTcw;
  int mnScaleLevels;
  float mfLogScaleFactor;
  vector<float> mvScaleFactors;
  static float mnMinX;
  static float mnMaxX;
  static float mnMinY;
  static float mnMaxY;
  ORBextractor* mpORBextractorLeft, *mpORBextractorRight;
  void ComputeStereoMatches();
};

class KeyFrame {
 public:
  cv::Mat GetCameraCenter();
  cv::Mat GetRotation();
  cv::Mat GetTranslation();
  void AddMapPoint(MapPoint* pMP, const size_t &idx);
  std::set<MapPoint*> GetMapPoints();
  std::vector<MapPoint*> GetMapPointMatches();
  MapPoint* GetMapPoint(const size_t &idx);
  const float fx, fy, cx, cy, invfx, invfy, mbf, mb, mThDepth;
  const int N;
  const std::vector<cv::KeyPoint> mvKeysUn;
  const std::vector<float> mvuRight;
  const cv::Mat mDescriptors;
  DBoW2::FeatureVector mFeatVec;
  const int mnScaleLevels;
  const float mfLogScaleFactor;
  const std::vector<float> mvScaleFactors;
  const std::vector<float> mvLevelSigma2;
  const std::vector<float> mvInvLevelSigma2;
  const int mnMinX;
  const int mnMinY;
  const int mnMaxX;
  const int mnMaxY;
#ifdef ORB_RUN_HARNESS
  KeyFrame(const Frame& F, const cv::Mat& Rcw, const cv::Mat& tcw, const cv::Mat& Ow,
           const std::vector<float>& levelSigma2, const std::vector<float>& invLevelSigma2);
  cv::Mat Rcw_, tcw_, Ow_;
  std::vector<MapPoint*> mvpMapPoints_;
  void ReplaceMapPointMatch(size_t idx, MapPoint* pMP);
  void EraseMapPointMatch(size_t idx);
#endif
};

class MapPoint {
 public:
  cv::Mat GetWorldPos();
  cv::Mat GetNormal();
  int Observations();
  void AddObservation(KeyFrame* pKF,size_t idx);
  int GetIndexInKeyFrame(KeyFrame* pKF);
  bool IsInKeyFrame(KeyFrame* pKF);
  bool isBad();
  void Replace(MapPoint* pMP);
  cv::Mat GetDescriptor();
  float mTrackProjX;
  float mTrackProjY;
  float mTrackProjXR;
  bool mbTrackInView;
  int mnTrackScaleLevel;
  float mTrackViewCos;
  float GetMinDistance();  // INTEGRATION CHANGE (include/MapPoint.h): mfMinDistance under mMutexPos
  float GetMaxDistance();  // INTEGRATION CHANGE (include/MapPoint.h): mfMaxDistance under mMutexPos
  void CopyDescriptor(unsigned char* dst);  // INTEGRATION CHANGE (include/MapPoint.h): mDescriptor's 32 bytes under mMutexFeatures
 protected:
  float mfMinDistance;
  float mfMaxDistance;
  std::mutex mMutexPos;
#ifdef ORB_RUN_HARNESS
 public:
  MapPoint(const float* pos, const float* normal, float minDist, float maxDist,
           const unsigned char* desc, int extraObservations, bool bad);
  cv::Mat pos_, normal_, desc_;
  std::map<KeyFrame*, size_t> obs_;
  int extraObs_ = 0;  // observations by keyframes outside the scenario
  bool bad_ = false;
  int id_ = -1;       // scenario id (harness output)
#endif
};

class ORBmatcher {
 public:
  ORBmatcher(float nnratio=0.6, bool checkOri=true);
  static int DescriptorDistance(const cv::Mat &a, const cv::Mat &b);
  int SearchByProjection(Frame &F, const std::vector<MapPoint*> &vpMapPoints, const float th=3);
  int SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, const float th, const bool bMono);
  int SearchByProjection(Frame &CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*> &sAlreadyFound, const float th, const int ORBdist);
  int SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*> &vpPoints, std::vector<MapPoint*> &vpMatched, int th);
  int SearchByBoW(KeyFrame *pKF, Frame &F, std::vector<MapPoint*> &vpMapPointMatches);
  int SearchByBoW(KeyFrame *pKF1, KeyFrame* pKF2, std::vector<MapPoint*> &vpMatches12);
  int SearchForInitialization(Frame &F1, Frame &F2, std::vector<cv::Point2f> &vbPrevMatched, std::vector<int> &vnMatches12, int windowSize=10);
  int SearchForTriangulation(KeyFrame *pKF1, KeyFrame* pKF2, cv::Mat F12, std::vector<pair<size_t, size_t> > &vMatchedPairs, const bool bOnlyStereo);
  int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint *> &vpMatches12, const float &s12, const cv::Mat &R12, const cv::Mat &t12, const float th);
  int Fuse(KeyFrame* pKF, const vector<MapPoint *> &vpMapPoints, const float th=3.0);
  int Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*> &vpPoints, float th, vector<MapPoint *> &vpReplacePoint);
 public:
  static const int TH_LOW;
  static const int TH_HIGH;
  static const int HISTO_LENGTH;
 protected:
  bool CheckDistEpipolarLine(const cv::KeyPoint &kp1, const cv::KeyPoint &kp2, const cv::Mat &F12, const KeyFrame *pKF);
  float RadiusByViewingCos(const float &viewCos);
  void ComputeThreeMaxima(std::vector<int>* histo, const int L, int &ind1, int &ind2, int &ind3);
  float mfNNratio;
  bool mbCheckOrientation;
};
}  // namespace ORB_SLAM2
