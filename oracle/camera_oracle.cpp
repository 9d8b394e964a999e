// camera_oracle.cpp -- CPU ORACLE for keypoint undistortion.  TEST
// INFRASTRUCTURE ONLY: linked into liborb_oracle.so, loaded by tests/ only.
//
// Frame::UndistortKeyPoints (src/Frame.cc:452-482) and Frame::ComputeImageBounds
// (src/Frame.cc:484-514) call cv::undistortPoints(mat, mat, mK, mDistCoef,
// cv::Mat(), mK).  OpenCV is a third-party dependency absent from the
// reference tree (version not pinned: OpenCV 2.4.3+ / 3.x, CMakeLists.txt:31-37);
// this restates cvUndistortPoints (modules/imgproc/src/undistort.cpp) as it
// reads in 2.4.x and 3.x, which agree here:
//   * cvConvert of the CV_32F camera matrix and coefficients to double;
//     fx = A[0][0], fy = A[1][1], cx = A[0][2], cy = A[1][2], ifx = 1./fx;
//   * x = (x - cx)*ifx, y = (y - cy)*ify; then 5 iterations of
//       r2 = x*x + y*y
//       icdist = (1 + ((k7*r2 + k6)*r2 + k5)*r2)/(1 + ((k4*r2 + k1)*r2 + k0)*r2)
//       deltaX = 2*k2*x*y + k3*(r2 + 2*x*x) + k8*r2 + k9*r2*r2
//       deltaY = k2*(r2 + 2*y*y) + 2*k3*x*y + k10*r2 + k11*r2*r2
//       x = (x0 - deltaX)*icdist, y = (y0 - deltaY)*icdist
//     (2.4.x has no k5..k11 terms: they are zero for ORB-SLAM2's 4/5
//     coefficients and add exact zeros; 3.x's identity tilt matrix and
//     criteria COUNT 5 change nothing);
//   * RR = P * R = mK * I; xx = RR00*x + RR01*y + RR02, ww = 1./(RR20*x + RR21*y + RR22);
//     dst = (float)(xx*ww), (float)(yy*ww).
// PARITY STATUS: unpinned against OpenCV itself (not installable here);
// cross-checked against the pure-Python restatement in tests/pyref.py.
#include <stdint.h>
#include <string.h>

#include <algorithm>

namespace {

struct Cam {
  double fx, fy, cx, cy, ifx, ify, rr[9], k[12];
};

bool make_cam(const float* K, const float* dist, int n_dist, Cam& c) {
  if (!(n_dist == 4 || n_dist == 5 || n_dist == 8 || n_dist == 12)) return false;
  memset(&c, 0, sizeof(c));
  double A[9];
  for (int i = 0; i < 9; ++i) A[i] = (double)K[i];
  c.fx = A[0]; c.fy = A[4]; c.cx = A[2]; c.cy = A[5];
  c.ifx = 1. / c.fx;
  c.ify = 1. / c.fy;
  // cvMatMul(&_PP, &_RR, &_RR) with RR = I: every entry is PP[i][j] exactly
  for (int i = 0; i < 9; ++i) c.rr[i] = A[i];
  for (int i = 0; i < n_dist; ++i) c.k[i] = (double)dist[i];
  return true;
}

void undistort(const Cam& c, float u, float v, float& ou, float& ov) {
  const double* k = c.k;
  double x = u, y = v;
  x = (x - c.cx) * c.ifx;
  y = (y - c.cy) * c.ify;
  double x0 = x, y0 = y;
  for (int j = 0; j < 5; j++) {
    double r2 = x * x + y * y;
    double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                    (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
    double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
    double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
    x = (x0 - deltaX) * icdist;
    y = (y0 - deltaY) * icdist;
  }
  const double* RR = c.rr;
  double xx = RR[0] * x + RR[1] * y + RR[2];
  double yy = RR[3] * x + RR[4] * y + RR[5];
  double ww = 1. / (RR[6] * x + RR[7] * y + RR[8]);
  ou = (float)(xx * ww);
  ov = (float)(yy * ww);
}

struct Key {  // cv::KeyPoint / orb_keypoint_t (28 bytes)
  float x, y, size, angle, response;
  int32_t octave, class_id;
};

}  // namespace

extern "C" {

// cv::undistortPoints on n (x, y) float pairs.  Returns 0, or -1 for an
// unsupported coefficient count.
int oracle_undistort_points(int n, const float* xy, const float* K, const float* dist, int n_dist,
                            float* out) {
  Cam c;
  if (!make_cam(K, dist, n_dist, c)) return -1;
  for (int i = 0; i < n; ++i) undistort(c, xy[2 * i], xy[2 * i + 1], out[2 * i], out[2 * i + 1]);
  return 0;
}

// Frame::UndistortKeyPoints (src/Frame.cc:452-482).
int oracle_undistort_keypoints(int n, const void* keys, const float* K, const float* dist,
                               int n_dist, void* keys_un) {
  Cam c;
  if (!make_cam(K, dist, n_dist, c)) return -1;
  const Key* in = (const Key*)keys;
  Key* out = (Key*)keys_un;
  if (dist[0] == 0.0f) {
    memmove(out, in, (size_t)n * sizeof(Key));
    return 0;
  }
  for (int i = 0; i < n; ++i) {
    Key kp = in[i];
    undistort(c, in[i].x, in[i].y, kp.x, kp.y);
    out[i] = kp;
  }
  return 0;
}

// Frame::ComputeImageBounds (src/Frame.cc:484-514): {mnMinX, mnMaxX, mnMinY, mnMaxY}.
int oracle_compute_image_bounds(int cols, int rows, const float* K, const float* dist, int n_dist,
                                float* b) {
  Cam c;
  if (!make_cam(K, dist, n_dist, c)) return -1;
  if (dist[0] != 0.0f) {
    const float m[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
    float u[8];
    for (int i = 0; i < 4; ++i) undistort(c, m[2 * i], m[2 * i + 1], u[2 * i], u[2 * i + 1]);
    b[0] = std::min(u[0], u[4]);
    b[1] = std::max(u[2], u[6]);
    b[2] = std::min(u[1], u[3]);
    b[3] = std::max(u[5], u[7]);
  } else {
    b[0] = 0.0f;
    b[1] = (float)cols;
    b[2] = 0.0f;
    b[3] = (float)rows;
  }
  return 0;
}

}  // extern "C"
