// camera_kernels.hip -- gfx950 kernel for keypoint undistortion:
// Frame::UndistortKeyPoints (src/Frame.cc:452-482) and the corner pass of
// Frame::ComputeImageBounds (src/Frame.cc:484-514), both of which call
// cv::undistortPoints(src, dst, mK, mDistCoef, cv::Mat(), mK).
//
// OpenCV's cvUndistortPoints (modules/imgproc/src/undistort.cpp, 2.4.x and
// 3.x; pinned in SURVEY.md Appendix A as "OCV3-scalar"): float points and the
// CV_32F camera matrix / coefficients are widened to double, the distortion
// is inverted by 5 fixed-point iterations, and the result is mapped through
// RR = P * R = mK (R = identity).  Every double operation below is written in
// OpenCV's evaluation order; the library is built with -ffp-contract=off, so
// each product and sum rounds separately as on the CPU.  Thin-prism terms
// (k[8..11]) are kept so 4-, 5-, 8- and 12-coefficient models all take the
// same path (zero terms add exact zeros); the tilted model (14 coefficients)
// is not used by ORB-SLAM2 and is rejected by the host.
//
// One thread per point; a frame's keypoints are 28-byte records, of which the
// kernel rewrites pt.x / pt.y and copies the other five fields.  Double-rate
// VALU on CDNA4 makes this a few hundred nanoseconds per frame: it is a
// latency-bound epilogue, kept separate so it can run after any extractor.
#include "orb_device.h"

struct UndistortParams {
  double fx, fy, cx, cy, ifx, ify;  // A = mK (double), ifx = 1./fx
  double rr[9];                     // RR = mK * I
  double k[12];                     // k1 k2 p1 p2 k3 k4 k5 k6 s1 s2 s3 s4
};

__device__ __forceinline__ void undistort_one(const UndistortParams& P, float u, float v,
                                              float* ox, float* oy) {
  const double* k = P.k;
  double x = (double)u, y = (double)v;
  x = (x - P.cx) * P.ifx;
  y = (y - P.cy) * P.ify;
  const double x0 = x, y0 = y;
  for (int j = 0; j < 5; ++j) {
    const double r2 = x * x + y * y;
    const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                          (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
    const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
    const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
    x = (x0 - deltaX) * icdist;
    y = (y0 - deltaY) * icdist;
  }
  const double* RR = P.rr;
  const double xx = RR[0] * x + RR[1] * y + RR[2];
  const double yy = RR[3] * x + RR[4] * y + RR[5];
  const double ww = 1. / (RR[6] * x + RR[7] * y + RR[8]);
  *ox = (float)(xx * ww);
  *oy = (float)(yy * ww);
}

// Points as (x, y) float pairs: n points, or n_frames x stride keypoint
// records when `keys` is set (counts[f] valid records in frame f).
__global__ __launch_bounds__(256) void k_undistort_points(UndistortParams P, int n,
                                                          const float2* __restrict__ in,
                                                          float2* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float2 p = in[i];
  float2 q;
  undistort_one(P, p.x, p.y, &q.x, &q.y);
  out[i] = q;
}

struct KeyRec {
  float x, y, size, angle, response;
  int32_t octave, class_id;
};

__global__ __launch_bounds__(256) void k_undistort_keys(UndistortParams P, int nFrames,
                                                        const int32_t* __restrict__ counts,
                                                        int nSingle, int stride,
                                                        const KeyRec* __restrict__ in,
                                                        KeyRec* __restrict__ out, int copyOnly) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  const int f = (int)(g / stride), i = (int)(g - (long long)f * stride);
  if (f >= nFrames) return;
  const int n = counts ? counts[f] : nSingle;
  if (i >= n) return;
  KeyRec r = in[g];
  if (!copyOnly) undistort_one(P, r.x, r.y, &r.x, &r.y);  // mDistCoef(0) == 0: mvKeysUn = mvKeys
  out[g] = r;
}

extern "C" hipError_t orb_k_undistort_points(const void* params, int n, const float* in,
                                             float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_undistort_points, dim3((n + 255) / 256), dim3(256), 0, s,
                     *(const UndistortParams*)params, n, (const float2*)in, (float2*)out);
  return hipGetLastError();
}

extern "C" hipError_t orb_k_undistort_keys(const void* params, int nFrames, const int32_t* counts,
                                           int nSingle, int stride, const void* in, void* out,
                                           int copyOnly, hipStream_t s) {
  const long long total = (long long)nFrames * stride;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_undistort_keys, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     *(const UndistortParams*)params, nFrames, counts, nSingle, stride,
                     (const KeyRec*)in, (KeyRec*)out, copyOnly);
  return hipGetLastError();
}

extern "C" size_t orb_k_undistort_params_size() { return sizeof(UndistortParams); }
