// orb_device.h -- device-side helpers shared by the extractor and matcher kernels.
//
// Every float expression here is evaluated exactly as written: the library is
// compiled with -ffp-contract=off and -fhip-fp32-correctly-rounded-divide-sqrt,
// so results are bit-identical to the CPU oracle built with g++ -ffp-contract=off
// (SURVEY.md §7 H4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ORB_MAX_LEVELS 16
#define ORB_WAVE 64

// ---------------------------------------------------------------- rounding
// cvRound = round half to even
__device__ __forceinline__ int cv_round(float v) { return (int)__builtin_rintf(v); }
// std::round / roundf: half away from zero (src/ORBmatcher.cc:254, src/Frame.cc:428)
__device__ __forceinline__ float round_half_away(float v) { return __builtin_roundf(v); }

// -------------------------------------------------- A.4 OpenCV fastAtan2
__device__ __forceinline__ float fast_atan2_deg(float y, float x) {
  const float r2d = (float)(180.0 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d;
  const float p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
  const float eps = (float)2.2204460492503131e-16;
  const float ax = fabsf(x), ay = fabsf(y);
  // both branches of the reference's if / else as selects (the same float
  // operations in the same order; no divergent branch between the two
  // keypoints a wave orients)
  const bool xm = ax >= ay;
  const float c = __fdiv_rn(xm ? ay : ax, (xm ? ax : ay) + eps);
  const float c2 = c * c;
  const float pa = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  float a = xm ? pa : 90.f - pa;
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// ---------------------------------------------- A.6 pinned sin/cos (double)
// fdlibm-style Cody-Waite reduction by pi/2 and degree-13/14 kernels in double,
// rounded once to float.  Same operation sequence as the oracle.
__device__ __forceinline__ void pinned_sincos(float angle, float* s_out, float* c_out) {
  const double x = (double)angle;
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
  const double k = __builtin_rint(x * invpio2);
  const double r = (x - k * pio2_1) - k * pio2_1t;
  const double z = r * r;
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  const double sn = r + (z * r) * (S1 + z * ps);
  const double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cs = w + (((1.0 - w) - hz) + z * pc);
  const int q = ((int)k) & 3;
  // quadrant q: (s, c) = (sn, cs), (cs, -sn), (-sn, -cs), (-cs, sn).  Rounding
  // to float commutes with negation, so both are rounded first and the
  // quadrant is applied as selects and sign flips (no divergent branch
  // between the two keypoints a wave orients)
  const float fs = (float)sn, fc = (float)cs;
  const bool odd = q & 1;
  const uint32_t sgnS = (uint32_t)(q & 2) << 30, sgnC = (uint32_t)((q + 1) & 2) << 30;
  *s_out = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, odd ? fc : fs) ^ sgnS);
  *c_out = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, odd ? fs : fc) ^ sgnC);
}

// ------------------------------------------------ A.7 pinned log (double)
// Natural log by the classic fdlibm scheme: x = 2^k (1+f) with 1+f in
// [sqrt(2)/2, sqrt(2)), s = f/(2+f), log(1+f) = f - (hf - s (hf + R(s^2)))
// with a degree-14 even polynomial R; all in double, same operation sequence
// as the oracle.  MapPoint::PredictScale's logf(ratio) is pinned to
// (float)pinned_log((double)ratio).  Inputs are floats widened to double, so
// no subnormal double ever reaches it.
__device__ __forceinline__ double pinned_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (!(x > 0.0)) return x == 0.0 ? -__builtin_inf() : __builtin_nan("");
  if (x == __builtin_inf()) return x;
  const unsigned long long bits = (unsigned long long)__double_as_longlong(x);
  int hx = (int)(bits >> 32);
  const unsigned int lx = (unsigned int)bits;
  int k = (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int i = (hx + 0x95f64) & 0x100000;  // 1 when the mantissa is >= sqrt(2)
  const double m = __longlong_as_double(
      (long long)(((unsigned long long)(unsigned int)(hx | (i ^ 0x3ff00000)) << 32) | lx));
  k += i >> 20;
  const double f = m - 1.0, dk = (double)k;
  if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2^-20
    if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f), z = s * s, w = z * z;
  const double t1 = w * (L2 + w * (L4 + w * L6));
  const double t2 = z * (L1 + w * (L3 + w * (L5 + w * L7)));
  const double R = t2 + t1;
  if (((hx - 0x6147a) | (0x6b851 - hx)) > 0) {
    const double hf = 0.5 * f * f;
    return k == 0 ? f - (hf - s * (hf + R)) : dk * ln2_hi - ((hf - (s * (hf + R) + dk * ln2_lo)) - f);
  }
  return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// Buffer resources: 32-bit per-lane offsets (no 64-bit address VALU) and a
// hardware range check per dword (a dword load that ends past `bytes` reads
// as 0, a store past it is dropped).  Build only from wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t buf_ld32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
}
__device__ __forceinline__ uint32_t buf_ld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b8(r, (int)off, 0, 0);
}
__device__ __forceinline__ void buf_st32(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, 0, 0);
}

// A byte image behind a buffer resource built from its 4-aligned-down base:
// image byte o lives at resource offset o + sh.
struct ImgRsrc {
  __amdgpu_buffer_rsrc_t r;
  uint32_t sh;
};
__device__ __forceinline__ ImgRsrc img_rsrc(const uint8_t* p, uint32_t bytes) {
  ImgRsrc ir;
  ir.sh = (uint32_t)((uintptr_t)p & 3);
  ir.r = make_rsrc(p - ir.sh, (bytes + ir.sh + 3) & ~3u);
  return ir;
}

// Staging split in two for software pipelining.  A workgroup walking the same
// tile of several images (resize, blur) stages, per thread, NQ dwords of a
// tile of nR rows x rowW dwords (nR * rowW <= NQ * 256; element
// i = q*256 + tid -> row i / rowW, dword i % rowW).  The caller computes the
// element byte offsets once (they are the same in every image), issue() puts
// one image's loads in flight into registers, and commit() realigns them into
// LDS.  The next image's tile is issued before the current one is computed,
// so its HBM round trip overlaps that work.  Aligned (wave-uniform) tiles skip
// the second load and realign by 0.  The division by rowW is a multiply-high:
// i / d = umulhi(2i, ceil(2^31 / d)) for i < 2^20, d >= 1 (2^31 rather than
// 2^32 so that d = 1 has a 32-bit magic).
__device__ __forceinline__ uint32_t div_magic(int d) {
  return (uint32_t)((0x7FFFFFFFull + (uint64_t)d) / (uint64_t)d);
}
template <int NQ>
struct TilePrefetch {
  uint32_t lo[NQ], hi[NQ], sh[NQ];
  // off[q] = byte offset of element q inside the image
  __device__ __forceinline__ void issue(const ImgRsrc& im, bool aligned, const uint32_t* off) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t o = off[q] + im.sh;
      sh[q] = o & 3u;
      lo[q] = buf_ld32(im.r, o & ~3u);
      hi[q] = aligned ? 0u : buf_ld32(im.r, (o & ~3u) + 4);
    }
  }
  __device__ __forceinline__ void commit(uint32_t* lds, int ldsPitch, int nR, int rowW,
                                         uint32_t magic) const {
    // the thread index is laundered through an empty asm so that the LDS
    // addresses are recomputed per image instead of held across the image loop
    int tid = (int)threadIdx.x;
    __asm__ volatile("" : "+v"(tid));
    const int n = nR * rowW;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t i = (uint32_t)(q * 256 + tid);
      const uint32_t r = __umulhi(i << 1, magic), c = i - r * (uint32_t)rowW;
      if ((int)i < n) lds[r * ldsPitch + c] = __builtin_amdgcn_alignbyte(hi[q], lo[q], sh[q]);
    }
  }
};

// ------------------------------------------------------------- Hamming
// DescriptorDistance (src/ORBmatcher.cc:1814-1830) == popcount(a ^ b) over 256 bits.
__device__ __forceinline__ int hamming256(const ulonglong4 a, const ulonglong4 b) {
  return __popcll(a.x ^ b.x) + __popcll(a.y ^ b.y) + __popcll(a.z ^ b.z) + __popcll(a.w ^ b.w);
}
__device__ __forceinline__ ulonglong4 load_desc(const uint8_t* p) {
  return *reinterpret_cast<const ulonglong4*>(p);
}

// ------------------------------------------------------ wave primitives
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Inclusive prefix sum over the 64 lanes with DPP (row_shr 1/2/4/8 inside
// each 16-lane row, then row_bcast 15 and 31 across rows): six VALU ops, no
// LDS round trips.  All 64 lanes must be active.
__device__ __forceinline__ int wave_incl_scan(int v) {
  // row_shr steps with bound_ctrl (lanes shifted in read 0): hipcc folds each
  // into one v_add_u32_dpp instead of a v_mov_b32_dpp + v_add pair
  v += __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_mov_dpp(v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_mov_dpp(v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Sum over the 64 lanes, returned (wave-uniform) in every lane.
__device__ __forceinline__ int wave_sum(int v) {
  return __builtin_amdgcn_readlane(wave_incl_scan(v), 63);
}

// Block-wide exclusive scan of one value per thread; returns the exclusive
// prefix, *total receives the block sum.  `tmp` = LDS scratch of >= 17 ints.
// Must be called by all threads of the block.
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* total) {
  const int l = lane_id(), w = (int)(threadIdx.x >> 6), nw = (int)((blockDim.x + 63) >> 6);
  const int inc = wave_incl_scan(v);
  if (l == 63) tmp[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < nw; ++i) { const int t = tmp[i]; tmp[i] = acc; acc += t; }
    tmp[16] = acc;
  }
  __syncthreads();
  const int r = tmp[w] + inc - v;
  *total = tmp[16];
  __syncthreads();
  return r;
}

// Packed candidate keypoint: x (12b) | y (12b) << 12 | FAST score (8b) << 24.
__device__ __forceinline__ uint32_t pack_key(int x, int y, int s) {
  return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)s << 24);
}
__device__ __forceinline__ int key_x(uint32_t k) { return (int)(k & 0xFFFu); }
__device__ __forceinline__ int key_y(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
__device__ __forceinline__ int key_s(uint32_t k) { return (int)(k >> 24); }

// Workgroups are dispatched round-robin over the 8 XCDs (linear id L runs on
// XCD L % 8), and each XCD has its own L2.  With a (work item, image) grid that
// spreads one image's neighbouring cells / keypoint runs over all eight L2s, so
// every XCD fetches every image.  xcd_swizzle remaps the linear id so that XCD
// k runs one contiguous range of (blockIdx.x, blockIdx.y): the workgroups in
// flight on an XCD cover a couple of images, whose rows its L2 then serves.
#ifndef ORB_XCD_SWIZZLE
#define ORB_XCD_SWIZZLE 1
#endif
__device__ __forceinline__ void xcd_swizzle(int& bx, int& by) {
  const int gx = gridDim.x, n = gx * gridDim.y;
  const int L = blockIdx.x + gx * blockIdx.y;
  if (!ORB_XCD_SWIZZLE) {
    bx = blockIdx.x;
    by = blockIdx.y;
    return;
  }
  const int xcd = L & 7, pos = L >> 3, q = n >> 3, r = n & 7;
  const int logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  by = logical / gx;
  bx = logical - by * gx;
}
// The same over a 3-D grid (x fastest, then y, then z): XCD k runs one
// contiguous range of (x, y, z).
#ifndef ORB_XCD_SWIZZLE3
#define ORB_XCD_SWIZZLE3 1
#endif
__device__ __forceinline__ void xcd_swizzle3(int& bx, int& by, int& bz) {
  const int gx = gridDim.x, gxy = gx * gridDim.y, n = gxy * gridDim.z;
  if (!ORB_XCD_SWIZZLE3) {
    bx = blockIdx.x;
    by = blockIdx.y;
    bz = blockIdx.z;
    return;
  }
  const int L = blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z;
  const int xcd = L & 7, pos = L >> 3, q = n >> 3, r = n & 7;
  const int logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  bz = logical / gxy;
  const int rem = logical - bz * gxy;
  by = rem / gx;
  bx = rem - by * gx;
}

