// extractor_kernels.hip -- gfx950 kernels of the ORB extractor (ORBextractor::operator()).
//
// Pipeline for a batch of B images (every launch covers all B images; HBM
// layout in DESIGN.md §3):
//   k_pyr_resize   x (nlevels-1)  bilinear level l from level l-1    src/ORBextractor.cc:1172-1207
//   k_fast_cells   x 3            FAST-9/16 + cell-local NMS + iniTh  src/ORBextractor.cc:785-865
//                                 -> minTh fallback, one wave per cell; level 0's cells,
//                                 then levels 1-2, on a side stream beside the resize
//                                 chain; levels >= 3 after it
//   (k_fast_band   x 1            the same per band of cells; single frames, oversized cells)
//   k_octree       x 1            DistributeOctTree, one workgroup    src/ORBextractor.cc:558-782
//                                 per (image, level), list order emulated exactly
//   k_orient_desc  x 1            IC_Angle + rBRIEF-256 with the 7x7  src/ORBextractor.cc:77-164,
//                                 blur fused (each sample blurred     1131-1167
//                                 from LDS row sums), two keypoints per wave, rescale
//   (k_blur_levels: one image's blurred levels on demand, orb_extractor_blurred_level)
// Bit-exactness contract: every output byte equals the CPU oracle
// (oracle/orb_oracle.cpp) on the same image.
#include <stdlib.h>
#include <type_traits>
#include <algorithm>
#include "orb_device.h"
#include "orb_plan.h"
#include "orb_pattern_data.h"
#include "../../include/orb_abi.h"

// ============================================================ k_pyr_resize
// cv::resize(prev, level, sz, 0, 0, INTER_LINEAR) on 8U with OpenCV's 11-bit
// fixed-point weights.  The weight tables are computed
// on the host with the reference's float/double expressions; the kernel only
// does the integer taps.  One workgroup per 128 x 32 output tile: the source
// window is staged in LDS as aligned dwords (realigned from any source stride),
// each thread produces 4 columns x 4 rows and stores whole dwords, so a wave
// writes two full 128-byte rows per store.
#define PYR_TW 128
#ifndef PYR_IMAGES_PER_WG
#define PYR_IMAGES_PER_WG 16  // images per k_pyr_resize workgroup
#endif
#define PYR_TH 32
#ifndef PYR_TARGET_WGS
// > 0: fewer images per workgroup below this many workgroups per level.  At
// 2048, 16 C5 frames resize in 0.138 instead of 0.198 ms and C3 gains 2.5 %,
// but C5's pipelined rate loses 5.5 % (the wider resize crowds the matcher's
// 16-CU resolve) and the headline is unchanged (profiles/r05_resize_target.txt)
#define PYR_TARGET_WGS 0
#endif
// Staged source window (rows x dwords): >= the source rows a 32-row output
// tile touches, multiple of 4, and >= the dwords of source row a 128-column
// tile touches + 2 read-ahead.  Narrow: scale factors <= 1.25 (every ORB-SLAM2
// configuration uses 1.2); wide: <= 1.9 (the planner checks every tile).
#define PYR_SROWS 44
#define PYR_SW 44
#define PYR_SROWS_WIDE 64
#define PYR_SW_WIDE 64

// Levels whose tiles fit neither staged window (per-level downscales beyond
// ~1.9): one thread per 4 output pixels, its taps read straight from the
// source level with byte loads -- the same integer expressions as
// k_pyr_resize, bit-identical, without the staging.
__global__ __launch_bounds__(256) void k_pyr_resize_generic(
    const uint8_t* __restrict__ src, long long srcImgPitch, int srcStride, int sw, int sh,
    uint8_t* __restrict__ dst, long long dstImgPitch, int dstStride, int dw, int dh,
    const int* __restrict__ xofs, const int* __restrict__ alpha, const int* __restrict__ yofs,
    const int* __restrict__ beta) {
  const int xs = 4 * (blockIdx.x * 64 + (int)(threadIdx.x & 63));
  const int y = blockIdx.y * 4 + (int)(threadIdx.x >> 6);
  if (xs >= dw || y >= dh) return;
  const ImgRsrc im = img_rsrc(src + (long long)blockIdx.z * srcImgPitch,
                              (uint32_t)((sh - 1) * srcStride + sw));
  const int sy0 = min(max(yofs[y], 0), sh - 1), sy1 = min(max(yofs[y] + 1, 0), sh - 1);
  const uint32_t b = (uint32_t)beta[y], b0 = b & 0xFFFFu, b1 = b >> 16;
  const uint32_t r0 = (uint32_t)(sy0 * srcStride) + im.sh, r1 = (uint32_t)(sy1 * srcStride) + im.sh;
  uint32_t packed = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int dx = min(xs + j, dw - 1);
    const int sx = xofs[dx], sx1 = min(sx + 1, sw - 1);  // past xmax the weights are (2048, 0)
    const uint32_t a = (uint32_t)alpha[dx], a0 = a & 0xFFFFu, a1 = a >> 16;
    const uint32_t h0 = a0 * buf_ld8(im.r, r0 + sx) + a1 * buf_ld8(im.r, r0 + sx1);
    const uint32_t h1 = a0 * buf_ld8(im.r, r1 + sx) + a1 * buf_ld8(im.r, r1 + sx1);
    int v = min((int)((__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22), 255);
    __asm__ volatile("" : "+v"(v));  // see k_pyr_resize
    packed |= (uint32_t)v << (8 * j);
  }
  const __amdgpu_buffer_rsrc_t rd =
      make_rsrc(dst + (long long)blockIdx.z * dstImgPitch, (uint32_t)(dh * dstStride));
  buf_st32(rd, (uint32_t)(y * dstStride + xs), packed);
}

// Source-window staging in 16-byte groups: element i of a window of nR rows x
// nG groups (4 dwords each) is row i / nG, group i % nG.  One b128 load per
// group (+ one dword for the realignment of an unaligned source) instead of
// one or two dword loads per dword, one b128 LDS store.  The window's dword
// pitch is a multiple of 4 and >= 4 nG, so a group never crosses a row.
#ifndef PYR_LOAD16
#define PYR_LOAD16 1
#endif
template <int NQ>
struct TilePrefetch16 {
  uint32_t w[NQ][5], sh[NQ];
  __device__ __forceinline__ void issue(const ImgRsrc& im, bool aligned, const uint32_t* off) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t o = off[q] + im.sh;
      sh[q] = o & 3u;
      const uint32_t a = o & ~3u;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(im.r, (int)a, 0, 0);
      w[q][0] = (uint32_t)v[0];
      w[q][1] = (uint32_t)v[1];
      w[q][2] = (uint32_t)v[2];
      w[q][3] = (uint32_t)v[3];
      w[q][4] = aligned ? 0u : buf_ld32(im.r, a + 16);
    }
  }
  __device__ __forceinline__ void commit(uint32_t* lds, int ldsPitch, int nR, int nG,
                                         uint32_t magic, bool aligned) const {
    int tid = (int)threadIdx.x;
    __asm__ volatile("" : "+v"(tid));  // see TilePrefetch::commit
    const int n = nR * nG;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t i = (uint32_t)(q * 256 + tid);
      const uint32_t r = __umulhi(i << 1, magic), g = i - r * (uint32_t)nG;
      if ((int)i < n) {
        uint4 d;
        if (aligned) {
          d = make_uint4(w[q][0], w[q][1], w[q][2], w[q][3]);
        } else {
          d.x = __builtin_amdgcn_alignbyte(w[q][1], w[q][0], sh[q]);
          d.y = __builtin_amdgcn_alignbyte(w[q][2], w[q][1], sh[q]);
          d.z = __builtin_amdgcn_alignbyte(w[q][3], w[q][2], sh[q]);
          d.w = __builtin_amdgcn_alignbyte(w[q][4], w[q][3], sh[q]);
        }
        *reinterpret_cast<uint4*>(lds + r * ldsPitch + 4 * g) = d;
      }
    }
  }
};

template <bool ALIGNED, int SROWS = PYR_SROWS, int SW = PYR_SW>
__global__ __launch_bounds__(256) void k_pyr_resize(
    const uint8_t* __restrict__ src, long long srcImgPitch, int srcStride, int sw, int sh,
    uint8_t* __restrict__ dst, long long dstImgPitch, int dstStride, int dw, int dh,
    const int* __restrict__ xofs, const int* __restrict__ alpha,
    const int* __restrict__ yofs, const int* __restrict__ beta, int nImg) {
  // alpha/beta pack the two 11-bit weights as (w1 << 16) | (w0 & 0xFFFF).
  // A workgroup takes one output tile of images blockIdx.z, + gridDim.z, ...:
  // weight tables and the source window are loaded once, and the next image's
  // window is loaded into registers while the current one is computed.
  __shared__ __attribute__((aligned(16))) uint32_t tile[SROWS][SW];
  const int tid = threadIdx.x;
  const int tx = tid & 31, ty = tid >> 5;
  // XCD-contiguous tile order: a tile's neighbours (whose source windows
  // share 128-byte lines with it) run on the same XCD and hit its L2
  int bx, by, bz;
  xcd_swizzle3(bx, by, bz);
  const int x0 = bx * PYR_TW, y0 = by * PYR_TH;
  const int xs = x0 + 4 * tx;
  // this thread's weight tables, issued together with the source loads so the
  // workgroup pays one memory round trip before its compute
  int xo[4], al[4], yo[PYR_TH / 8], be[PYR_TH / 8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int dx = min(xs + j, dw - 1);
    xo[j] = xofs[dx];
    al[j] = alpha[dx];
  }
#pragma unroll
  for (int rr = 0; rr < PYR_TH / 8; ++rr) {
    const int y = min(y0 + (PYR_TH / 8) * ty + rr, dh - 1);
    yo[rr] = yofs[y];
    be[rr] = beta[y];
  }
  const int xl = min(x0 + PYR_TW - 1, dw - 1), yl = min(y0 + PYR_TH - 1, dh - 1);
  const int sxA = xofs[x0], sxB = min(xofs[xl] + 1, sw - 1);
  const int syA = min(max(yofs[y0], 0), sh - 1), syB = min(max(yofs[yl] + 1, 0), sh - 1);
  const int colBase = sxA & ~3;
  const int nW = ((sxB - colBase) >> 2) + 1, nR = syB - syA + 1;
  // staging: ALIGNED sources need one dword load per LDS dword, others two
  // (realigned with v_alignbyte); PYR_LOAD16: one b128 (+ one dword) per 4
  static_assert(SW % 4 == 0, "window pitch must hold whole 16-byte groups");
  const int nStage = PYR_LOAD16 ? (nW + 3) >> 2 : nW;  // staged elements per row
  const uint32_t magic = div_magic(nStage);
  constexpr int NQ = PYR_LOAD16 ? (SROWS * (SW / 4) + 255) / 256 : (SROWS * SW + 255) / 256;
  typename std::conditional<PYR_LOAD16, TilePrefetch16<NQ>, TilePrefetch<NQ>>::type pf;
  // staged element q of this thread: the same offset in every image, computed once
  uint32_t eoff[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t i = (uint32_t)min(q * 256 + tid, nR * nStage - 1);
    const uint32_t r = __umulhi(i << 1, magic), c = i - r * (uint32_t)nStage;
    eoff[q] = (syA + r) * (uint32_t)srcStride + (uint32_t)colBase + (PYR_LOAD16 ? 16 : 4) * c;
  }
  auto issue = [&](int z) {
    pf.issue(img_rsrc(src + (long long)z * srcImgPitch, (uint32_t)((sh - 1) * srcStride + sw)),
             ALIGNED, eoff);
  };
  int z = bz;
  if (z >= nImg) return;
  issue(z);
  // Horizontal taps with v_perm + v_dot2: the thread's 4 columns read source
  // bytes sx0 .. sx0+6 (scale <= 1.25), realigned once per source row into
  // (W0, W1); column j's pair (S[sx], S[sx+1]) is one v_perm into u16 lanes
  // and h = a0*S[sx] + a1*S[sx+1] one v_dot2_u32_u16.  Columns past xmax carry
  // weights (2048, 0) from the host table, which is exactly OpenCV's
  // S[sx]*2048 there.
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const int rel0 = xo[0] - colBase;
  const int k0 = rel0 >> 2, sh0 = rel0 & 3;
  uint32_t sel[4];
  u16x2 wts[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t bj = (uint32_t)(xo[j] - xo[0]);
    sel[j] = bj | (0x0Cu << 8) | ((bj + 1) << 16) | (0x0Cu << 24);
    wts[j] = __builtin_bit_cast(u16x2, (uint32_t)al[j]);
  }
  auto hrow = [&](int srow, uint32_t* h) {
    const uint32_t* R = tile[srow] + k0;
    const uint32_t w0 = R[0], w1 = R[1], w2 = R[2];
    const uint32_t W0 = __builtin_amdgcn_alignbyte(w1, w0, sh0);
    const uint32_t W1 = __builtin_amdgcn_alignbyte(w2, w1, sh0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      h[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(W1, W0, sel[j])),
                                    wts[j], 0u, false);
  };
  auto compute = [&](int zc) {
    // destination: arena level, pitch a multiple of 128 >= dw rounded to 4, so a
    // whole dword store at xs < dw stays inside the row (padding bytes unused)
    const __amdgpu_buffer_rsrc_t rd =
        make_rsrc(dst + (long long)zc * dstImgPitch, (uint32_t)(dh * dstStride));
#pragma unroll
    for (int rr = 0; rr < PYR_TH / 8; ++rr) {
      const int y = y0 + (PYR_TH / 8) * ty + rr;
      if (y >= dh) break;
      const uint32_t b0 = (uint32_t)be[rr] & 0xFFFFu, b1 = (uint32_t)be[rr] >> 16;
      uint32_t h0[4], h1[4];
      hrow(min(max(yo[rr], 0), sh - 1) - syA, h0);
      hrow(min(max(yo[rr] + 1, 0), sh - 1) - syA, h1);
      uint32_t packed = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // h <= 255*2048 and b <= 2048: 24-bit multiplies, sum < 2^31
        int v = min((int)((__umul24(h0[j], b0) + __umul24(h1[j], b1) + (1u << 21)) >> 22), 255);
        // opaque to instruction selection: ROCm 7.2 hipcc fuses shift+clamp+pack of
        // byte pairs into v_ashr_pk_u8_i32 and then ORs the next bytes into its
        // undefined upper half (observed miscompile on gfx950)
        __asm__ volatile("" : "+v"(v));
        packed |= (uint32_t)v << (8 * j);
      }
      buf_st32(rd, (uint32_t)(y * dstStride + xs), packed);
    }
  };
  for (; z < nImg; z += gridDim.z) {
    __syncthreads();  // the previous image's taps have read the window
#if PYR_LOAD16
    pf.commit(&tile[0][0], SW, nR, nStage, magic, ALIGNED);
#else
    pf.commit(&tile[0][0], SW, nR, nStage, magic);
#endif
    if (z + (int)gridDim.z < nImg) issue(z + gridDim.z);
    __syncthreads();
    if (xs >= dw) continue;
    compute(z);
  }
}

// ========================================================== k_pyr_resize2
// Two pyramid levels per launch: level l + 1 (the output tile, 128 x 32, as
// k_pyr_resize) from level l, and level l from level l - 1, in one workgroup.
// The workgroup computes the region R1 of level l that its output tile's taps
// read (plus the level-l pixels it owns, below) into LDS from the level l - 1
// window S0, writes the level-l pixels it owns to the arena, and computes its
// level-(l+1) tile from R1 without a global round trip.  Ownership partitions
// level l: tile (bx, by) owns columns [X0(bx), X0(bx + 1)) with X0(b) the
// 4-aligned first source column of output column 128 b (X0(0) = 0, the last
// tile to the level's width), rows likewise; R1 covers both the owned range
// and the taps, so a level-l pixel next to a tile edge is computed twice from
// the same integer expressions (identical bytes) and stored once.  Every level-l
// pixel is the OpenCV INTER_LINEAR value of k_pyr_resize (SURVEY.md Appendix
// A.2), so the pyramid is bit-identical; the launch replaces two dependent
// launches and level l is never read back from HBM.  The planner enables it
// for a pair of narrow levels whose every tile fits the windows below
// (orb_plan: lv[l].resize2).
#define PYR2_S0R 56   // level l-1 window rows
#define PYR2_S0W 56   // level l-1 window dwords per row (incl. 2 read-ahead)
#define PYR2_R1R PYR_SROWS  // level-l region rows (the narrow source window)
#define PYR2_R1W PYR_SW     // level-l region dwords per row (incl. 2 read-ahead)
#define PYR2_TAB 176        // level-l columns of the region's x tables (>= 4 x PYR2_R1W)

template <bool ALIGNED>
__global__ __launch_bounds__(256) void k_pyr_resize2(
    const uint8_t* __restrict__ src, long long srcImgPitch, int srcStride, int w0, int h0,
    uint8_t* __restrict__ mid, long long midImgPitch, int midStride, int w1, int h1,
    const int* __restrict__ xo1, const int* __restrict__ al1, const int* __restrict__ yo1,
    const int* __restrict__ be1, uint8_t* __restrict__ dst, long long dstImgPitch, int dstStride,
    int w2, int h2, const int* __restrict__ xo2, const int* __restrict__ al2,
    const int* __restrict__ yo2, const int* __restrict__ be2, int nImg) {
  __shared__ __attribute__((aligned(16))) uint32_t s0[PYR2_S0R][PYR2_S0W];
  __shared__ __attribute__((aligned(16))) uint32_t r1[PYR2_R1R][PYR2_R1W];
  __shared__ __attribute__((aligned(16))) int sXo[PYR2_TAB], sAl[PYR2_TAB];
  __shared__ int sYo[PYR2_R1R], sBe[PYR2_R1R];
  const int tid = threadIdx.x;
  const int tx = tid & 31, ty = tid >> 5;
  int bx, by, bz;
  xcd_swizzle3(bx, by, bz);
  const int x0 = bx * PYR_TW, y0 = by * PYR_TH;
  const int xs = x0 + 4 * tx;
  // ---- level l+1 taps of this thread (as k_pyr_resize)
  int xo[4], al[4], yo[PYR_TH / 8], be[PYR_TH / 8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int dx = min(xs + j, w2 - 1);
    xo[j] = xo2[dx];
    al[j] = al2[dx];
  }
#pragma unroll
  for (int rr = 0; rr < PYR_TH / 8; ++rr) {
    const int y = min(y0 + (PYR_TH / 8) * ty + rr, h2 - 1);
    yo[rr] = yo2[y];
    be[rr] = be2[y];
  }
  // ---- R1: level-l columns [X0, X1e), rows [Y0, Y1e); owned [X0, ownX) x [Y0, ownY)
  const int xl = min(x0 + PYR_TW - 1, w2 - 1), yl = min(y0 + PYR_TH - 1, h2 - 1);
  const int X0 = x0 == 0 ? 0 : (xo2[x0] & ~3);
  const int ownX = x0 + PYR_TW >= w2 ? w1 : (xo2[x0 + PYR_TW] & ~3);
  const int X1e = max(min(xo2[xl] + 1, w1 - 1) + 1, ownX);
  const int Y0 = y0 == 0 ? 0 : min(max(yo2[y0], 0), h1 - 1);
  const int ownY = y0 + PYR_TH >= h2 ? h1 : min(max(yo2[y0 + PYR_TH], 0), h1 - 1);
  const int Y1e = max(min(max(yo2[yl] + 1, 0), h1 - 1) + 1, ownY);
  const int nG1 = (X1e - X0 + 3) >> 2, nR1 = Y1e - Y0;
  // ---- S0: the level l-1 window R1's taps read
  const int c0a = xo1[X0], c0b = min(xo1[min(X0 + 4 * nG1 - 1, w1 - 1)] + 1, w0 - 1);
  const int colBase0 = c0a & ~3;
  const int r0a = min(max(yo1[Y0], 0), h0 - 1), r0b = min(max(yo1[Y1e - 1] + 1, 0), h0 - 1);
  const int nW0 = ((c0b - colBase0) >> 2) + 1, nR0 = r0b - r0a + 1;
  // R1's tables in LDS (read per item below)
  for (int i = tid; i < 4 * nG1; i += 256) {
    const int dx = min(X0 + i, w1 - 1);
    sXo[i] = xo1[dx];
    sAl[i] = al1[dx];
  }
  if (tid < nR1) {  // both source rows of level-l row Y0 + tid, relative to r0a
    const int yy = yo1[Y0 + tid];
    sYo[tid] = (min(max(yy, 0), h0 - 1) - r0a) | ((min(max(yy + 1, 0), h0 - 1) - r0a) << 16);
    sBe[tid] = be1[Y0 + tid];
  }
  const int nStage = (nW0 + 3) >> 2;
  const uint32_t magic = div_magic(nStage);
  constexpr int NQ = (PYR2_S0R * (PYR2_S0W / 4) + 255) / 256;
  TilePrefetch16<NQ> pf;
  uint32_t eoff[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t i = (uint32_t)min(q * 256 + tid, nR0 * nStage - 1);
    const uint32_t r = __umulhi(i << 1, magic), c = i - r * (uint32_t)nStage;
    eoff[q] = (r0a + r) * (uint32_t)srcStride + (uint32_t)colBase0 + 16 * c;
  }
  auto issue = [&](int z) {
    pf.issue(img_rsrc(src + (long long)z * srcImgPitch, (uint32_t)((h0 - 1) * srcStride + w0)),
             ALIGNED, eoff);
  };
  int z = bz;
  if (z >= nImg) return;
  issue(z);
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  // one 4-column group of 2 source rows -> 4 horizontal sums (as k_pyr_resize's hrow)
  auto hsum = [](const uint32_t* R, int sh, const uint32_t* sel, const u16x2* wts, uint32_t* h) {
    const uint32_t w0_ = R[0], w1_ = R[1], w2_ = R[2];
    const uint32_t W0 = __builtin_amdgcn_alignbyte(w1_, w0_, sh);
    const uint32_t W1 = __builtin_amdgcn_alignbyte(w2_, w1_, sh);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      h[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(W1, W0, sel[j])),
                                    wts[j], 0u, false);
  };
  auto vsum = [](const uint32_t* ha, const uint32_t* hb, uint32_t b) {
    const uint32_t b0 = b & 0xFFFFu, b1 = b >> 16;
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int v = min((int)((__umul24(ha[j], b0) + __umul24(hb[j], b1) + (1u << 21)) >> 22), 255);
      __asm__ volatile("" : "+v"(v));  // see k_pyr_resize
      packed |= (uint32_t)v << (8 * j);
    }
    return packed;
  };
  // level l+1 taps from R1 (relative to X0 / Y0)
  const int rel0 = xo[0] - X0;
  const int k0 = rel0 >> 2, sh0 = rel0 & 3;
  uint32_t sel[4];
  u16x2 wts[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t bj = (uint32_t)(xo[j] - xo[0]);
    sel[j] = bj | (0x0Cu << 8) | ((bj + 1) << 16) | (0x0Cu << 24);
    wts[j] = __builtin_bit_cast(u16x2, (uint32_t)al[j]);
  }
  const int nItems = nR1 * nG1;
  const uint32_t gMagic = div_magic(nG1);
  for (; z < nImg; z += gridDim.z) {
    __syncthreads();  // the previous image's R1 reads are done (and the tables on the first pass)
    pf.commit(&s0[0][0], PYR2_S0W, nR0, nStage, magic, ALIGNED);
    if (z + (int)gridDim.z < nImg) issue(z + gridDim.z);
    __syncthreads();
    // ---- R1 (level l) from S0, owned groups to the arena
    {
      const __amdgpu_buffer_rsrc_t rm =
          make_rsrc(mid + (long long)z * midImgPitch, (uint32_t)(h1 * midStride));
      for (int i = tid; i < nItems; i += 256) {
        const int r = (int)__umulhi((uint32_t)i << 1, gMagic), g = i - r * nG1;
        const int4 xq = *reinterpret_cast<const int4*>(&sXo[4 * g]);
        const int4 aq = *reinterpret_cast<const int4*>(&sAl[4 * g]);
        const int xa[4] = {xq.x, xq.y, xq.z, xq.w}, aa[4] = {aq.x, aq.y, aq.z, aq.w};
        const int rl = xa[0] - colBase0;
        uint32_t s1[4];
        u16x2 w1v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t bj = (uint32_t)(xa[j] - xa[0]);
          s1[j] = bj | (0x0Cu << 8) | ((bj + 1) << 16) | (0x0Cu << 24);
          w1v[j] = __builtin_bit_cast(u16x2, (uint32_t)aa[j]);
        }
        const int sy = sYo[r] & 0xFFFF, sy1 = sYo[r] >> 16;
        uint32_t ha[4], hb[4];
        hsum(&s0[sy][rl >> 2], rl & 3, s1, w1v, ha);
        hsum(&s0[sy1][rl >> 2], rl & 3, s1, w1v, hb);
        const uint32_t v = vsum(ha, hb, (uint32_t)sBe[r]);
        r1[r][g] = v;
        if (Y0 + r < ownY && X0 + 4 * g < ownX)
          buf_st32(rm, (uint32_t)((Y0 + r) * midStride + X0 + 4 * g), v);
      }
    }
    __syncthreads();
    // ---- level l+1 tile from R1
    if (xs < w2) {
      const __amdgpu_buffer_rsrc_t rd =
          make_rsrc(dst + (long long)z * dstImgPitch, (uint32_t)(h2 * dstStride));
#pragma unroll
      for (int rr = 0; rr < PYR_TH / 8; ++rr) {
        const int y = y0 + (PYR_TH / 8) * ty + rr;
        if (y >= h2) break;
        uint32_t ha[4], hb[4];
        hsum(&r1[min(max(yo[rr], 0), h1 - 1) - Y0][k0], sh0, sel, wts, ha);
        hsum(&r1[min(max(yo[rr] + 1, 0), h1 - 1) - Y0][k0], sh0, sel, wts, hb);
        buf_st32(rd, (uint32_t)(y * dstStride + xs), vsum(ha, hb, (uint32_t)be[rr]));
      }
    }
  }
}

// ============================================================ k_fast_band
// FAST arc strength at the pixel `c` points to (LDS band of biased f16 pixels,
// row pitch `p` elements): m = max(best dark 9-arc, best bright 9-arc), where
// an arc's strength is the min over its 9 pixels of |I(p) - I(q)| on the
// matching side.  FAST(t) detects the pixel iff m > t, and for a detected
// corner OpenCV's cornerScore<16> is m - 1 whatever t is (SURVEY.md
// Appendix A.1).
typedef short s16x2 __attribute__((ext_vector_type(2)));

typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));

// Band pixels are staged as f16 1024 + I (bit pattern 0x6400 | I): every
// difference of two pixels, and every pixel +- (t + 1) with t <= 255, is an
// integer in a range f16 represents exactly, so the packed f16 min/max/add
// below are exact integer arithmetic with no conversion after staging.
#define FAST_BIAS 0x64006400u

__device__ __forceinline__ int fast_score(const _Float16* c, int p) {
  const int off[16] = {3 * p,      3 * p + 1,  2 * p + 2,  p + 3,       3,  -p + 3,
                       -2 * p + 2, -3 * p + 1, -3 * p,     -3 * p - 1, -2 * p - 2, -p - 3,
                       -3,         p - 3,      2 * p - 2,  3 * p - 1};
  // lane .x carries d = v - ring (dark side), .y carries -d (bright side):
  // the packed three-input v_pk_minimum3_f16 / v_pk_maximum3_f16 of gfx950 do
  // the arc network in 40 instructions.
  const _Float16 v = c[0];
  const h16x2 vv = {v, -v}, sg = {(_Float16)-1.0f, (_Float16)1.0f};
  h16x2 q[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const _Float16 ck = c[off[k]];
    const h16x2 cc = {ck, ck};
    q[k] = __builtin_elementwise_fma(cc, sg, vv);  // (v - ck, ck - v), exact
  }
  // 9-arc minimum = min3 of three 3-runs; best = max over the 16 starts
  h16x2 w3[16];
#pragma unroll
  for (int k = 0; k < 16; ++k)
    w3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(q[k], q[(k + 1) & 15]),
                                          q[(k + 2) & 15]);
  h16x2 w9[16];
#pragma unroll
  for (int k = 0; k < 16; ++k)
    w9[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(w3[k], w3[(k + 3) & 15]),
                                          w3[(k + 6) & 15]);
  h16x2 m5[6];
#pragma unroll
  for (int k = 0; k < 5; ++k)
    m5[k] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(w9[3 * k], w9[3 * k + 1]),
                                          w9[3 * k + 2]);
  m5[5] = w9[15];
  const h16x2 ma = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m5[0], m5[1]), m5[2]);
  const h16x2 mb = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m5[3], m5[4]), m5[5]);
  const h16x2 best = __builtin_elementwise_maximum(ma, mb);
  return (int)(float)__builtin_fmaxf16(best.x, best.y);
}

// One workgroup per (band, image).  A band is a run of cells of one cell row
// of one level (OrbBandDesc).  Cell detection windows (ROI shrunk by 3,
// src/ORBextractor.cc:819-843) tile the band interior without overlap, so
// every pixel's FAST arc strength is computed at most once for the whole band.
//
// LDS band: R rows x P f16 elements; element e of a row is band column
// e - FAST_LPAD, so interior column 3 (the first detectable one) sits at
// element 8 and 8-pixel groups of the interior start 16-byte aligned.
// Phase A (every cell, FAST at iniThFAST): compass pretest on 8 pixels per
// lane (packed f16, four pixel pairs), candidates appended to a queue that is
// scored in dense flushes (arc strengths), NMS of pixels with m > iniTh.
// Phase B (only cells with no phase-A keypoint, src/ORBextractor.cc:846-850):
// the same at minThFAST over those cells' windows, reusing phase-A strengths.
// NMS is per cell: a window's edge acts as cv::FAST's zero border (column
// edge flags); survivors go to an interior bitmap and one wave per cell
// compacts its window row by row (lane = row).  Output per cell: keypoints
// in row-major window order (cv::FAST's order), packed x | y<<12 | score<<24
// in level coordinates, and their count.
#define FAST_GROUPS 256    // 8-pixel groups pretested per round (one per thread)
#define FAST_QCAP 2560     // candidate queue (u16 element offsets)
#define FAST_QFLUSH (FAST_QCAP - 8 * FAST_GROUPS)  // score once the queue holds more
#define FAST_CORNERS 1024  // corner list capacity; beyond it NMS runs densely
#define FAST_LOADS 8       // source dwords per thread in flight while staging
#define FAST_LPAD 5        // element of band column 0
// Strength byte of a group pixel outside the interior: 1 is never a corner
// (m >= 2) and never suppresses one in NMS, so it only has to stop scoring.
#define FAST_OUTSIDE 0x01

__device__ __forceinline__ unsigned long long bit_run(const uint32_t* bits, int start, int n) {
  // bits [start, start + n) of a little-endian bit array, n <= 64
  const int w = start >> 5, sh = start & 31;
  unsigned long long v = (unsigned long long)bits[w] | ((unsigned long long)bits[w + 1] << 32);
  v >>= sh;
  if (sh) v |= (unsigned long long)bits[w + 2] << (64 - sh);
  return n >= 64 ? v : (v & ((1ull << n) - 1ull));
}

#ifndef FC_PRETEST4
#define FC_PRETEST4 1
#endif
// Compass pretest of a pixel pair (f16 halves): a pixel can be a FAST(t)
// corner only if two circularly adjacent compass pixels (circle positions
// 0,4,8,12) are both darker than v - t or both brighter than v + t.  Each
// adjacent pair takes one pixel of {0, 8} and one of {4, 12}, so
//   dark   <=>  max(min(q0, q8), min(q4, q12)) <= v - (t + 1)
//   bright <=>  min(max(q0, q8), max(q4, q12)) >= v + (t + 1).
// The sign bit (15 / 31) of the result is set for a pixel that fails both.
__device__ __forceinline__ uint32_t pretest_pair(uint32_t v, uint32_t q0, uint32_t q4, uint32_t q8,
                                                 uint32_t q12, h16x2 T) {
  const h16x2 V = __builtin_bit_cast(h16x2, v);
  const h16x2 Q0 = __builtin_bit_cast(h16x2, q0), Q4 = __builtin_bit_cast(h16x2, q4);
  const h16x2 Q8 = __builtin_bit_cast(h16x2, q8), Q12 = __builtin_bit_cast(h16x2, q12);
  const h16x2 A = __builtin_elementwise_maximum(__builtin_elementwise_minimum(Q0, Q8),
                                                __builtin_elementwise_minimum(Q4, Q12));
  const h16x2 B = __builtin_elementwise_minimum(__builtin_elementwise_maximum(Q0, Q8),
                                                __builtin_elementwise_maximum(Q4, Q12));
#if FC_PRETEST4
  // dark <=> V - A >= T, bright <=> B - V >= T: one max and one subtraction
  // of T instead of V -+ T, two differences and an AND (exact: every operand
  // is a small integer in f16)
  const h16x2 r = __builtin_elementwise_maximum(V - A, B - V) - T;
  return __builtin_bit_cast(uint32_t, r);
#else
  const h16x2 x = (V - T) - A;  // >= +0: dark
  const h16x2 y = B - (V + T);  // >= +0: bright
  return __builtin_bit_cast(uint32_t, x) & __builtin_bit_cast(uint32_t, y);
#endif
}

__global__ __launch_bounds__(256) void k_fast_band(
    const uint8_t* __restrict__ img0, long long img0Pitch, int img0Stride,
    const uint8_t* __restrict__ arena, long long arenaPitch, OrbPlanDesc plan,
    const OrbBandDesc* __restrict__ bands, const OrbCellDesc* __restrict__ cells, int nBands,
    uint32_t* __restrict__ cellKeys, int32_t* __restrict__ cellCount, int32_t* __restrict__ errFlag) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qCount, cCount;
  __shared__ uint32_t fbMask[2];  // cells (of this band) that fall back to minThFAST
  __shared__ int16_t cellX0[64], cellWW[64];  // cell windows: first interior column, width
  __shared__ int nFbK;
  const int img = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the image's status starts clean (k_octree may flag it, k_orient_desc reads it)
  if (blockIdx.x == 0 && tid == 0) errFlag[img] = 0;
  const int nw = blockDim.x >> 6;
  const int bandElems = plan.maxBandBytes;
  const int bitStride = ((bandElems >> 5) + 4) & ~1;  // even: colf / fbCol stay 8-aligned
  uint32_t* roi32 = (uint32_t*)smem;                            // R x P f16 band pixels
  const _Float16* roih = (const _Float16*)smem;
  uint8_t* sc = smem + 2 * bandElems;                           // R x P arc strengths
  uint16_t* queue = (uint16_t*)(sc + bandElems);                // FAST_QCAP candidates
  uint16_t* corners = queue + FAST_QCAP;                        // FAST_CORNERS corners
  uint32_t* bitsIni = (uint32_t*)(corners + FAST_CORNERS);      // interior survivors, iniTh
  uint32_t* bitsMin = bitsIni + bitStride;                      // interior survivors, minTh
  uint8_t* colf = (uint8_t*)(bitsMin + bitStride);              // window edge flags per column
  uint8_t* fbCol = colf + ((bandElems / 7 + 15) & ~7);          // 1: column in a fallback cell

  // A workgroup takes bands blockIdx.x, + gridDim.x, ...: the next band's
  // pixels and cell descriptors are loaded into registers while the current
  // band is processed, so each band's HBM round trip overlaps the previous
  // band's work.  Band pixels: source dword k of row r = bytes
  // [x0 - LPAD + 4k, +4) of the row (level 0 rows can start at any byte:
  // caller stride), through a buffer resource (32-bit offsets), the row split
  // by a 32-bit multiply-high instead of a division.  One batch of FAST_LOADS
  // dwords per thread covers a band (host-checked).
  uint32_t plo[FAST_LOADS], phi[FAST_LOADS], psft[FAST_LOADS];
  OrbCellDesc pcell = {};
  auto issue = [&](const OrbBandDesc& q) {
    const int ql = q.level, qR = q.y1 - q.y0, qC = q.x1 - q.x0;
    const uint8_t* qlvl;
    int qpitch;
    if (ql == 0) {
      qlvl = img0 + (long long)img * img0Pitch;
      qpitch = img0Stride;
    } else {
      qlvl = arena + (long long)img * arenaPitch + plan.lv[ql].arenaOff;
      qpitch = plan.lv[ql].pitch;
    }
    const int nS = ((qC + 20) & ~7) >> 2;  // source dwords per row
    const int n = max(qR * nS, 1);
    const uint32_t magic = (uint32_t)((0xFFFFFFFFull + (uint64_t)nS) / (uint64_t)nS);  // ceil(2^32/nS)
    const ImgRsrc im = img_rsrc(qlvl, (uint32_t)((plan.lv[ql].h - 1) * qpitch + plan.lv[ql].w));
    const uint32_t org = (uint32_t)(q.y0 * qpitch + q.x0 - FAST_LPAD) + im.sh;
#pragma unroll
    for (int k8 = 0; k8 < FAST_LOADS; ++k8) {
      const uint32_t i = (uint32_t)min(k8 * 256 + tid, n - 1);  // branch-free loads
      const uint32_t r = __umulhi(i, magic), k = i - r * (uint32_t)nS;
      const uint32_t o = org + r * (uint32_t)qpitch + 4 * k;
      psft[k8] = o & 3u;
      plo[k8] = buf_ld32(im.r, o & ~3u);
      phi[k8] = buf_ld32(im.r, (o & ~3u) + 4);
    }
    if (tid < q.nCells) pcell = cells[q.cellBeg + tid];
  };
  int b = blockIdx.x;
  if (b >= nBands) return;
  OrbBandDesc nbd = bands[b];
  issue(nbd);
  for (; b < nBands; b += gridDim.x) {
  const OrbBandDesc bd = nbd;
  const OrbCellDesc myCell = pcell;
  const int R = bd.y1 - bd.y0, C = bd.x1 - bd.x0;
  const long long slot0 = (long long)img * plan.ncells + bd.cellBeg;
  const bool tiny = R < 7 || C < 7;
  const int P = (C + 20) & ~7;  // LDS row pitch (elements): groups read up to element C + 12
  const int PD = P >> 1;        // dwords per LDS row (f16 pairs)
  if (!tiny) {
    // prefetched band -> LDS: each source dword becomes two f16 pairs (v_perm + bias)
    const int n = R * (P >> 2);
#pragma unroll
    for (int k8 = 0; k8 < FAST_LOADS; ++k8) {
      const int i = k8 * 256 + tid;
      if (i < n) {
        const uint32_t w = __builtin_amdgcn_alignbyte(phi[k8], plo[k8], psft[k8]);
        uint2 h;
        h.x = __builtin_amdgcn_perm(0u, w, 0x0C010C00u) | FAST_BIAS;
        h.y = __builtin_amdgcn_perm(0u, w, 0x0C030C02u) | FAST_BIAS;
        reinterpret_cast<uint2*>(roi32)[i] = h;
      }
    }
  }
  if (b + (int)gridDim.x < nBands) {
    nbd = bands[b + gridDim.x];
    issue(nbd);
  }
  if (tiny) {
    for (int c = tid; c < bd.nCells; c += 256) cellCount[slot0 + c] = 0;
    continue;
  }
  const int iw = C - 6, ih = R - 6, ni = iw * ih;
  const int nK = (iw + 7) >> 3;  // 8-pixel groups per interior row
  const int nBitWords = (ni >> 5) + 3;
  // cell windows of the band (<= 64 cells, host-checked)
  int cx0 = 0, ww = 0;
  if (tid < bd.nCells) {
    cx0 = myCell.x0 - bd.x0;
    ww = myCell.x1 - myCell.x0 - 6;
    cellX0[tid] = (int16_t)(ww > 0 ? cx0 : 0x7FFF);
    cellWW[tid] = (int16_t)ww;
  }
  for (int i = tid; i < nBitWords; i += 256) bitsIni[i] = 0;
  for (int i = tid; i < iw; i += 256) colf[i] = 0;
  if (tid == 0) {
    qCount = cCount = 0;
    fbMask[0] = fbMask[1] = 0;
  }
  __syncthreads();
  if (tid < bd.nCells && ww > 0) {
    colf[cx0] |= 1;           // left window edge: x-1 is outside
    colf[cx0 + ww - 1] |= 2;  // right window edge: x+1 is outside
  }
  const int ti = min(max(plan.iniTh, 0), 255), tm = min(max(plan.minTh, 0), 255);
  // Pixels j >= nvLast of a row's last group lie past the interior.  Phase A
  // does not mask them in the pretest: their strength byte starts at
  // FAST_OUTSIDE instead of 0, so a queued one is never scored or listed
  // (NMS and compaction never read those columns).
  const int nvLast = iw - 8 * (nK - 1);
  const unsigned long long outsideLast =
      nvLast >= 8 ? 0ull : (0x0101010101010101ull << (8 * nvLast));

  // Group columns pretested by a pass: all of them in phase A, only those
  // touching a fallback cell in phase B (fbK, built before phase B).
  uint16_t* fbK = (uint16_t*)(fbCol + ((bandElems / 7 + 15) & ~7));

  // Score the queued candidates (dense: 256 per pass) and list the corners
  // (m > t).  In phase B strengths already known from phase A are kept.
  // Phase A (fresh): nothing is scored yet, so the arc strength is computed
  // unconditionally and its 16 ring reads go out together with the strength
  // byte read (which only tells FAST_OUTSIDE pixels apart).
  auto flush = [&](int t, int nq, bool fresh) {
    for (int j0 = 0; j0 < nq; j0 += 256) {
      const int j = j0 + tid;
      bool corner = false;
      int off = 0;
      if (j < nq) {
        off = queue[j];
        int m;
        if (fresh) {
          const int s = min(max(fast_score(roih + off, P), 0), 255);
          m = sc[off];
          if (m == 0) {
            m = s;
            sc[off] = (uint8_t)m;
          }
        } else {
          m = sc[off];  // 0: not scored yet; phase B keeps phase-A strengths
          if (m == 0) {
            m = min(max(fast_score(roih + off, P), 0), 255);
            sc[off] = (uint8_t)m;
          }
        }
        corner = m > t && m >= 2;
      }
      const unsigned long long bal = __ballot(corner);
      int cb = 0;
      if (lane == 0 && bal) cb = atomicAdd(&cCount, __popcll(bal));
      cb = __builtin_amdgcn_readfirstlane(cb) +
           (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      if (corner && cb < FAST_CORNERS) corners[cb] = (uint16_t)off;
    }
    __syncthreads();
    if (tid == 0) qCount = 0;
    __syncthreads();
  };

  // One FAST pass at threshold t: pretest, queue, arc strengths, corner list.
  auto fast_pass = [&](int t, auto fbTag) {
    constexpr bool FB = decltype(fbTag)::value;
    h16x2 T;
    T.x = T.y = (_Float16)(float)(t + 1);
    const int nKp = FB ? nFbK : nK;
    const int nG = ih * nKp;
    const float invK = 1.0f / (float)nKp;
    for (int g0 = 0; g0 < nG; g0 += FAST_GROUPS) {
      const int gi = g0 + tid;
      uint32_t rp[4] = {0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
      int off = 0;
      if (gi < nG) {
        const int rr = (int)(((float)gi + 0.5f) * invK), kk = gi - rr * nKp;
        const int k = FB ? (int)fbK[kk] : kk;
        const int r = rr + 3;
        off = r * P + 8 + 8 * k;  // element of interior column 8k
        const uint32_t* row = roi32 + r * PD + 4 + 4 * k;
        const uint2 a = *reinterpret_cast<const uint2*>(row - 2);
        const uint4 b = *reinterpret_cast<const uint4*>(row);
        const uint2 c = *reinterpret_cast<const uint2*>(row + 4);
        const uint4 u = *reinterpret_cast<const uint4*>(row + 3 * PD);  // circle 0 (y + 3)
        const uint4 d = *reinterpret_cast<const uint4*>(row - 3 * PD);  // circle 8 (y - 3)
        const uint32_t D[8] = {a.x, a.y, b.x, b.y, b.z, b.w, c.x, c.y};  // dwords -2 .. 5
        const uint32_t U[4] = {u.x, u.y, u.z, u.w}, Dn[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t q4 = __builtin_amdgcn_alignbyte(D[i + 4], D[i + 3], 2);   // x + 3
          const uint32_t q12 = __builtin_amdgcn_alignbyte(D[i + 1], D[i], 2);      // x - 3
          rp[i] = pretest_pair(D[i + 2], U[i], q4, Dn[i], q12, T);
        }
        if (FB) {
          // only pixels of fallback cells (fbCol is 0 past the interior): one
          // 8-byte read of the group's column flags
          const unsigned long long fm = *reinterpret_cast<const unsigned long long*>(fbCol + 8 * k);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (!((fm >> (8 * j)) & 0xFFull)) rp[j >> 1] |= (j & 1) ? 0x80000000u : 0x8000u;
        } else {
          // strengths start at 0 (8 bytes, 8-aligned), FAST_OUTSIDE past the interior
          const unsigned long long z = k == nK - 1 ? outsideLast : 0ull;
          *reinterpret_cast<unsigned long long*>(sc + off) = z;
        }
      }
      // wave-aggregated append: one LDS atomic per wave, lane offsets by mbcnt
      unsigned long long bj[8];
      bool pass[8];
      int tot = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = rp[j >> 1];
        pass[j] = (j & 1) ? ((int)w >= 0) : ((short)(w & 0xFFFFu) >= 0);
        bj[j] = __ballot(pass[j]);
        tot += __popcll(bj[j]);
      }
      if (tot) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&qCount, tot);
        base = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(bj[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bj[j], (uint32_t)base));
          if (pass[j]) queue[pos] = (uint16_t)(off + j);
          base += __popcll(bj[j]);
        }
      }
      __syncthreads();
      // every wave reads the count before any wave appends again: the flush
      // synchronises; a round without one takes a second barrier
      const int nq = qCount;
      if (nq > FAST_QFLUSH || g0 + FAST_GROUPS >= nG) flush(t, nq, !FB);
      else __syncthreads();
    }
  };

  // NMS at threshold t of every corner (m > t) into `bits`: a corner survives
  // iff no neighbour inside its window has nb > t && nb >= m.  Dense over the
  // (fallback-)interior when the corner list overflowed.
  auto nms_pass = [&](int t, uint32_t* bits, bool fallbackOnly) {
    const int nc = cCount;
    const bool dense = nc > FAST_CORNERS;
    const int nItems = dense ? ni : nc;
    for (int j = tid; j < nItems; j += 256) {
      int x, y, off;
      if (dense) {
        y = (int)(((float)j + 0.5f) / (float)iw);
        x = j - y * iw;
        off = (y + 3) * P + (x + 8);
        if (fallbackOnly && !fbCol[x]) continue;
      } else {
        off = corners[j];
        const int ry = (int)(((float)off + 0.5f) / (float)P);
        y = ry - 3;
        x = off - ry * P - 8;
      }
      // the strength, the column's window-edge flags and all 8 neighbours are
      // read in one LDS round trip (every neighbour element lies inside the
      // band); neighbours outside the cell window count as 0 (cv::FAST's border)
      const uint8_t* c = sc + off;
      const int m = c[0], cf = colf[x];
      const int r0 = c[-P - 1], r1 = c[-P], r2 = c[-P + 1], r3 = c[-1], r4 = c[1], r5 = c[P - 1],
                r6 = c[P], r7 = c[P + 1];
      if (m <= t || m < 2) continue;
      const bool L = !(cf & 1), Rt = !(cf & 2), U = y > 0, D = y < ih - 1;
      const int nb[8] = {(U && L) ? r0 : 0, U ? r1 : 0, (U && Rt) ? r2 : 0, L ? r3 : 0,
                         Rt ? r4 : 0, (D && L) ? r5 : 0, D ? r6 : 0, (D && Rt) ? r7 : 0};
      bool ok = true;
#pragma unroll
      for (int k = 0; k < 8; ++k) ok = ok && !(nb[k] > t && nb[k] >= m);
      if (ok) {
        const int bit = y * iw + x;
        atomicOr(&bits[bit >> 5], 1u << (bit & 31));
      }
    }
  };

  // Compaction of cell ci from `bits`, one wave, lane = window row (ih <= 64,
  // host-checked).  Returns the cell's key count (wave-uniform).
  auto compact = [&](int ci, const uint32_t* bits) -> int {
    const int cx0 = cellX0[ci], ww = cellWW[ci];
    if (ww <= 0) return 0;
    uint32_t* out = cellKeys + (slot0 + ci) * plan.keyCap;
    unsigned long long row = lane < ih ? bit_run(bits, lane * iw + cx0, ww) : 0ull;
    const int cnt = __popcll(row);
    const int incl = wave_incl_scan(cnt);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    int o = incl - cnt;
    // two keys per iteration: both strength reads are in flight together
    const uint8_t* srow = sc + (lane + 3) * P + cx0 + 8;
    const uint32_t kx = (uint32_t)(bd.x0 + 3 + cx0), ky = (uint32_t)(bd.y0 + 3 + lane);
    while (row) {
      const int x0 = __builtin_ctzll(row);
      row &= row - 1;
      const bool two = row != 0;
      const int x1 = two ? __builtin_ctzll(row) : x0;
      if (two) row &= row - 1;
      const int m0 = srow[x0], m1 = srow[x1];
      out[o] = pack_key(kx + x0, ky, m0 - 1);
      if (two) out[o + 1] = pack_key(kx + x1, ky, m1 - 1);
      o += two ? 2 : 1;
    }
    return total;
  };

  // ---- phase A: every cell at iniThFAST
  fast_pass(ti, std::false_type{});
  nms_pass(ti, bitsIni, false);
  __syncthreads();
  for (int ci = wave; ci < bd.nCells; ci += nw) {
    const int n = compact(ci, bitsIni);
    if (lane == 0) {
      if (n == 0 && tm != ti) atomicOr(&fbMask[ci >> 5], 1u << (ci & 31));
      else cellCount[slot0 + ci] = n;
    }
  }
  if (tid == 0) cCount = 0;
  __syncthreads();
  if ((fbMask[0] | fbMask[1]) == 0) { continue; }  // LDS free: barrier above
  // ---- phase B: cells without an iniThFAST keypoint, at minThFAST, over the
  // group columns that touch one (wave 0 lists them in order with ballots).
  // Column flags fbCol[x] (x < 8 nK) = column x lies in a fallback cell: the
  // cells tile the interior left to right, so x's cell is the last one
  // starting at or before x.
  for (int x = tid; x < 8 * nK; x += 256) {
    uint8_t f = 0;
    if (x < iw) {
      int c = 0;
      while (c + 1 < bd.nCells && cellX0[c + 1] <= x) ++c;
      f = (uint8_t)((fbMask[c >> 5] >> (c & 31)) & 1u);
    }
    fbCol[x] = f;
  }
  for (int i = tid; i < nBitWords; i += 256) bitsMin[i] = 0;
  __syncthreads();
  if (wave == 0) {
    int cnt = 0;
    for (int k0 = 0; k0 < nK; k0 += 64) {
      const int k = k0 + lane;
      bool hit = false;
      if (k < nK) hit = *reinterpret_cast<const unsigned long long*>(fbCol + 8 * k) != 0ull;
      const unsigned long long b = __ballot(hit);
      if (hit) fbK[cnt + __popcll(b & ((1ull << lane) - 1ull))] = (uint16_t)k;
      cnt += __popcll(b);
    }
    if (lane == 0) nFbK = cnt;
  }
  __syncthreads();
  fast_pass(tm, std::true_type{});
  nms_pass(tm, bitsMin, true);
  __syncthreads();
  for (int ci = wave; ci < bd.nCells; ci += nw) {
    if (!((fbMask[ci >> 5] >> (ci & 31)) & 1u)) continue;
    const int n = compact(ci, bitsMin);
    if (lane == 0) cellCount[slot0 + ci] = n;
  }
  __syncthreads();  // the next band's pixels overwrite LDS
  }  // band loop
}

// v_cndmask with a wave-uniform 64-bit lane mask as the condition: lanes whose
// bit is set take ifSet.  (A select on a per-lane bool derived from a ballot
// makes hipcc rebuild the mask through VGPR 0/1 values and compares.)
__device__ __forceinline__ int lane_select(unsigned long long mask, int ifSet, int ifClear) {
  int r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(ifClear), "v"(ifSet), "s"(mask));
  return r;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ============================================================ k_fast_cells
// FAST per cell, one wave per cell (src/ORBextractor.cc:816-865), no
// workgroup barriers: a wave stages its cell's ROI (cell + the 3-px FAST
// border) as bytes in its own LDS slice, pretests 8 pixels per lane (compass
// test), queues the candidates with wave ballots, scores them (arc strengths),
// lists the corners (m > t), runs the cell-local 3x3 NMS into a row bitmap and
// compacts it row by row (lane = window row).  A cell without a keypoint at
// iniThFAST reruns the same at minThFAST over its window, keeping the
// strengths already computed (:846-850).  Output per cell: keys in row-major
// window order (cv::FAST's order), packed x | y << 12 | score << 24 in level
// coordinates, and their count.
//
// Arithmetic: a pixel byte I is read as the f16 whose bit pattern is I, i.e.
// the subnormal I * 2^-24 (f16 subnormals are kept: the kernel runs with
// .amdhsa_float_denorm_mode_16_64 3).  Differences and sums of such values
// (|.| < 1024 * 2^-24) are exact, so the packed f16 three-input min / max of
// gfx950 do exact integer arithmetic on pixels with no conversion: a byte
// loaded by ds_read_u8 is already its f16, and a pair of bytes becomes an f16
// pair with one v_perm.  The tile is one byte per pixel, which keeps a wave's
// LDS slice at ~7 KB (22-24 waves per CU; occupancy is what this
// latency-bound kernel's time follows).
#ifndef FC_WAVES
#define FC_WAVES 1      // waves per workgroup (LDS slices; swept 1-4)
#endif
#ifndef FC_CPW
#define FC_CPW 4        // cells per wave (software-pipelined ROI loads)
#endif
#ifndef FC_QCAP
// candidate queue per wave (one pretest round adds <= 512; a flush once it
// holds more than 128): 640 against 768 trims the wave's LDS slice to 5.7 KB,
// FAST alone 1.334 -> 1.283 ms per 1024 frames (profiles/r04_variants.txt)
#define FC_QCAP 640
#endif
#ifndef FC_CCAP
#define FC_CCAP 256     // corner list per wave; beyond it the NMS runs densely
#endif
#ifndef FC_PAD
#define FC_PAD 0        // extra LDS row pitch (bytes, multiple of 8)
#endif
#ifndef FC_LOAD3
#define FC_LOAD3 0      // three 16-byte row loads instead of four where the ROI fits (A/B knob)
#endif
#ifndef FC_ROWMAJOR
#define FC_ROWMAJOR 1   // candidates queued in row-major order, keys written by NMS in order
#endif
#ifndef FC_PERM
#define FC_PERM (!FC_ROWMAJOR)  // pretest lane -> pixel-group permutation (LDS banking)
#endif
// Attribution builds (phase stubs, per-phase clock stamps; results wrong,
// never shipped) are patches against this file: tools/attribution/.

// LDS row pitch (bytes) of a cell ROI C pixels wide: byte 5 is ROI column 0,
// byte 8 interior column 0 (ROI column 3); groups of 8 interior pixels read
// [8k, 8k + 24).  FC_TIGHT: the pitch only has to hold the row (bytes 0 ..
// C + 4, a multiple of 8 for the b64 reads): a row's last group may read up to
// 12 bytes into the next row, but only for pixels past the interior, which the
// pass mask drops (every ORB-SLAM2 grid: ROI widths 36-43 -> 48 instead of 56
// bytes, and with the NMS bitmap gone from the row-major path, 7.0 -> 5.9 KB
// of LDS per wave: 22 -> 27 waves per CU, the limit of this kernel's occupancy)
#ifndef FC_TIGHT
#define FC_TIGHT 1
#endif
__host__ __device__ inline int fc_pitch(int C) {
  return (FC_TIGHT ? ((C + 12) & ~7) : ((C + 20) & ~7)) + FC_PAD;
}
__host__ __device__ inline int fc_tile_elems(int maxRows, int maxCols) {
  return (maxRows * fc_pitch(maxCols) + 15) & ~15;  // 16-byte aligned strength map
}
__host__ __device__ inline int fc_wave_bytes(int tileElems) {
  // byte tile + strengths + queue + corners (+ 64 rows x 64-bit NMS bitmap,
  // column-major path only)
  return ((2 * tileElems + 2 * FC_QCAP + 2 * FC_CCAP + ((FC_ROWMAJOR && FC_TIGHT) ? 0 : 512)) + 15) &
         ~15;
}
#define FC_CONST_PITCH (FC_TIGHT ? 48 : 56)  // the compile-time instance

// f16 pair {byte i0, byte i1} of the 8 bytes {hi:lo} (i in 0..7, lo first)
__device__ __forceinline__ uint32_t byte_pair(uint32_t hi, uint32_t lo, int i0, int i1) {
  return __builtin_amdgcn_perm(hi, lo, (uint32_t)i0 | 0x0C00u | ((uint32_t)i1 << 16) | 0x0C000000u);
}

// FAST arc strength of the byte pixel at `c` (row pitch p bytes), as
// fast_score on the subnormal encoding above.  Dark and bright strengths ride
// in one f16 pair (lo, hi) = (-max c, min c) over the ring: the first min3
// layer reads each ring byte from the low half for both lanes (op_sel_hi 0)
// and negates the low lane (neg_lo), so the raw ds_read_u8 values need no
// conversion; the pixel value enters once at the end:
//   dark = max_k min_arc (v - c) = v + max_k (-max_arc c),
//   bright = max_k min_arc (c - v) = max_k min_arc c - v.
#ifndef FC_SCORE_RAW
#define FC_SCORE_RAW 1
#endif
__device__ __forceinline__ uint32_t pk_min3_negpair(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_pk_minimum3_f16 %0, %1, %2, %3 op_sel_hi:[0,0,0] neg_lo:[1,1,1]"
      : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
template <bool CONST_P>
__device__ __forceinline__ int fast_score_u8(const uint8_t* tile, int coff, int p) {
  const uint8_t* c = tile + coff;
  const int off[16] = {3 * p,      3 * p + 1,  2 * p + 2,  p + 3,       3,  -p + 3,
                       -2 * p + 2, -3 * p + 1, -3 * p,     -3 * p - 1, -2 * p - 2, -p - 3,
                       -3,         p - 3,      2 * p - 2,  3 * p - 1};
#if FC_SCORE_RAW
  // one base at the ring's top-left corner: every read is a non-negative
  // immediate offset when p is a compile-time constant
  // (the base offset is made opaque: hipcc would otherwise fold it back into
  // c + off[k] and add the negative offsets one by one)
  int o0 = coff - (3 * p + 3);
  if (CONST_P) __asm__ volatile("" : "+v"(o0));
  uint32_t r[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) r[k] = tile[o0 + off[k] + 3 * p + 3];
  h16x2 w3[16];
#pragma unroll
  for (int k = 0; k < 16; ++k)
    w3[k] = __builtin_bit_cast(h16x2, pk_min3_negpair(r[k], r[(k + 1) & 15], r[(k + 2) & 15]));
#else
  const _Float16 v = __builtin_bit_cast(_Float16, (uint16_t)c[0]);
  const h16x2 vv = {v, -v}, sg = {(_Float16)-1.0f, (_Float16)1.0f};
  h16x2 q[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const _Float16 ck = __builtin_bit_cast(_Float16, (uint16_t)c[off[k]]);
    const h16x2 cc = {ck, ck};
    q[k] = __builtin_elementwise_fma(cc, sg, vv);  // (v - ck, ck - v), exact
  }
  h16x2 w3[16];
#pragma unroll
  for (int k = 0; k < 16; ++k)
    w3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(q[k], q[(k + 1) & 15]),
                                          q[(k + 2) & 15]);
#endif
  h16x2 w9[16];
#pragma unroll
  for (int k = 0; k < 16; ++k)
    w9[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(w3[k], w3[(k + 3) & 15]),
                                          w3[(k + 6) & 15]);
  h16x2 m5[6];
#pragma unroll
  for (int k = 0; k < 5; ++k)
    m5[k] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(w9[3 * k], w9[3 * k + 1]),
                                          w9[3 * k + 2]);
  m5[5] = w9[15];
  const h16x2 ma = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m5[0], m5[1]), m5[2]);
  const h16x2 mb = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m5[3], m5[4]), m5[5]);
  h16x2 best = __builtin_elementwise_maximum(ma, mb);
#if FC_SCORE_RAW
  {
    const _Float16 v = __builtin_bit_cast(_Float16, (uint16_t)c[0]);
    const h16x2 vv = {v, -v};
    best = best + vv;  // (dark, bright): exact sums of subnormals
  }
#endif
  // the subnormal's bit pattern is the integer strength; negative -> 0
  const int s = (int)(short)__builtin_bit_cast(uint16_t, __builtin_fmaxf16(best.x, best.y));
  return min(max(s, 0), 255);
}

// PT > 0: the launch's LDS row pitch as a compile-time constant (every cell's
// rows at pitch PT >= fc_pitch(C)), so every ring / neighbour / row read is an
// immediate offset from one address; PT = 0: per-cell fc_pitch(C)
#ifndef FC_WPE
// waves per SIMD the register allocation must allow: 7, so that the SGPRs
// (98 without it) do not cap the kernel below its LDS limit of 27-28 waves per
// CU (SGPR budget 800 per SIMD in granules of 16, +16 per wave: 98 -> 6 waves,
// <= 96 -> 7; MI355X_MICROARCH "Residency")
#define FC_WPE 7
#endif
template <int PT>
#if FC_WPE > 0
__global__ __launch_bounds__(64 * FC_WAVES) __attribute__((amdgpu_waves_per_eu(FC_WPE)))
#else
__global__ __launch_bounds__(64 * FC_WAVES)
#endif
void k_fast_cells(
    const uint8_t* __restrict__ img0, long long img0Pitch, int img0Stride,
    const uint8_t* __restrict__ arena, long long arenaPitch, OrbPlanDesc plan,
    const OrbCellDesc* __restrict__ cells, uint32_t* __restrict__ cellKeys,
    int32_t* __restrict__ cellCount, int tileElems, int cellBeg, int cellEnd,
    int32_t* __restrict__ errFlag) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bx, img;
  xcd_swizzle(bx, img);
  // the image's status starts clean (k_octree may flag it, k_orient_desc reads it)
  // (errFlag null: the caller cleared the flags before any octree could run)
  if (errFlag && bx == 0 && threadIdx.x == 0) errFlag[img] = 0;
  uint8_t* tile = smem + wave * fc_wave_bytes(tileElems);
  uint8_t* sc = tile + tileElems;  // strengths, same byte layout as the tile
  uint16_t* queue = (uint16_t*)(sc + tileElems);
  uint16_t* corners = queue + FC_QCAP;
  uint32_t* bits = (uint32_t*)(corners + FC_CCAP);  // row y: words 2y, 2y+1
  // this wave's cells: (bx * FC_CPW + j) * FC_WAVES + wave, j < FC_CPW; the
  // next cell's ROI is loaded into registers while this one is processed
  auto cell_of = [&](int j) { return cellBeg + (bx * FC_CPW + j) * FC_WAVES + wave; };
  // ---- staging: lane r loads ROI row r, bytes [x0 - LPAD, x0 - LPAD + P)
  // of level row y0 + r, as four 16-byte loads from the 4-aligned byte at or
  // below its start (any caller stride), realigned in registers
  uint32_t raw[16], rsh = 0;
  auto issue = [&](const OrbCellDesc& q) {
    const int ql = q.level, qR = q.y1 - q.y0;
    const uint8_t* lvl;
    int pitch;
    if (ql == 0) {
      lvl = img0 + (long long)img * img0Pitch;
      pitch = img0Stride;
    } else {
      lvl = arena + (long long)img * arenaPitch + plan.lv[ql].arenaOff;
      pitch = plan.lv[ql].pitch;
    }
    const ImgRsrc im = img_rsrc(lvl, (uint32_t)((plan.lv[ql].h - 1) * pitch + plan.lv[ql].w));
    const int r = min(lane, max(qR - 1, 0));
    const uint32_t o = (uint32_t)((q.y0 + r) * pitch + q.x0 - FAST_LPAD) + im.sh;
    rsh = o & 3u;
    const uint32_t a0 = o & ~3u;
#if FC_LOAD3
    // the row's bytes 0 .. C + 4 end inside the first 48 loaded bytes unless
    // the cell is wider than 40 - rsh: the 4th 16-byte load only then (the
    // stored bytes past C + 4 are never read for an interior pixel)
    const int nLoads = (int)rsh + (q.x1 - q.x0) + FAST_LPAD > 48 ? 4 : 3;
#else
    const int nLoads = 4;
#endif
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k == 3 && nLoads < 4) break;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(im.r, (int)(a0 + 16 * k), 0, 0);
      raw[4 * k] = (uint32_t)v[0];
      raw[4 * k + 1] = (uint32_t)v[1];
      raw[4 * k + 2] = (uint32_t)v[2];
      raw[4 * k + 3] = (uint32_t)v[3];
    }
  };
  int ci = cell_of(0);
  if (ci >= cellEnd) return;
  OrbCellDesc ncd = cells[ci];
  issue(ncd);
  for (int jc = 0; jc < FC_CPW && ci < cellEnd; ++jc) {
  const OrbCellDesc cd = ncd;
  const int R = cd.y1 - cd.y0, C = cd.x1 - cd.x0;
  const long long slot = (long long)img * plan.ncells + ci;
  const bool tiny = R < 7 || C < 7;
  const int P = PT ? PT : fc_pitch(C);
  if (!tiny && lane < R) {
    const int nS = P >> 2;  // dwords per row (<= 14, host-checked): the row, no further
    uint2* dst = reinterpret_cast<uint2*>(tile + lane * P);
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (2 * k < nS)
        dst[k] = make_uint2(__builtin_amdgcn_alignbyte(raw[2 * k + 1], raw[2 * k], rsh),
                            __builtin_amdgcn_alignbyte(raw[2 * k + 2], raw[2 * k + 1], rsh));
    }
  }
#if FC_ROWMAJOR
  // strengths start at 0 over the whole map: the halo and the columns past the
  // interior are never scored, so NMS reads 0 there without bounds tests
  {
    uint4* sc16 = reinterpret_cast<uint4*>(tile + tileElems);
    for (int i = lane; i < (tileElems >> 4); i += 64) sc16[i] = make_uint4(0u, 0u, 0u, 0u);
  }
#endif
  const int ciNext = jc + 1 < FC_CPW ? cell_of(jc + 1) : cellEnd;
  if (ciNext < cellEnd) {
    ncd = cells[ciNext];
    issue(ncd);
  }
  if (tiny) {
    if (lane == 0) cellCount[slot] = 0;
    ci = ciNext;
    continue;
  }
  const int iw = C - 6, ih = R - 6;
  const int nK = (iw + 7) >> 3;  // 8-pixel groups per interior row
  const int nvLast = iw - 8 * (nK - 1);
  [[maybe_unused]] const unsigned long long outsideLast =
      nvLast >= 8 ? 0ull : (0x0101010101010101ull << (8 * nvLast));
  const int ti = min(max(plan.iniTh, 0), 255), tm = min(max(plan.minTh, 0), 255);
  // quotients q = (int)((x + 0.5) * (1 / d)) for x < 2^13, d <= 88 are exact
  // with the hardware reciprocal (<= 1 ulp): (x + 0.5) / d sits >= 0.5 / d
  // (>= 0.0057) from an integer, the reciprocal and product err < 2e-5.  An
  // IEEE division (this library's default for 1.0f / x) costs ~11 VALU each
  const float invK = __builtin_amdgcn_rcpf((float)nK), invP = __builtin_amdgcn_rcpf((float)P),
              invW = __builtin_amdgcn_rcpf((float)iw);
  wave_lds_sync();

  int nq = 0, nc = 0;  // wave-uniform queue / corner counts
  // score the queued candidates, list the corners (m > t)
  auto flush = [&](int t, bool fresh) {
    for (int j0 = 0; j0 < nq; j0 += 64) {
      const int j = j0 + lane;
      bool corner = false;
      int off = 0;
      if (j < nq) {
        off = queue[j];
        int m;
        if (fresh) {
          // phase A queues interior pixels only (fast_pass masks the columns
          // past the window), and none has a strength yet: no strength read
          m = fast_score_u8<(PT != 0)>(tile, off, P);
          sc[off] = (uint8_t)m;
        } else {
          m = sc[off];  // 0: not scored yet; phase B keeps phase-A strengths
          if (m == 0) {
            m = fast_score_u8<(PT != 0)>(tile, off, P);
            sc[off] = (uint8_t)m;
          }
        }
        corner = m > t && m >= 2;
      }
      const unsigned long long bal = __ballot(corner);
      const int pos = nc + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      if (corner && pos < FC_CCAP) corners[pos] = (uint16_t)off;
      nc += __popcll(bal);
    }
    nq = 0;
  };
  // One FAST pass at threshold t over the window: pretest, queue, strengths,
  // corners.  Lane state: its pixel group (group k of an interior row) and the
  // group's tile byte `off`, advanced by 64 groups per round with adds.
  // Invalid lanes (past the window) and the pixels past the interior in a
  // row's last group are masked out of the queue by SGPR lane masks; the
  // queue writes of lanes that do not pass go to a per-lane trash word (the
  // NMS bitmap, unused while a pass runs) instead of branching on EXEC.
  auto fast_pass = [&](int t, bool fresh) {
    h16x2 T;
    T.x = T.y = __builtin_bit_cast(_Float16, (uint16_t)(t + 1));
    const int nG = ih * nK;
#if FC_PERM
    // The queue is a set (scores, corners and the NMS bitmap do not depend on
    // its order), so lanes may take the round's 64 pixel groups in any order:
    // spread each LDS lane group's rows over the banks.
    const int pl = 4 * (int)((0xFEAB6732DC894510ull >> (4 * (lane >> 2))) & 15u) + (lane & 3);
#else
    const int pl = lane;
#endif
    const int rr0 = (int)(((float)pl + 0.5f) * invK);
    int k = pl - rr0 * nK;
    int off = (rr0 + 3) * P + 8 + 8 * k;  // byte of interior column 8k
    const int rInc = (int)(64.5f * invK), kInc = 64 - rInc * nK;  // wave-uniform, = 64 / nK
    const int dOff = rInc * P + 8 * kInc, wrapOff = P - 8 * nK;
    // trash slots in the NMS bitmap, as indices into the queue (u16) and the
    // strength map (u64 words): 4- and 8-byte lane strides
    [[maybe_unused]] const int trashQ = (int)(reinterpret_cast<uint16_t*>(bits) - queue) + 2 * lane;
    unsigned long long* const sc64 = reinterpret_cast<unsigned long long*>(sc);
    [[maybe_unused]] const int trashS = (int)(reinterpret_cast<unsigned long long*>(bits) - sc64) + lane;
    for (int g0 = 0; g0 < nG; g0 += 64) {
      const bool valid = g0 + pl < nG;
      const bool last = k == nK - 1;
      const int o = valid ? off : 3 * P + 8;  // invalid lanes read group 0 (masked below)
      {
      // bytes o-8 .. o+15 of the row, and o .. o+7 three rows down / up
      const uint2* rw = reinterpret_cast<const uint2*>(tile + o);
      const uint2 A = rw[-1], B = rw[0], Cc = rw[1];
      const uint2 Uu = *reinterpret_cast<const uint2*>(tile + o + 3 * P);  // circle 0 (y + 3)
      const uint2 Dd = *reinterpret_cast<const uint2*>(tile + o - 3 * P);  // circle 8 (y - 3)
      // f16 pairs of pixels (2i, 2i+1): v, x + 3, y + 3, y - 3, x - 3
      const uint32_t q4_0 = byte_pair(B.y, B.x, 3, 4);
      const uint32_t V[4] = {byte_pair(B.y, B.x, 0, 1), byte_pair(B.y, B.x, 2, 3),
                             byte_pair(Cc.x, B.y, 0, 1), byte_pair(Cc.x, B.y, 2, 3)};
      const uint32_t Q4[4] = {q4_0, byte_pair(Cc.x, B.y, 1, 2), byte_pair(Cc.x, B.y, 3, 4),
                              byte_pair(Cc.y, Cc.x, 1, 2)};
      const uint32_t Q0[4] = {byte_pair(Uu.y, Uu.x, 0, 1), byte_pair(Uu.y, Uu.x, 2, 3),
                              byte_pair(Uu.y, Uu.x, 4, 5), byte_pair(Uu.y, Uu.x, 6, 7)};
      const uint32_t Q8[4] = {byte_pair(Dd.y, Dd.x, 0, 1), byte_pair(Dd.y, Dd.x, 2, 3),
                              byte_pair(Dd.y, Dd.x, 4, 5), byte_pair(Dd.y, Dd.x, 6, 7)};
      const uint32_t Q12[4] = {byte_pair(A.y, A.x, 5, 6), byte_pair(B.x, A.y, 3, 4),
                               byte_pair(B.x, A.y, 5, 6), q4_0};
      uint32_t rp[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) rp[i] = pretest_pair(V[i], Q0[i], Q4[i], Q8[i], Q12[i], T);
#if !FC_ROWMAJOR
      if (fresh)  // strengths start at 0, FAST_OUTSIDE past the interior (o is a multiple of 8)
        sc64[valid ? (o >> 3) : trashS] = last ? outsideLast : 0ull;
#endif
#if FC_ROWMAJOR
      // lane-major append: lane = pixel group in row-major order, so the queue
      // (and the corner list built from it) is in cv::FAST's row-major order
      // and NMS can write the keys in place.  Pass mask: the sign bits of the
      // eight f16 results (bit 15 / 31 of rp[i] = pixels 2i / 2i+1), masked to
      // the lane's interior pixels.
      // gather the sign bytes (bytes 1, 3 of each rp[i]: pixels 0..7), move the
      // sign bits to bit 0 (pixels 0-3) / bit 4 (pixels 4-7) of each byte, and
      // collect them into bits 24..31 with one multiply (no carries: every
      // partial product lands on its own bit); a set sign bit = no pass
      const uint32_t X = __builtin_amdgcn_perm(rp[1], rp[0], 0x07050301u);
      const uint32_t Y = __builtin_amdgcn_perm(rp[3], rp[2], 0x07050301u);
      const uint32_t fails = ((X >> 7) & 0x01010101u) | ((Y >> 3) & 0x10101010u);
      uint32_t mk = ~((fails * 0x01020408u) >> 24) &
                    (valid ? (last ? (1u << nvLast) - 1u : 0xFFu) : 0u);
      const int cnt = __builtin_popcount(mk);
      int incl = wave_incl_scan(cnt);
      // opaque: otherwise hipcc forms incl - cnt from the scan's partial DPP
      // terms and keeps each as a separate v_mov_b32_dpp + v_add
      __asm__ volatile("" : "+v"(incl));
      int pos = nq + incl - cnt;
      while (mk) {
        const int j = __builtin_ctz(mk);
        mk &= mk - 1u;
        queue[pos++] = (uint16_t)(off + j);
      }
      nq += __builtin_amdgcn_readlane(incl, 63);
#else
      // pixel j of a valid lane is interior when j < nvLast or the group is not a row's last
      const unsigned long long vm = __ballot(valid), vIn = __ballot(valid && !last);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = rp[j >> 1];
        const bool sgn = (j & 1) ? ((int)w >= 0) : ((short)(w & 0xFFFFu) >= 0);
        const unsigned long long bj = __ballot(sgn) & (j < nvLast ? vm : vIn);
        const int pos = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bj >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bj, (uint32_t)nq));
        queue[lane_select(bj, pos, trashQ)] = (uint16_t)(off + j);
        nq += __popcll(bj);
      }
#endif
      }  // pretest
      k += kInc;
      off += dOff;
      if (k >= nK) {
        k -= nK;
        off += wrapOff;
      }
      if (nq > FC_QCAP - 512 || g0 + 64 >= nG) {
        wave_lds_sync();
        flush(t, fresh);
        wave_lds_sync();
      }
    }
  };
  // cell-local NMS at t into the row bitmap: a corner survives iff no
  // neighbour inside the window has nb > t && nb >= m (outside counts as 0)
  auto nms = [&](int t) {
    for (int i = lane; i < 2 * ih; i += 64) bits[i] = 0;
    wave_lds_sync();
    const bool dense = nc > FC_CCAP;
    const int nItems = dense ? ih * iw : nc;
    for (int j = lane; j < nItems; j += 64) {
      int x, y, off;
      if (dense) {
        y = (int)(((float)j + 0.5f) * invW);
        x = j - y * iw;
        off = (y + 3) * P + (x + 8);
      } else {
        off = corners[j];
        const int ry = (int)(((float)off + 0.5f) * invP);
        y = ry - 3;
        x = off - ry * P - 8;
      }
      const uint8_t* cp = sc + off;
      const int m = cp[0];
      const int r0 = cp[-P - 1], r1 = cp[-P], r2 = cp[-P + 1], r3 = cp[-1], r4 = cp[1],
                r5 = cp[P - 1], r6 = cp[P], r7 = cp[P + 1];
      if (m <= t || m < 2) continue;
      const bool L = x > 0, Rt = x < iw - 1, U = y > 0, D = y < ih - 1;
      const int nb[8] = {(U && L) ? r0 : 0, U ? r1 : 0, (U && Rt) ? r2 : 0, L ? r3 : 0,
                         Rt ? r4 : 0, (D && L) ? r5 : 0, D ? r6 : 0, (D && Rt) ? r7 : 0};
      bool ok = true;
#pragma unroll
      for (int k = 0; k < 8; ++k) ok = ok && !(nb[k] > t && nb[k] >= m);
      if (ok) atomicOr(&bits[2 * y + (x >> 5)], 1u << (x & 31));
    }
    wave_lds_sync();
  };
  // keys of the window in row-major order (lane = window row, ih <= 64)
  uint32_t* out = cellKeys + slot * plan.keyCap;
  // FC_ROWMAJOR: the corner list (or, dense, the window) is in row-major
  // order, so each survivor's key goes straight to its output position
  auto nms_emit = [&](int t) -> int {
    const bool dense = nc > FC_CCAP;
    const int nItems = dense ? ih * iw : nc;
    const uint32_t kx0 = (uint32_t)(cd.x0 + 3), ky0 = (uint32_t)(cd.y0 + 3);
    int nOut = 0;
    for (int j0 = 0; j0 < nItems; j0 += 64) {
      const int j = j0 + lane;
      bool ok = false;
      int x = 0, y = 0, m = 0;
      if (j < nItems) {
        int off;
        if (dense) {
          y = (int)(((float)j + 0.5f) * invW);
          x = j - y * iw;
          off = (y + 3) * P + (x + 8);
        } else {
          off = corners[j];
          const int ry = (int)(((float)off + 0.5f) * invP);
          y = ry - 3;
          x = off - ry * P - 8;
        }
        int oq = off - P - 1;  // 3x3 window from its top-left byte (opaque: see fast_score_u8)
        if (PT) __asm__ volatile("" : "+v"(oq));
        const uint8_t* cq = sc + oq;
        m = cq[P + 1];
        // neighbours outside the interior read 0 (the map is cleared per cell)
        const int nb[8] = {cq[0], cq[1], cq[2], cq[P], cq[P + 2], cq[2 * P], cq[2 * P + 1],
                           cq[2 * P + 2]};
        ok = m > t && m >= 2;
#pragma unroll
        for (int k = 0; k < 8; ++k) ok = ok && !(nb[k] > t && nb[k] >= m);
      }
      const unsigned long long bal = __ballot(ok);
      const int pos = nOut + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      if (ok) out[pos] = pack_key(kx0 + x, ky0 + y, m - 1);
      nOut += __popcll(bal);
    }
    return nOut;
  };
  auto compact = [&]() -> int {
    unsigned long long row = 0ull;
    if (lane < ih) {
      const uint2 w = *reinterpret_cast<const uint2*>(bits + 2 * lane);
      row = (unsigned long long)w.x | ((unsigned long long)w.y << 32);
    }
    const int cnt = __popcll(row);
    const int incl = wave_incl_scan(cnt);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    int o = incl - cnt;
    const uint8_t* srow = sc + (lane + 3) * P + 8;
    const uint32_t kx = (uint32_t)(cd.x0 + 3), ky = (uint32_t)(cd.y0 + 3 + lane);
    while (row) {
      const int x0 = __builtin_ctzll(row);
      row &= row - 1;
      const bool two = row != 0;
      const int x1 = two ? __builtin_ctzll(row) : x0;
      if (two) row &= row - 1;
      const int m0 = srow[x0], m1 = srow[x1];
      out[o] = pack_key(kx + x0, ky, m0 - 1);
      if (two) out[o + 1] = pack_key(kx + x1, ky, m1 - 1);
      o += two ? 2 : 1;
    }
    return total;
  };
  // ---- phase A at iniThFAST
#if FC_ROWMAJOR
  (void)nms;
  (void)compact;
#endif
  fast_pass(ti, true);
#if FC_ROWMAJOR
  int n = nms_emit(ti);
#else
  nms(ti);
  int n = compact();
#endif
  if (n == 0 && tm != ti) {
    // ---- phase B: no keypoint at iniThFAST -> minThFAST (:846-850)
    nc = 0;
    fast_pass(tm, false);
#if FC_ROWMAJOR
    n = nms_emit(tm);
#else
    nms(tm);
    n = compact();
#endif
  }
  if (lane == 0) cellCount[slot] = n;
  ci = ciNext;
  wave_lds_sync();  // the next cell's staging overwrites the tile
  }  // cell loop
}

// ================================================================ k_octree
// ExtractorNode::DivideNode + ORBextractor::DistributeOctTree
// (src/ORBextractor.cc:500-782), one workgroup per (level, image).
//
// The reference grows a std::list with push_front and erase, sorts split
// candidates by (size, node address) and stops mid-pass once the list holds
// N nodes.  Its list order is fully determined by creation order:
//   after a regular pass: [children in reverse creation order] ++ [untouched
//   single-key nodes in previous order]; after a final-phase pass:
//   [children in reverse creation order] ++ [surviving nodes in previous order].
// So the kernel keeps the live nodes as an array in list order plus a creation
// sequence number (the stand-in for the heap address), and
// each pass is a handful of data-parallel steps: quadrant counts by key,
// prefix sums over nodes to place children, and a key re-labelling.  A key's
// node keeps the keys in vToDistributeKeys order, so the per-node winner is the
// first key with maximal response (:763-779) = max of (response, -index).
struct OctNode {
  int16_t x0, y0, x1, y1;  // rectangle in border-relative coordinates (UL, BR)
  int cnt;                 // vKeys.size()
  int seq;                 // creation order
};

__device__ __forceinline__ int oct_quad(uint32_t key, const OctNode& n) {
  const int kx = key_x(key) - 16, ky = key_y(key) - 16;  // minBorderX = minBorderY = 16
  const int mx = n.x0 + ((n.x1 - n.x0 + 1) >> 1);        // ceil((UR.x-UL.x)/2), :502
  const int my = n.y0 + ((n.y1 - n.y0 + 1) >> 1);
  return (kx < mx ? 0 : 1) + (ky < my ? 0 : 2);  // n1, n2, n3, n4 = 0, 1, 2, 3 (:534-544)
}

__device__ __forceinline__ OctNode oct_child(const OctNode& p, int q, int cnt, int seq) {
  const int mx = p.x0 + ((p.x1 - p.x0 + 1) >> 1);
  const int my = p.y0 + ((p.y1 - p.y0 + 1) >> 1);
  OctNode c;
  c.x0 = (int16_t)((q & 1) ? mx : p.x0);
  c.x1 = (int16_t)((q & 1) ? p.x1 : mx);
  c.y0 = (int16_t)((q & 2) ? my : p.y0);
  c.y1 = (int16_t)((q & 2) ? p.y1 : my);
  c.cnt = cnt;
  c.seq = seq;
  return c;
}

// In-place chunked exclusive scan over an LDS int array of length n; returns the total.
__device__ int block_scan_array(int* a, int n, int* tmp) {
  const int T = blockDim.x, t = threadIdx.x;
  const int per = (n + T - 1) / T;
  const int b = min(t * per, n), e = min(b + per, n);
  int s = 0;
  for (int i = b; i < e; ++i) s += a[i];
  int total;
  int ex = block_excl_scan(s, tmp, &total);
  for (int i = b; i < e; ++i) {
    const int v = a[i];
    a[i] = ex;
    ex += v;
  }
  __syncthreads();
  return total;
}

// Two in-place chunked exclusive scans (a[0..na), b[0..nb)) plus the block
// sum of one value per thread, sharing one round of barriers (four, against
// eleven for three separate scans).  tmp: >= 51 ints of LDS.  Must be called
// by all threads; the arrays' writers need no barrier before the call.
__device__ void block_scan2(int* a, int na, int* b, int nb, int extra, int* tmp, int* totA,
                            int* totB, int* totX) {
  const int T = blockDim.x, t = threadIdx.x;
  const int pa = (na + T - 1) / T, pb = (nb + T - 1) / T;
  const int ba = min(t * pa, na), ea = min(ba + pa, na);
  const int bb = min(t * pb, nb), eb = min(bb + pb, nb);
  __syncthreads();
  int sa = 0, sb = 0;
  for (int i = ba; i < ea; ++i) sa += a[i];
  for (int i = bb; i < eb; ++i) sb += b[i];
  const int l = lane_id(), w = t >> 6, nw = (T + 63) >> 6;
  const int ia = wave_incl_scan(sa), ib = wave_incl_scan(sb), ix = wave_incl_scan(extra);
  if (l == 63) {
    tmp[w] = ia;
    tmp[16 + w] = ib;
    tmp[32 + w] = ix;
  }
  __syncthreads();
  if (t < 3) {
    int acc = 0;
    for (int i = 0; i < nw; ++i) {
      const int v = tmp[16 * t + i];
      tmp[16 * t + i] = acc;
      acc += v;
    }
    tmp[48 + t] = acc;
  }
  __syncthreads();
  int xa = tmp[w] + ia - sa, xb = tmp[16 + w] + ib - sb;
  *totA = tmp[48];
  *totB = tmp[49];
  *totX = tmp[50];
  for (int i = ba; i < ea; ++i) {
    const int v = a[i];
    a[i] = xa;
    xa += v;
  }
  for (int i = bb; i < eb; ++i) {
    const int v = b[i];
    b[i] = xb;
    xb += v;
  }
  __syncthreads();
}

__device__ void block_bitonic_desc(unsigned long long* v, int n2) {
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n2; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = v[i], b = v[ixj];
          const bool descBlock = (i & k) == 0;
          if (descBlock ? (a < b) : (a > b)) {
            v[i] = b;
            v[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

#define OCT_RANK_MAX 512
// Rank up to OCT_RANK_MAX distinct keys by counting (every thread scans the keys
// as LDS broadcasts; RQ keys per thread), then scatter them sorted descending.
template <int RQ>
__device__ __forceinline__ void oct_rank_by_count(unsigned long long* sortBuf, int ncand, int t, int T) {
  unsigned long long mine[RQ];
  int rank[RQ];
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int j = t + q * T;
    mine[q] = j < ncand ? sortBuf[j] : 0ull;
    rank[q] = 0;
  }
  for (int i = 0; i < ncand; ++i) {
    const unsigned long long k = sortBuf[i];
#pragma unroll
    for (int q = 0; q < RQ; ++q) rank[q] += k > mine[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < RQ; ++q)
    if (t + q * T < ncand) sortBuf[rank[q]] = mine[q];
  __syncthreads();
}

#define OCT_MAX_PASSES 512
#define OCT_REG_KEYS 8  // keys per thread held in registers (n <= 8 x 512), small batches
#ifndef OCT_BATCH_THREADS
#define OCT_BATCH_THREADS 256  // workgroup of the batch octree (A/B: 128)
#endif
#ifndef OCT_REG_THREADS
#define OCT_REG_THREADS 512  // workgroup of the register-key octree (calls of <= 16 frames)
#endif

template <bool REG, bool GNODES>
__global__ __launch_bounds__(512) void k_octree(
    OrbPlanDesc plan, const int32_t* __restrict__ cellCount, const uint32_t* __restrict__ cellKeys,
    uint32_t* __restrict__ gKeys, uint16_t* __restrict__ gNid, int ldsKeyCap, int nodeCapMax,
    int maxCellsPerLevel, uint32_t* __restrict__ outKeys, int32_t* __restrict__ outCount,
    int32_t* __restrict__ errFlag, int levelBeg, int maxPasses, unsigned char* __restrict__ gNodes,
    long long nodeStride) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int tmp[52];
  __shared__ int sh[8];
  // grid (images, levels levelBeg..): the dispatcher walks x first, so every
  // image's lowest level (the most keys, the longest workgroups) starts before
  // the next, and the short upper levels fill the tail
  const int l = levelBeg + blockIdx.y, img = blockIdx.x, T = blockDim.x, t = threadIdx.x;
  const OrbLevelDesc& L = plan.lv[l];
  const int NC = nodeCapMax;
  int n2 = 1;
  while (n2 < NC) n2 <<= 1;
  // ---- node tables: LDS carve (all offsets multiples of 16), or, for
  // feature counts whose tables outgrow a CU's LDS, the same carve in a global
  // scratch slice per (image, level) (one workgroup's barriers order it; only
  // the keys stay in LDS then)
  // (GNODES is a template parameter so that the LDS build keeps ds_*
  // instructions: a pointer that may be either would compile to flat ones)
  // (the slice is indexed by the absolute level, so launches over disjoint
  // level ranges of one batch could run concurrently)
  unsigned char* p = GNODES ? gNodes + ((long long)img * plan.nlevels + l) * nodeStride : smem;
  unsigned long long* sortBuf = (unsigned long long*)p; p += (size_t)n2 * 8;
  OctNode* A = (OctNode*)p; p += (size_t)NC * sizeof(OctNode);
  OctNode* B = (OctNode*)p; p += (size_t)NC * sizeof(OctNode);
  int* q4 = (int*)p; p += (size_t)NC * 16;       // quadrant counts, then child indices
  int* g0 = (int*)p; p += (size_t)NC * 4;
  int* g1 = (int*)p; p += (size_t)NC * 4;
  int* g2 = (int*)p; p += (size_t)NC * 4;
  int* rk = (int*)p; p += (size_t)NC * 4;
  int* cellBase = (int*)p; p += (size_t)((maxCellsPerLevel + 3) & ~3) * 4;
  if (GNODES) p = smem;
  uint32_t* Klds = (uint32_t*)p; p += (size_t)ldsKeyCap * 4;
  uint16_t* Nlds = (uint16_t*)p;

  const int cb = L.cellBeg, nc = L.cellEnd - L.cellBeg;
  const long long cellSlot0 = (long long)img * plan.ncells + cb;
  for (int i = t; i < nc; i += T) cellBase[i] = cellCount[cellSlot0 + i];
  __syncthreads();
  const int n = block_scan_array(cellBase, nc, tmp);
  uint32_t* K;
  uint16_t* NID;
  if (n <= ldsKeyCap) {
    K = Klds;
    NID = Nlds;
  } else {
    K = gKeys + cellSlot0 * plan.keyCap;  // this level's slot range, reused compacted
    NID = gNid + cellSlot0 * plan.keyCap;
  }
  // n < 2^24 (x, y < 4096): node labels NID are node indices (< nodeCap <= 65535),
  // the final-phase sort key packs (size: 24 bits, creation order: 24 bits, node: 16 bits)
  errFlag += img;  // per-image status (read back through the image's count)
  for (int c = t; c < nc; c += T) {
    const int cnt = cellCount[cellSlot0 + c], base = cellBase[c];
    const uint32_t* src = cellKeys + (cellSlot0 + c) * plan.keyCap;
    for (int i = 0; i < cnt; ++i) K[base + i] = src[i];
  }
  // REG (a frame or two per call, one workgroup per level): each thread's keys
  // k = t, t + T, ... live in registers (key and node id) for the whole
  // distribution when the level has at most OCT_REG_KEYS * T of them: a pass's
  // per-key steps are then independent register work with only the node
  // lookups in LDS, instead of dependent LDS round trips per key.  Batches keep
  // K / NID in memory: the registers would cost them occupancy (6 -> 4 waves
  // per SIMD, 0.129 -> 0.167 ms per 512 frames).
  const bool inReg = REG && n <= OCT_REG_KEYS * T;
  uint32_t kr[OCT_REG_KEYS];
  int nr[OCT_REG_KEYS];
  auto each_key = [&](auto&& f) {
    if (inReg) {
#pragma unroll
      for (int i = 0; i < OCT_REG_KEYS; ++i) {
        const int k = t + i * T;
        if (k < n) f(kr[i], nr[i], k);
      }
    } else {
      for (int k = t; k < n; k += T) {
        const uint32_t key = K[k];
        int nid = NID[k];
        f(key, nid, k);
        NID[k] = (uint16_t)nid;
      }
    }
  };
  __syncthreads();  // K complete
  if (inReg) {
#pragma unroll
    for (int i = 0; i < OCT_REG_KEYS; ++i) {
      const int k = t + i * T;
      kr[i] = k < n ? K[k] : 0u;
      nr[i] = 0;
    }
  }
  // ---- roots (src/ORBextractor.cc:562-604)
  const int nIni = L.nIni;
  const float hX = L.hX;
  for (int i = t; i < nIni; i += T) g0[i] = 0;
  __syncthreads();
  each_key([&](uint32_t key, int& nid, int) {
    const float xr = (float)(key_x(key) - 16);
    const int r = min((int)__fdiv_rn(xr, hX), nIni - 1);  // vpIniNodes[kp.pt.x/hX]
    nid = r;
    atomicAdd(&g0[r], 1);
  });
  __syncthreads();
  if (t == 0) {
    int a = 0;
    for (int i = 0; i < nIni; ++i) {
      g1[i] = a;
      if (g0[i] > 0) {
        OctNode nd;
        nd.x0 = (int16_t)(int)(hX * (float)i);
        nd.x1 = (int16_t)(int)(hX * (float)(i + 1));
        nd.y0 = 0;
        nd.y1 = (int16_t)L.Hr;
        nd.cnt = g0[i];
        nd.seq = i;
        A[a++] = nd;
      }
    }
    sh[0] = a;
  }
  __syncthreads();
  each_key([&](uint32_t, int& nid, int) { nid = g1[nid]; });
  int alive = sh[0];
  const int N = L.quota;
  int seqNext = nIni;
  bool finalPhase = false;
  int pass = 0;
  __syncthreads();
  for (; pass < maxPasses; ++pass) {
    const int prev = alive;
    if (!finalPhase) {
      // ================= regular pass: divide every node with > 1 key (:625-684)
      for (int i = t; i < alive * 4; i += T) q4[i] = 0;
      __syncthreads();
      each_key([&](uint32_t key, int& nid, int) {
        const OctNode nd = A[nid];
        if (nd.cnt > 1) atomicAdd(&q4[nid * 4 + oct_quad(key, nd)], 1);
      });
      __syncthreads();
      int nteLocal = 0;
      for (int a = t; a < alive; a += T) {
        int nce = 0;
        if (A[a].cnt > 1) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = q4[a * 4 + q];
            nce += c > 0;
            nteLocal += c > 1;
          }
        }
        g0[a] = nce;
        g1[a] = A[a].cnt > 1 ? 0 : 1;
      }
      int nToExpand, S, NM;
      block_scan2(g0, alive, g1, alive, nteLocal, tmp, &S, &NM, &nToExpand);
      if (S + NM > NC) {
        if (t == 0) atomicOr(errFlag, 2);
        break;
      }
      for (int a = t; a < alive; a += T) {
        const OctNode nd = A[a];
        if (nd.cnt > 1) {
          int pos = g0[a];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = q4[a * 4 + q];
            if (c > 0) {
              const int ni = S - 1 - pos;
              B[ni] = oct_child(nd, q, c, seqNext + pos);
              q4[a * 4 + q] = ni;
              ++pos;
            }
          }
        } else {
          const int ni = S + g1[a];
          B[ni] = nd;
          q4[a * 4] = ni;
        }
      }
      __syncthreads();
      each_key([&](uint32_t key, int& nid, int) {
        const OctNode nd = A[nid];
        nid = q4[nid * 4 + (nd.cnt > 1 ? oct_quad(key, nd) : 0)];
      });
      __syncthreads();
      OctNode* sw = A; A = B; B = sw;
      alive = S + NM;
      seqNext += S;
      if (alive >= N || alive == prev) break;                 // :688-691
      if (alive + nToExpand * 3 > N) finalPhase = true;      // :692
    } else {
      // ================= final phase pass (:695-756)
      if (seqNext >= (1 << 24)) {  // creation order no longer fits the sort key (24 bits)
        if (t == 0) atomicOr(errFlag, 8);
        break;
      }
      for (int a = t; a < alive; a += T) g0[a] = A[a].cnt > 1 ? 1 : 0;
      __syncthreads();
      const int ncand = block_scan_array(g0, alive, tmp);
      if (ncand == 0) break;  // nothing to divide: size == prevSize
      int m2 = 1;
      while (m2 < ncand) m2 <<= 1;
      for (int i = t; i < m2; i += T) sortBuf[i] = 0ull;
      __syncthreads();
      for (int a = t; a < alive; a += T) {
        const OctNode nd = A[a];
        if (nd.cnt > 1)  // sort key (size, creation order); node index rides in the low bits
          sortBuf[g0[a]] = ((unsigned long long)nd.cnt << 40) |
                           ((unsigned long long)(uint32_t)nd.seq << 16) | (unsigned)a;
        q4[a * 4 + 0] = q4[a * 4 + 1] = q4[a * 4 + 2] = q4[a * 4 + 3] = 0;
        rk[a] = 0x7fffffff;
      }
      __syncthreads();
      // largest (size, seq) first == reverse of std::sort.  Keys are distinct
      // (creation order is unique), so up to OCT_RANK_MAX candidates are ranked
      // by counting (every thread scans the keys as LDS broadcasts: two
      // barriers) instead of the bitonic network's log^2 barrier steps.
      if (ncand <= OCT_RANK_MAX) {
        // (OCT_RANK_MAX / T candidates per thread: workgroups of 256 or 512)
        if (T >= OCT_RANK_MAX)
          oct_rank_by_count<1>(sortBuf, ncand, t, T);
        else if (T >= 256)
          oct_rank_by_count<OCT_RANK_MAX / 256>(sortBuf, ncand, t, T);
        else
          oct_rank_by_count<OCT_RANK_MAX / 128>(sortBuf, ncand, t, T);
      } else {
        block_bitonic_desc(sortBuf, m2);
      }
      for (int j = t; j < ncand; j += T) rk[(int)(sortBuf[j] & 0xFFFF)] = j;
      each_key([&](uint32_t key, int& nid, int) {
        const OctNode nd = A[nid];
        if (nd.cnt > 1) atomicAdd(&q4[nid * 4 + oct_quad(key, nd)], 1);
      });
      if (t == 0) sh[1] = ncand - 1;
      __syncthreads();
      // node j in sorted order adds (non-empty children - 1) nodes; stop after
      // the first division that brings the list to >= N (:749-750)
      for (int j = t; j < ncand; j += T) {
        const int a = (int)(sortBuf[j] & 0xFFFF);
        int nce = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) nce += q4[a * 4 + q] > 0;
        g1[j] = nce;
        g2[j] = nce - 1;
      }
      __syncthreads();
      block_scan_array(g2, ncand, tmp);  // exclusive
      for (int j = t; j < ncand; j += T)
        if (alive + g2[j] + (g1[j] - 1) >= N) atomicMin(&sh[1], j);
      __syncthreads();
      const int jstop = sh[1];
      for (int j = t; j < ncand; j += T)
        if (j > jstop) g1[j] = 0;
      for (int a = t; a < alive; a += T) g2[a] = (rk[a] <= jstop) ? 0 : 1;
      // child base per divided node, position of each kept node
      int S, keep, unused;
      block_scan2(g1, ncand, g2, alive, 0, tmp, &S, &keep, &unused);
      if (S + keep > NC) {
        if (t == 0) atomicOr(errFlag, 2);
        break;
      }
      for (int a = t; a < alive; a += T) {
        const OctNode nd = A[a];
        const int j = rk[a];
        if (j <= jstop) {
          int pos = g1[j];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = q4[a * 4 + q];
            if (c > 0) {
              const int ni = S - 1 - pos;
              B[ni] = oct_child(nd, q, c, seqNext + pos);
              q4[a * 4 + q] = ni;
              ++pos;
            }
          }
        } else {
          const int ni = S + g2[a];
          B[ni] = nd;
          q4[a * 4] = ni;
        }
      }
      __syncthreads();
      each_key([&](uint32_t key, int& nid, int) {
        const OctNode nd = A[nid];
        nid = q4[nid * 4 + (rk[nid] <= jstop ? oct_quad(key, nd) : 0)];
      });
      __syncthreads();
      OctNode* sw = A; A = B; B = sw;
      alive = S + keep;
      seqNext += S;
      if (alive >= N || alive == prev) break;  // :753-754
    }
  }
  if (pass >= maxPasses && t == 0) atomicOr(errFlag, 4);
  // ---- retain the best key of each node (:760-779)
  uint32_t* best = (uint32_t*)g0;
  for (int a = t; a < alive; a += T) best[a] = 0u;
  __syncthreads();
  each_key([&](uint32_t key, int& nid, int k) {
    atomicMax(&best[nid], ((uint32_t)key_s(key) << 24) | (uint32_t)(0xFFFFFF - k));
  });
  __syncthreads();
  uint32_t* out = outKeys + (long long)img * plan.slotsPerImage + L.outOff;
  for (int a = t; a < alive; a += T) out[a] = K[0xFFFFFF - (int)(best[a] & 0xFFFFFF)];
  if (t == 0) outCount[img * plan.nlevels + l] = alive;
}

// ============================================================ k_blur_levels
// GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) of every level of every
// image (src/ORBextractor.cc:1143-1145), 8U integer kernel [18,34,49,55,49,34,18]
// (SURVEY.md Appendix A.3).  One workgroup per 64x16 output tile (tiles of all
// levels flattened into one launch); the 70x22 source tile with reflect-101
// borders is staged in LDS, the row pass is kept as exact u16 sums.
__constant__ int8_t c_pattern[2 * ORB_PATTERN_POINTS];
#define ORB_PATCH_DW 12  // LDS row pitch (dwords) of the staged 37 x 37 descriptor patch
__constant__ int c_umax[16];
// IC_Angle byte masks: row v+15 (v in [-15, 15]), dword k of the 32 bytes at
// columns -16..15: 0xFF where |u| <= umax[|v|] (built from umax on upload)
__constant__ uint32_t c_icmask[32][8];

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

#define BLUR_SH (ORB_BLUR_TH + 6)  // staged source rows y0-3 .. y0+TH+2
#define BLUR_WROW (ORB_BLUR_TW / 4 + 2)  // dwords per staged row: bytes x0-4 .. x0+TW+3
#define BLUR_RP2 (ORB_BLUR_TW + 4)       // row-pass pitch in dwords (one column per dword), padded


__global__ __launch_bounds__(256) void k_blur_levels(
    const uint8_t* __restrict__ img0, long long img0Pitch, int img0Stride,
    const uint8_t* __restrict__ arena, long long arenaPitch, OrbPlanDesc plan,
    const OrbTileDesc* __restrict__ tiles, uint8_t* __restrict__ blur, long long blurPitch,
    int nImg) {
  // Source tile staged as aligned dwords, byte b of a row = level column
  // x0-4+b (realigned from any stride); every LDS access is an aligned dword
  // or 8 bytes (unaligned sub-dword LDS reads are replayed by the hardware).
  __shared__ __attribute__((aligned(16))) uint32_t raw[BLUR_SH][BLUR_WROW + 1];
  // row-pass sums, two staged rows per dword: rowp2[p][c] = sum(2p, c) | sum(2p+1, c) << 16
  __shared__ __attribute__((aligned(16))) uint32_t rowp2[BLUR_SH / 2][BLUR_RP2];
  const int tid = threadIdx.x;
  const OrbTileDesc td = tiles[blockIdx.x];
  const int l = td.level;
  const OrbLevelDesc& L = plan.lv[l];
  // A workgroup blurs one tile of images blockIdx.y, + gridDim.y, ...; the
  // next image's source rows are loaded into registers while the current one
  // is computed (TilePrefetch), so its HBM round trip overlaps this image's work.
  // Staging: rows outside the level are reflected (REFLECT_101) when
  // addressed; columns are loaded with the dword start clamped into the row,
  // and the few bytes a border tile needs outside [0, w) are patched from
  // their reflected columns afterwards.
  const int colA = td.x0 - 4;  // level column of staged byte 0
  // rows outside the level only for the first / last tile row (uniform test)
  const bool rowsInside = td.y0 >= 3 && td.y0 + BLUR_SH - 3 <= L.h;
  auto level_of = [&](int im, int* pitch) -> const uint8_t* {
    if (l == 0) {
      *pitch = img0Stride;
      return img0 + (long long)im * img0Pitch;
    }
    *pitch = L.pitch;
    return arena + (long long)im * arenaPitch + L.arenaOff;
  };
  constexpr int NQ = (BLUR_SH * BLUR_WROW + 255) / 256;
  TilePrefetch<NQ> pf;
  const uint32_t magic = div_magic(BLUR_WROW);
  // Staged element q of this thread sits at the same offset in every image of
  // the tile: row (reflected on border tiles) x pitch + dword start clamped
  // into the row (4-aligned on aligned levels), computed once.  Level 0 is
  // staged as unaligned unless every image base and row start is 4-aligned.
  int pitch0;
  level_of(0, &pitch0);
  const bool alignedAll =
      l > 0 || ((img0Stride & 3) == 0 && (img0Pitch & 3) == 0 && (((uintptr_t)img0) & 3) == 0);
  const int cmax = alignedAll ? ((L.w - 1) & ~3) : L.w - 1;
  uint32_t eoff[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t i = (uint32_t)min(q * 256 + tid, BLUR_SH * BLUR_WROW - 1);
    const int r = (int)__umulhi(i << 1, magic), c = (int)i - r * BLUR_WROW;
    const int y = td.y0 - 3 + r;
    eoff[q] = (uint32_t)((rowsInside ? y : reflect101(y, L.h)) * pitch0 + min(max(colA + 4 * c, 0), cmax));
  }
  auto issue = [&](int im) {
    int pitch;
    const uint8_t* lvl = level_of(im, &pitch);
    pf.issue(img_rsrc(lvl, (uint32_t)((L.h - 1) * pitch + L.w)), alignedAll, eoff);
  };
  int img = blockIdx.y;
  if (img >= nImg) return;
  issue(img);
  for (; img < nImg; img += gridDim.y) {
  // raw is free: the previous image's row pass ended before its second barrier
  pf.commit(&raw[0][0], BLUR_WROW + 1, BLUR_SH, BLUR_WROW, magic);
  if (img + (int)gridDim.y < nImg) issue(img + gridDim.y);
  const bool leftB = colA < 0, rightB = td.x0 + ORB_BLUR_TW + 3 > L.w;
  if (leftB || rightB) {  // uniform per workgroup
    __syncthreads();
    uint8_t* rb = reinterpret_cast<uint8_t*>(&raw[0][0]);
    constexpr int RB = (BLUR_WROW + 1) * 4;  // staged row pitch in bytes
    // byte (r, b) holds column colA + b; fix columns -4..-1 and w..w+2 (the
    // only out-of-range columns an in-range output reads)
    for (int i = tid; i < BLUR_SH * 7; i += 256) {
      const int r = i / 7, j = i - r * 7;
      const int x = j < 4 ? -4 + j : L.w + (j - 4);
      const int b = x - colA;
      if (b >= 0 && b < 4 * BLUR_WROW) {
        const int bs = reflect101(x, L.w) - colA;
        rb[r * RB + b] = (bs >= 0 && bs < 4 * BLUR_WROW) ? rb[r * RB + bs] : 0;
      }
    }
  }
  __syncthreads();
  // Integer 7-tap kernel [18,34,49,55,49,34,18] (sums to 257 per axis).  Row
  // pass: the 7-tap sum at byte offset s of a dword triple (w0, w1, w2) is
  // v_dot4_u32_u8 of each dword with the kernel shifted to that offset (2 or 3
  // dot4, no byte realignment); column pass: four v_dot2_u32_u16 over row pairs.
  constexpr uint32_t k0 = 18, k1 = 34, k2 = 49, k3 = 55, k4 = 49, k5 = 34, k6 = 18;
  constexpr uint32_t S0a = (k0 << 8) | (k1 << 16) | (k2 << 24), S0b = k3 | (k4 << 8) | (k5 << 16) | (k6 << 24);
  constexpr uint32_t S1a = (k0 << 16) | (k1 << 24), S1b = k2 | (k3 << 8) | (k4 << 16) | (k5 << 24), S1c = k6;
  constexpr uint32_t S2a = k0 << 24, S2b = k1 | (k2 << 8) | (k3 << 16) | (k4 << 24), S2c = k5 | (k6 << 8);
  constexpr uint32_t S3b = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24), S3c = k4 | (k5 << 8) | (k6 << 16);
  // row pass: task (row pair p, group g) -> sums of columns 4g..4g+3 of staged
  // rows 2p, 2p+1 (output column x0+4g+i reads staged bytes 4g+i+1 .. 4g+i+7)
  constexpr int G = ORB_BLUR_TW / 4;
  for (int id = tid; id < (BLUR_SH / 2) * G; id += 256) {
    const int pr = id / G, g = id - pr * G;
    uint32_t o[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t* rw = raw[2 * pr + h] + g;
      const uint32_t w0 = rw[0], w1 = rw[1], w2 = rw[2];
      o[h][0] = __builtin_amdgcn_udot4(w0, S0a, __builtin_amdgcn_udot4(w1, S0b, 0u, false), false);
      o[h][1] = __builtin_amdgcn_udot4(w0, S1a, __builtin_amdgcn_udot4(w1, S1b,
                                       __builtin_amdgcn_udot4(w2, S1c, 0u, false), false), false);
      o[h][2] = __builtin_amdgcn_udot4(w0, S2a, __builtin_amdgcn_udot4(w1, S2b,
                                       __builtin_amdgcn_udot4(w2, S2c, 0u, false), false), false);
      o[h][3] = __builtin_amdgcn_udot4(w1, S3b, __builtin_amdgcn_udot4(w2, S3c, 0u, false), false);
    }
    uint4 pk;
    pk.x = o[0][0] | (o[1][0] << 16);
    pk.y = o[0][1] | (o[1][1] << 16);
    pk.z = o[0][2] | (o[1][2] << 16);
    pk.w = o[0][3] | (o[1][3] << 16);
    *reinterpret_cast<uint4*>(&rowp2[pr][4 * g]) = pk;
  }
  __syncthreads();
  // column pass: thread -> columns 4qx..4qx+3 x output rows 2p, 2p+1 for
  // p = qp and qp + 8; output row y reads staged rows y..y+6 = pairs
  // y/2 .. y/2+3 with weights (k0,k1)(k2,k3)(k4,k5)(k6,0) for even y and
  // (0,k0)(k1,k2)(k3,k4)(k5,k6) for odd y.
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 E0 = {18, 34}, E1 = {49, 55}, E2 = {49, 34}, E3 = {18, 0};
  const u16x2 O0 = {0, 18}, O1 = {34, 49}, O2 = {55, 49}, O3 = {34, 18};
  const int qx = tid & (G - 1), qp = tid / G;
  uint8_t* dst = blur + (long long)img * blurPitch + L.blurOff;
  const int x = td.x0 + 4 * qx;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int pp = qp + 8 * half;
    uint4 pv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) pv[k] = *reinterpret_cast<const uint4*>(&rowp2[pp + k][4 * qx]);
    uint32_t packedE = 0, packedO = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t se = 0, so = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t w = c == 0 ? pv[k].x : (c == 1 ? pv[k].y : (c == 2 ? pv[k].z : pv[k].w));
        const u16x2 v = __builtin_bit_cast(u16x2, w);
        se = __builtin_amdgcn_udot2(v, k == 0 ? E0 : (k == 1 ? E1 : (k == 2 ? E2 : E3)), se, false);
        so = __builtin_amdgcn_udot2(v, k == 0 ? O0 : (k == 1 ? O1 : (k == 2 ? O2 : O3)), so, false);
      }
      // the pinned kernel sums to 257 per axis: saturate (row sums <= 255*257 fit u16)
      int ve = min((int)((se + (1u << 15)) >> 16), 255), vo = min((int)((so + (1u << 15)) >> 16), 255);
      __asm__ volatile("" : "+v"(ve), "+v"(vo));  // see k_pyr_resize: keep the byte pack opaque
      packedE |= (uint32_t)ve << (8 * c);
      packedO |= (uint32_t)vo << (8 * c);
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int y = td.y0 + 2 * pp + rr;
      if (y >= L.h || x >= L.w) continue;
      const uint32_t packed = rr ? packedO : packedE;
      uint8_t* o = dst + (long long)y * L.blurPitch + x;
      if (x + 4 <= L.w) {
        *reinterpret_cast<uint32_t*>(o) = packed;  // blurPitch % 128 == 0, x % 4 == 0
      } else {
        for (int c = 0; x + c < L.w; ++c) o[c] = (uint8_t)(packed >> (8 * c));
      }
    }
  }
  }  // image loop
}

// =========================================================== k_orient_desc
// Two keypoints per wave: half-wave h (lanes 32h .. 32h+31) takes slot 2p+h
// of the wave's slot pair p.  Levels own even-sized slot ranges (the planner
// rounds nodeCap up to even), so both keypoints of a wave are on one level and
// the level's buffer resources stay wave-uniform; everything per keypoint
// (IC moments, angle, sincos, 256 tests) runs once per half-wave, so the
// per-keypoint scalar chain (fastAtan2, the pinned double sincos, address
// setup, epilogue) is issued once for two keypoints.
//   IC_Angle (src/ORBextractor.cc:77-113) on the un-blurred level: lane hl
//   takes row v = hl - 15 (hl < 31) and both 16-byte halves of its 32 columns
//   at -16..15; integer moments reduced across the half-wave.
//   rBRIEF (:119-164) on the blurred level: lane hl evaluates tests
//   hl + 32k (k < 8); ballot k holds tests 32k .. 32k+31 of both keypoints.
// Sum over the 32 lanes of each half-wave: quad, 8- and 16-lane steps as DPP
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: each pairs a
// lane with one holding the other half of its group), then lane ^ 16 by one
// ds_swizzle in bitmask mode (and 0x1F, xor 0x10) -- one LDS-path op where
// __shfl_xor would take five ds_bpermute round trips.
__device__ __forceinline__ int half_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);
  v += __builtin_amdgcn_ds_swizzle(v, 0x401F);
  return v;
}

// ===================================================== k_orient_desc (fused)
// IC_Angle + GaussianBlur 7x7 + rBRIEF + rescale in one pass, two keypoints
// per wave (half-wave per keypoint, slot pairing as described above).
// The blurred level is never materialised: descriptors sample only the 37 x 37
// blurred patch around a keypoint (rotated pattern within +-18 px), and that
// patch depends only on the 43 x 43 raw window around it, so each keypoint
// blurs its own window (src/ORBextractor.cc:1141-1151 blurs the whole level,
// then samples it; the bytes sampled are identical).
//   staging: lane hl < 22 loads raw rows cy-21+2hl and cy-21+2hl+1 (three
//     16-byte loads each) and realigns them in registers so byte b is column
//     cx-21+b; rows outside the level are reflected (REFLECT_101) when
//     addressed, columns outside it patched bytewise from their reflected
//     columns through LDS (keypoints sit >= 19 px inside, so a window
//     overhangs by at most 2 columns / rows per side).
//   IC_Angle (:77-113) from the rows in registers (rows 6..36).
//   row pass, from registers: the lane's two rows, ten 4-column groups of
//     u16 row sums (2.5 v_dot4 per sum), packed (row 2p | row 2p+1 << 16) and
//     stored as row-sum pair p in LDS (the only LDS the kernel uses).
//   rBRIEF (:119-164): each of the 512 samples takes the column pass of its
//     own pixel -- four v_dot2 over the packed row-sum pairs (the weights of
//     the row's parity), (sum + 2^15) >> 16 saturated -- instead of a column
//     pass over the whole 37 x 37 patch (about a third of its pixels are
//     sampled); ballots.
#ifndef DESC_RS_DW
#define DESC_RS_DW 40    // row-sum pair row pitch (dwords): 10 groups of 4 columns
#endif
#define DESC_RS_PAIRS 22 // 43 rows + the unused odd row of the last pair
struct DescWaveLds {
  uint32_t rsp[2][DESC_RS_PAIRS][DESC_RS_DW];
};

#ifndef DESC_PPW
#define DESC_PPW 4  // slot pairs per wave (software-pipelined: the next pair's window loads overlap this one)
#endif
#ifndef DESC_MIN_WAVES
#define DESC_MIN_WAVES 0  // __launch_bounds__ minimum waves per SIMD (A/B knob: 5 -> <= 96 VGPRs)
#endif
#if DESC_MIN_WAVES > 0
#define DESC_LAUNCH_BOUNDS __launch_bounds__(256, DESC_MIN_WAVES)
#else
#define DESC_LAUNCH_BOUNDS __launch_bounds__(256)
#endif
#ifndef DESC_LDS_TABLES
#define DESC_LDS_TABLES 1  // rBRIEF pattern floats and column weights in LDS (k_orient_desc)
#endif
#ifndef DESC_MAGIC_ROUND
#define DESC_MAGIC_ROUND 1  // rBRIEF sample coordinates rounded by the 1.5 * 2^23 adder
#endif
#ifndef DESC_ROW37
#define DESC_ROW37 1     // row pass stops at column 36, the last one a sample reaches
#endif
#ifndef DESC_SMALL_CT
#define DESC_SMALL_CT 1   // one-pair calls take k_orient_desc<1> (compile-time count), else <0>
#endif
// Attribution builds (phase stubs) and the measured-slower variants (LDS-DMA
// window staging, double-buffered rows, MFMA row pass, packed rotation) are
// patches against this file: tools/attribution/.

template <int PPW>
__global__ DESC_LAUNCH_BOUNDS void k_orient_desc(
    const uint8_t* __restrict__ img0, long long img0Pitch, int img0Stride,
    const uint8_t* __restrict__ arena, long long arenaPitch, OrbPlanDesc plan,
    const uint32_t* __restrict__ outKeys, const int32_t* __restrict__ outCount,
    const int32_t* __restrict__ errFlag, orb_keypoint_t* __restrict__ kps,
    uint8_t* __restrict__ desc, int capacity, int32_t* __restrict__ counts, int ppwRt,
    int slotBeg, int slotEnd) {
  // PPW > 0: compile-time pairs per wave (<4> batches, <1> one-pair calls);
  // PPW == 0: ppwRt
  const int ppw = PPW ? PPW : ppwRt;
  __shared__ __attribute__((aligned(16))) DescWaveLds sm[4];
#if DESC_LDS_TABLES
  // per workgroup: the rBRIEF pattern as floats (one ds_read_b128 per test
  // pair of points instead of a constant-memory load and four conversions),
  // and the column-pass weights of both row parities (one ds_read_b128 per
  // sample instead of four selects)
  __shared__ __attribute__((aligned(16))) float4 sPat[ORB_PATTERN_POINTS / 2];
  __shared__ __attribute__((aligned(16))) uint4 sW[2];
  {
    const int t = threadIdx.x;  // 256 threads, 256 tests
    sPat[t] = make_float4((float)c_pattern[4 * t], (float)c_pattern[4 * t + 1],
                          (float)c_pattern[4 * t + 2], (float)c_pattern[4 * t + 3]);
    if (t < 2)  // even rows: (18,34) (49,55) (49,34) (18,0); odd: (0,18) (34,49) (55,49) (34,18)
      sW[t] = t == 0 ? make_uint4(18u | 34u << 16, 49u | 55u << 16, 49u | 34u << 16, 18u)
                     : make_uint4(18u << 16, 34u | 49u << 16, 55u | 49u << 16, 34u | 18u << 16);
    __syncthreads();  // before any wave can leave early
  }
#endif
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int half = lane >> 5, hl = lane & 31;
  int bx, img;
  xcd_swizzle(bx, img);
  const int32_t* cnts = outCount + img * plan.nlevels;
  // the launch whose slot range ends the image writes its count (a launch over
  // the first levels runs beside the rest; its caller orders the last after it)
  if (bx == 0 && threadIdx.x == 0 && slotEnd == plan.slotsPerImage) {
    int tot = 0;
    for (int i = 0; i < plan.nlevels; ++i) tot += cnts[i];
    counts[img] = errFlag[img] ? (int32_t)ORB_EDEVICE : tot;  // failed image: negative count
  }
  // this wave's slot pairs: pairBase + 4 j, j < ppw <= DESC_PPW (the workgroup's
  // four waves interleave); lane 2 j + h holds the packed key of slot 2 (pairBase + 4 j) + h
  // slots [slotBeg, slotEnd): whole levels (level slot ranges are even)
  const int pairBase = (slotBeg >> 1) + bx * 4 * ppw + w;
  if (2 * pairBase >= slotEnd) return;
  const uint32_t* imgKeys = outKeys + (long long)img * plan.slotsPerImage;
  uint32_t keyv = 0;
  if (lane < 2 * ppw) {
    const int slot = 2 * (pairBase + 4 * (lane >> 1)) + (lane & 1);
    if (slot < slotEnd) keyv = imgKeys[slot];
  }
  // the image's per-level keypoint counts, lane l = level l, and their
  // exclusive prefix (output offsets): loaded once, read by v_readlane
  const int cntv = lane < plan.nlevels ? cnts[lane] : 0;
  const int cntx = wave_incl_scan(cntv) - cntv;
  // each level's first output slot, lane l = level l (ascending): a pair's
  // level is a ballot count instead of a loop of dependent scalar loads
  const int offv = lane < plan.nlevels ? plan.lv[lane].outOff : INT_MAX;
  uint32_t (*rsp)[DESC_RS_DW] = sm[w].rsp[half];
  // lane hl < 22 holds rows 2 hl and 2 hl + 1 (row 43 only feeds a zero weight)
  const bool second = hl < DESC_RS_PAIRS;
  // A pair is valid when its first slot holds a keypoint of its level; the
  // second half-wave duplicates the first when the level's count is odd.
  struct Pair {
    bool valid, active;
    int l, i, cx, cy;
    uint32_t key, key0, key1;  // key0 / key1: the keypoints of half 0 / half 1
  };
  auto setup = [&](int j) {
    Pair P;
    P.valid = false;
    const int slot0 = 2 * (pairBase + 4 * j);
    if (slot0 >= slotEnd) return P;
    const int l = __builtin_amdgcn_readfirstlane(__popcll(__ballot(offv <= slot0)) - 1);
    const int i0 = slot0 - __builtin_amdgcn_readlane(offv, l), nl = __builtin_amdgcn_readlane(cntv, l);
    if (i0 >= nl) return P;
    P.valid = true;
    P.l = l;
    P.active = i0 + half < nl;
    P.i = i0 + (P.active ? half : 0);
    const uint32_t k0 = __builtin_amdgcn_readlane(keyv, 2 * j);
    const uint32_t k1 = __builtin_amdgcn_readlane(keyv, 2 * j + 1);
    P.key = (half && P.active) ? k1 : k0;
    P.key0 = k0;
    P.key1 = i0 + 1 < nl ? k1 : k0;  // half 1 duplicates half 0 past the level's end
    P.cx = key_x(P.key);
    P.cy = key_y(P.key);
    return P;
  };
  // ---- staging: raw rows cy-21+r (REFLECT_101 rows), 12 dwords (3 x 16-byte
  // loads) from the 4-aligned byte at or below column cx-21
  uint32_t ra[12], rb[12], sha = 0, shb = 0;
  auto issue = [&](const Pair& P) {
    const OrbLevelDesc& L = plan.lv[P.l];
    const uint8_t* lvl;
    int pitch;
    if (P.l == 0) {
      lvl = img0 + (long long)img * img0Pitch;
      pitch = img0Stride;
    } else {
      lvl = arena + (long long)img * arenaPitch + L.arenaOff;
      pitch = L.pitch;
    }
    const ImgRsrc im = img_rsrc(lvl, (uint32_t)((L.h - 1) * pitch + L.w));
    // The realignment code: 0..3 = shift left by that many bytes (the row
    // starts inside the first loaded dword); 4 + s = shift right by s bytes:
    // the window of row 0 starts s bytes before the level's first byte
    // (cx - 21 + sh < 0: a keypoint 19 or 20 px from the left edge), so the
    // row is loaded from byte 0 and moved right (its first s bytes are
    // columns < 0, which the column patch below fills from their reflections).
    // Loading from the negative offset put the first 16 bytes out of the
    // buffer's range (read as 0): wrong blurred samples near the top-left corner.
    auto load_row = [&](int r, uint32_t* d) {
      int y = P.cy - 21 + r;
      y = y < 0 ? -y : (y >= L.h ? 2 * L.h - 2 - y : y);
      const int o = y * pitch + P.cx - 21 + (int)im.sh;
      const uint32_t a0 = o < 0 ? 0u : ((uint32_t)o & ~3u);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(im.r, (int)(a0 + 16 * k), 0, 0);
        d[4 * k] = (uint32_t)v[0];
        d[4 * k + 1] = (uint32_t)v[1];
        d[4 * k + 2] = (uint32_t)v[2];
        d[4 * k + 3] = (uint32_t)v[3];
      }
      return o < 0 ? 4u + (uint32_t)(-o) : ((uint32_t)o & 3u);
    };
    if (second) {
      sha = load_row(2 * hl, ra);
      shb = load_row(2 * hl + 1, rb);
    }
  };
  auto realign = [&](uint32_t* d, uint32_t sh) {
    if (sh < 4) {
#pragma unroll
      for (int k = 0; k < 11; ++k) d[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
      d[11] = __builtin_amdgcn_alignbyte(0u, d[11], sh);
    } else {  // right by sh - 4 bytes (row 0 of a window over the left edge)
      const uint32_t rs = 8u - sh;
#pragma unroll
      for (int k = 11; k > 0; --k) d[k] = __builtin_amdgcn_alignbyte(d[k], d[k - 1], rs);
      d[0] = __builtin_amdgcn_alignbyte(d[0], 0u, rs);
    }
  };
  auto store_row = [&](uint32_t* rowp, const uint32_t* d) {
    uint4* dst = reinterpret_cast<uint4*>(rowp);
    dst[0] = make_uint4(d[0], d[1], d[2], d[3]);
    dst[1] = make_uint4(d[4], d[5], d[6], d[7]);
    dst[2] = make_uint4(d[8], d[9], d[10], d[11]);
  };
  constexpr uint32_t k0 = 18, k1 = 34, k2 = 49, k3 = 55, k4 = 49, k5 = 34, k6 = 18;
  [[maybe_unused]] constexpr uint32_t T0a = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24), T0b = k4 | (k5 << 8) | (k6 << 16);
 [[maybe_unused]] constexpr uint32_t T1a = (k0 << 8) | (k1 << 16) | (k2 << 24), T1b = k3 | (k4 << 8) | (k5 << 16) | (k6 << 24);
 [[maybe_unused]] constexpr uint32_t T2a = (k0 << 16) | (k1 << 24), T2b = k2 | (k3 << 8) | (k4 << 16) | (k5 << 24), T2c = k6;
 [[maybe_unused]] constexpr uint32_t T3a = k0 << 24, T3b = k1 | (k2 << 8) | (k3 << 16) | (k4 << 24), T3c = k5 | (k6 << 8);
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 E0 = {18, 34}, E1 = {49, 55}, E2 = {49, 34}, E3 = {18, 0};
  const u16x2 O0 = {0, 18}, O1 = {34, 49}, O2 = {55, 49}, O3 = {34, 18};

  // IC_Angle byte masks of the lane's two rows (the rows are the same for
  // every keypoint pair): loaded once instead of per pair
  uint32_t mka[8], mkb[8];
  {
    const int ria = 2 * hl - 6, rib = 2 * hl + 1 - 6;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mka[k] = (ria >= 0 && ria <= 30) ? c_icmask[ria][k] : 0u;
      mkb[k] = (rib >= 0 && rib <= 30) ? c_icmask[rib][k] : 0u;
    }
  }
  Pair cur = setup(0);
  if (cur.valid) issue(cur);
  for (int j = 0; j < ppw; ++j) {
    const Pair P = cur;
    if (P.valid && second) {
      realign(ra, sha);
      realign(rb, shb);
    }
#define RA ra
#define RB rb
    // ---- IC_Angle from the rows in registers: row v = ri - 15 is staged row
    // ri + 6; columns u = -16..15 are staged bytes 5..36 (dwords 1..9 shifted
    // by one byte; reading dwords 1..9 as loaded under byte-shifted masks
    // measured slower: 0.464 vs 0.414 ms per 512 frames, profiles/r03_orient_row37.txt).
    // m10 = sum (u+16)*I - 16*sum I, m01 = sum v * rowsum.
    int m01 = 0, m10 = 0;
    auto ic_row = [&](const uint32_t* d, const uint32_t* mk, int ri) {  // staged row ri + 6, ri in [0, 31)
      uint32_t rs = 0, rm = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t dd = __builtin_amdgcn_alignbyte(d[k + 2], d[k + 1], 1) & mk[k];
        const uint32_t wt = (uint32_t)(4 * k) * 0x01010101u + 0x03020100u;
        rs = __builtin_amdgcn_udot4(dd, 0x01010101u, rs, false);
        rm = __builtin_amdgcn_udot4(dd, wt, rm, false);
      }
      m10 += (int)rm - 16 * (int)rs;
      m01 += (ri - 15) * (int)rs;
    };
    if (P.valid && second) {
      if (2 * hl >= 6 && 2 * hl <= 36) ic_row(RA, mka, 2 * hl - 6);
      if (2 * hl + 1 >= 6 && 2 * hl + 1 <= 36) ic_row(RB, mkb, 2 * hl + 1 - 6);
    }
    // (the rows stay in registers through the row pass: the next pair's loads
    // go out after it)
    if (!P.valid && j + 1 < ppw) {
      cur = setup(j + 1);
      if (cur.valid) issue(cur);
    }
    if (!P.valid) continue;  // wave-uniform
    const OrbLevelDesc& L = plan.lv[P.l];
    // The level's output offset is read here, with every lane active.  Read
    // inside the epilogue's `P.active && hl == 0` branch, hipcc sank the
    // v_sub that forms cntx into that branch, so the v_readlane of lane P.l
    // saw a lane the sub had not run in: a stale register (wrong slots in
    // k_orient_desc<1>, an out-of-range store and a device fault under
    // __launch_bounds__(256, 5)).
    const int base = __builtin_amdgcn_readlane(cntx, P.l);
    const int cx = P.cx, cy = P.cy, colA = cx - 21;
    if (colA < 0 || cx + 21 >= L.w) {
      // window overhangs a level column edge: the lane's two rows go through
      // the (not yet used) row-sum area, where the bytes of columns < 0 or >= w
      // take their REFLECT_101 column, and come back patched
      uint32_t* scr = &rsp[0][0] + 24 * hl;  // rows 2 hl, 2 hl + 1: 12 dwords each
      if (second) {
        store_row(scr, RA);
        store_row(scr + 12, RB);
        for (int s2 = 0; s2 < 2; ++s2) {
          uint8_t* rp = reinterpret_cast<uint8_t*>(scr + 12 * s2);
          for (int b = 0; b < -colA; ++b) rp[b] = rp[-(colA + b) - colA];
          for (int b = max(L.w - colA, 0); b < 43; ++b) rp[b] = rp[2 * L.w - 2 - (colA + b) - colA];
        }
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          RA[k] = scr[k];
          RB[k] = scr[12 + k];
        }
      }
      wave_lds_sync();
    }
    // ---- row pass: row-sum column c of staged row r = sum_i k_i * byte(r, c + i)
    // ---- row pass: row-sum column c of staged row r = sum_i k_i * byte(r, c + i)
    if (second) {  // the lane's row pair from registers, group by group
      // (samples reach columns 0..36 only: |rotated pattern point| <= 18.4,
      // so the last group computes column 36 alone)
#pragma unroll
      for (int g = 0; g < 10; ++g) {
        if (DESC_ROW37 && g == 9) {
          const uint32_t c0 = __builtin_amdgcn_udot4(RA[9], T0a, __builtin_amdgcn_udot4(RA[10], T0b, 0u, false), false);
          const uint32_t c1 = __builtin_amdgcn_udot4(RB[9], T0a, __builtin_amdgcn_udot4(RB[10], T0b, 0u, false), false);
          rsp[hl][36] = __builtin_amdgcn_perm(c1, c0, 0x05040100u);
          break;
        }
        uint32_t o[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t* rw = h ? RB : RA;
          const uint32_t w0 = rw[g], w1 = rw[g + 1], w2 = rw[g + 2];
          o[h][0] = __builtin_amdgcn_udot4(w0, T0a, __builtin_amdgcn_udot4(w1, T0b, 0u, false), false);
          o[h][1] = __builtin_amdgcn_udot4(w0, T1a, __builtin_amdgcn_udot4(w1, T1b, 0u, false), false);
          o[h][2] = __builtin_amdgcn_udot4(w0, T2a, __builtin_amdgcn_udot4(w1, T2b,
                                           __builtin_amdgcn_udot4(w2, T2c, 0u, false), false), false);
          o[h][3] = __builtin_amdgcn_udot4(w0, T3a, __builtin_amdgcn_udot4(w1, T3b,
                                           __builtin_amdgcn_udot4(w2, T3c, 0u, false), false), false);
        }
        // (row sums are < 2^16: one v_perm packs the pair)
        auto pk = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x05040100u); };
        *reinterpret_cast<uint4*>(&rsp[hl][4 * g]) =
            make_uint4(pk(o[0][0], o[1][0]), pk(o[0][1], o[1][1]), pk(o[0][2], o[1][2]),
                       pk(o[0][3], o[1][3]));
      }
    }
    if (j + 1 < ppw) {
      cur = setup(j + 1);
      if (cur.valid) issue(cur);
    }
    m01 = half_sum(m01);
    m10 = half_sum(m10);
    const float angle = fast_atan2_deg((float)m01, (float)m10);
    wave_lds_sync();
    // ---- rBRIEF sampling the blur directly: blurred pixel (ry, rx) of the
    // patch = column pass of row-sum rows 18+ry .. 24+ry at column 18+rx,
    // i.e. the four pairs (18+ry)/2 .. +3 with the parity's weights
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float a, b;
    {
      float sn, cs;
      pinned_sincos(angle * factorPI, &sn, &cs);
      a = cs;
      b = sn;
    }
    const uint32_t wE[4] = {__builtin_bit_cast(uint32_t, E0), __builtin_bit_cast(uint32_t, E1),
                            __builtin_bit_cast(uint32_t, E2), __builtin_bit_cast(uint32_t, E3)};
    const uint32_t wO[4] = {__builtin_bit_cast(uint32_t, O0), __builtin_bit_cast(uint32_t, O1),
                            __builtin_bit_cast(uint32_t, O2), __builtin_bit_cast(uint32_t, O3)};
#if DESC_LDS_TABLES
    (void)wE;
    (void)wO;
    // the patch centre's row-sum pair (an opaque base: hipcc would split the
    // constant between the address and the 8-bit ds_read2 offsets)
    const uint32_t* rs0 = &sm[0].rsp[0][0][0];
    int rsc = (int)(&rsp[0][0] - rs0) + (18 * (DESC_RS_DW / 2) + 18);
    __asm__ volatile("" : "+v"(rsc));
#if DESC_MAGIC_ROUND
    // cvRound by the adder: for |v| < 2^22, the bits of v + 1.5 * 2^23 are
    // 0x4B400000 + rint(v) (round half to even, as rintf), so a coordinate
    // costs one v_add_f32 instead of v_rndne + v_cvt; the biases of both
    // coordinates go into the base (0x4B400000 is even: parity and ry & ~1
    // read the same bits; its low 24 bits 0x400000 keep the signed 24-bit
    // multiply's operand positive)
    rsc -= 0x400000 * (DESC_RS_DW / 2) + 0x4B400000;
    // (by, bx): the adder's bit patterns of the rotated coordinates
    auto blurred = [&](int by, int bx) -> int {
      const uint32_t* p = rs0 + (rsc + __mul24(by & ~1, DESC_RS_DW / 2) + bx);
      const uint4 wv = sW[by & 1];
#else
    auto blurred = [&](float fy, float fx) -> int {
      const int ry = cv_round(fy), rx = cv_round(fx);
      // pair row (ry + 18) >> 1, column rx + 18: the constant part folds into
      // the LDS offset, (ry & ~1) * (DESC_RS_DW / 2) is a signed 24-bit
      // multiply (ry is -18..18; hipcc cannot bound a plain int product and
      // emits the quarter-rate v_mul_lo_u32), the parity row is ry & 1
      const uint32_t* p = rs0 + (rsc + __mul24(ry & ~1, DESC_RS_DW / 2) + rx);
      const uint4 wv = sW[ry & 1];
#endif
      const uint32_t wk[4] = {wv.x, wv.y, wv.z, wv.w};
      uint32_t s = 1u << 15;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        s = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p[k * DESC_RS_DW]),
                                   __builtin_bit_cast(u16x2, wk[k]), s, false);
      return min((int)(s >> 16), 255);
    };
#else
    auto blurred = [&](float fy, float fx) -> int {
      const int ry = cv_round(fy), rx = cv_round(fx);
      const int y = ry + 18;
      const uint32_t* p = &rsp[y >> 1][rx + 18];
      uint32_t s = 1u << 15;
      const bool odd = y & 1;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        s = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p[k * DESC_RS_DW]),
                                   __builtin_bit_cast(u16x2, odd ? wO[k] : wE[k]), s, false);
      return min((int)(s >> 16), 255);
    };
#endif
    unsigned long long words[8];
#pragma unroll
    for (int kq = 0; kq < 8; ++kq) {
      const int test = hl + 32 * kq;
#if DESC_LDS_TABLES
      const float4 pt = sPat[test];
      const float px0 = pt.x, py0 = pt.y, px1 = pt.z, py1 = pt.w;
#else
      const float px0 = (float)c_pattern[4 * test], py0 = (float)c_pattern[4 * test + 1];
      const float px1 = (float)c_pattern[4 * test + 2], py1 = (float)c_pattern[4 * test + 3];
#endif
#if DESC_MAGIC_ROUND
      const int v0 = blurred(__builtin_bit_cast(int, (px0 * b + py0 * a) + 12582912.0f),
                             __builtin_bit_cast(int, (px0 * a - py0 * b) + 12582912.0f));
      const int v1 = blurred(__builtin_bit_cast(int, (px1 * b + py1 * a) + 12582912.0f),
                             __builtin_bit_cast(int, (px1 * a - py1 * b) + 12582912.0f));
#else
      const int v0 = blurred(px0 * b + py0 * a, px0 * a - py0 * b);
      const int v1 = blurred(px1 * b + py1 * a, px1 * a - py1 * b);
#endif
      words[kq] = __ballot(v0 < v1);
    }
    if (P.active && hl == 0) {
      const long long o = (long long)img * capacity + base + P.i;
      uint32_t d[8];
#pragma unroll
      for (int kq = 0; kq < 8; ++kq) d[kq] = (uint32_t)(words[kq] >> (32 * half));
      uint4* dst = reinterpret_cast<uint4*>(desc + o * 32);
      dst[0] = make_uint4(d[0], d[1], d[2], d[3]);
      dst[1] = make_uint4(d[4], d[5], d[6], d[7]);
      orb_keypoint_t kp;
      kp.x = P.l ? (float)cx * L.scale : (float)cx;  // pt *= mvScaleFactor[level] (:1157-1165)
      kp.y = P.l ? (float)cy * L.scale : (float)cy;
      kp.size = L.sizeF;
      kp.angle = angle;
      kp.response = (float)key_s(P.key);
      kp.octave = P.l;
      kp.class_id = -1;
      kps[o] = kp;
    }
#undef RA
#undef RB
    // the next pair's staging overwrites raw: every lane's patch reads are done
    wave_lds_sync();
  }
}

// ============================================================ k_copy_pinned
// Host -> device copy as a kernel on the caller's queue.  A copy-engine DMA's
// completion reaches the next kernel on the compute queue ~7 us late
// (profiles/r06_dropin_timeline.txt: the image's and the matcher inputs' DMAs
// each followed by a 7 us idle gap); a kernel reading the pinned block over
// PCIe hands over with no cross-engine wait.  The loads are system-coherent
// (sc0 sc1: the host wrote the block just before the launch) and each thread
// moves 16-byte words, grid-stride.  bytes and both addresses 16-byte aligned
// (the launcher checks).
__global__ __launch_bounds__(256) void k_copy_pinned(uint4* __restrict__ dst, const uint8_t* src,
                                                     uint32_t n16) {
  const __amdgpu_buffer_rsrc_t r = make_rsrc(src, n16 * 16u);
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16u), 0, 17 /* sc0 sc1 */);
    dst[i] = make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
  }
}

// Device -> host counterpart: dwords stored system-coherent (sc0 sc1: written
// through to host memory, visible once the stream's completion is), as a
// kernel on the caller's queue right behind the kernel that produced them (a
// separate hipMemcpyAsync started 7 us after it, profiles/r06_dropin_timeline.txt).
__global__ __launch_bounds__(256) void k_copy_to_pinned(uint8_t* dst, const uint32_t* __restrict__ src,
                                                        uint32_t n4) {
  const __amdgpu_buffer_rsrc_t r = make_rsrc(dst, n4 * 4u);
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n4; i += gridDim.x * 256u)
    __builtin_amdgcn_raw_buffer_store_b32(src[i], r, (int)(i * 4u), 0, 17 /* sc0 sc1 */);
}

// ------------------------------------------------------------ host launchers
extern "C" {

hipError_t orb_k_copy_pinned(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if ((bytes & 15) || ((uintptr_t)dst & 15) || ((uintptr_t)src & 15) || bytes >= (1ull << 31))
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
  const uint32_t n16 = (uint32_t)(bytes >> 4);
  const uint32_t grid = std::min<uint32_t>((n16 + 255) / 256, 512);
  k_copy_pinned<<<grid, 256, 0, s>>>(reinterpret_cast<uint4*>(dst),
                                     reinterpret_cast<const uint8_t*>(src), n16);
  return hipGetLastError();
}

hipError_t orb_k_copy_to_pinned(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if ((bytes & 3) || ((uintptr_t)dst & 3) || ((uintptr_t)src & 3) || bytes >= (1ull << 31))
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
  const uint32_t n4 = (uint32_t)(bytes >> 2);
  const uint32_t grid = std::min<uint32_t>((n4 + 255) / 256, 512);
  k_copy_to_pinned<<<grid, 256, 0, s>>>(reinterpret_cast<uint8_t*>(dst),
                                        reinterpret_cast<const uint32_t*>(src), n4);
  return hipGetLastError();
}

hipError_t orb_k_upload_constants(hipStream_t s) {
  static int8_t pat[2 * ORB_PATTERN_POINTS];
  for (int i = 0; i < 2 * ORB_PATTERN_POINTS; ++i) pat[i] = (int8_t)kOrbPatternXY[i];
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_pattern), pat, sizeof(pat), 0,
                                        hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(s);  // the static staging array is reused
}

hipError_t orb_k_upload_umax(const int* umax16, hipStream_t s) {
  static uint32_t mask[32][8];
  for (int r = 0; r < 32; ++r)
    for (int k = 0; k < 8; ++k) {
      uint32_t m = 0;
      for (int j = 0; j < 4; ++j) {
        const int u = 4 * k + j - 16, v = r - 15;
        if (r < 31 && u >= -umax16[v < 0 ? -v : v] && u <= umax16[v < 0 ? -v : v]) m |= 0xFFu << (8 * j);
      }
      mask[r][k] = m;
    }
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_icmask), mask, sizeof(mask), 0,
                                        hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_umax), umax16, 16 * sizeof(int), 0,
                             hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(s);  // the static staging array is reused
}

hipError_t orb_k_pyr_resize(const uint8_t* src, long long srcImgPitch, int srcStride, int sw,
                            int sh, uint8_t* dst, long long dstImgPitch, int dstStride, int dw,
                            int dh, const int* xofs, const void* alpha, const int* yofs,
                            const void* beta, int mode, int nimg, hipStream_t s) {
  if (mode == ORB_RESIZE_GENERIC) {
    hipLaunchKernelGGL(k_pyr_resize_generic, dim3((dw + 255) / 256, (dh + 3) / 4, nimg), dim3(256), 0,
                       s, src, srcImgPitch, srcStride, sw, sh, dst, dstImgPitch, dstStride, dw, dh,
                       xofs, (const int*)alpha, yofs, (const int*)beta);
    return hipGetLastError();
  }
  // tile bounds (the planner picked the variant every tile of the level fits):
  // narrow for a per-level downscale <= 1.25, wide beyond
  const bool wide = mode == ORB_RESIZE_WIDE;
  // each workgroup resizes one tile of PYR_IMAGES_PER_WG images (default
  // 16: with two extraction lanes 12 / 16 / 24 measured 323.8k / 322.3-324.4k /
  // 324.7k against 321.3-321.8k frames/s for 8, profiles/r03_lanes.txt)
  // PYR_IMAGES_PER_WG images per workgroup; with PYR_TARGET_WGS > 0 fewer when
  // the level would launch under that many workgroups (a workgroup walks its
  // images one after another: C5's 16 1920x1080 frames are 510 workgroups of
  // 16 images on level 1)
  const int tiles = ((dw + PYR_TW - 1) / PYR_TW) * ((dh + PYR_TH - 1) / PYR_TH);
  const int perWg =
      PYR_TARGET_WGS > 0
          ? std::max(1, std::min(PYR_IMAGES_PER_WG, (int)((long long)tiles * nimg / std::max(PYR_TARGET_WGS, 1))))
          : PYR_IMAGES_PER_WG;
  dim3 grid((dw + PYR_TW - 1) / PYR_TW, (dh + PYR_TH - 1) / PYR_TH, (nimg + perWg - 1) / perWg),
      block(256);
  // every image base and row start 4-aligned: one load per staged dword
  const bool aligned = (srcStride & 3) == 0 && (((uintptr_t)src) & 3) == 0 && (srcImgPitch & 3) == 0;
#define ORB_RESIZE_LAUNCH(AL, R, W)                                                              \
  hipLaunchKernelGGL((k_pyr_resize<AL, R, W>), grid, block, 0, s, src, srcImgPitch, srcStride, sw, \
                     sh, dst, dstImgPitch, dstStride, dw, dh, xofs, (const int*)alpha, yofs,      \
                     (const int*)beta, nimg)
  if (!wide && aligned) ORB_RESIZE_LAUNCH(true, PYR_SROWS, PYR_SW);
  else if (!wide) ORB_RESIZE_LAUNCH(false, PYR_SROWS, PYR_SW);
  else if (aligned) ORB_RESIZE_LAUNCH(true, PYR_SROWS_WIDE, PYR_SW_WIDE);
  else ORB_RESIZE_LAUNCH(false, PYR_SROWS_WIDE, PYR_SW_WIDE);
#undef ORB_RESIZE_LAUNCH
  return hipGetLastError();
}

// Levels l and l + 1 in one launch (k_pyr_resize2): src = level l - 1, mid =
// level l, dst = level l + 1, each with its own tables (l from l - 1, l + 1
// from l).  The planner has checked every tile against the kernel's windows
// (orb_k_pyr_resize2_fits).
hipError_t orb_k_pyr_resize2(const uint8_t* src, long long srcImgPitch, int srcStride, int w0,
                             int h0, uint8_t* mid, long long midImgPitch, int midStride, int w1,
                             int h1, const int* xo1, const void* al1, const int* yo1,
                             const void* be1, uint8_t* dst, long long dstImgPitch, int dstStride,
                             int w2, int h2, const int* xo2, const void* al2, const int* yo2,
                             const void* be2, int nimg, hipStream_t s) {
  const dim3 grid((w2 + PYR_TW - 1) / PYR_TW, (h2 + PYR_TH - 1) / PYR_TH,
                  (nimg + PYR_IMAGES_PER_WG - 1) / PYR_IMAGES_PER_WG),
      block(256);
  const bool aligned = (srcStride & 3) == 0 && (((uintptr_t)src) & 3) == 0 && (srcImgPitch & 3) == 0;
  if (aligned)
    hipLaunchKernelGGL(k_pyr_resize2<true>, grid, block, 0, s, src, srcImgPitch, srcStride, w0, h0,
                       mid, midImgPitch, midStride, w1, h1, xo1, (const int*)al1, yo1,
                       (const int*)be1, dst, dstImgPitch, dstStride, w2, h2, xo2, (const int*)al2,
                       yo2, (const int*)be2, nimg);
  else
    hipLaunchKernelGGL(k_pyr_resize2<false>, grid, block, 0, s, src, srcImgPitch, srcStride, w0, h0,
                       mid, midImgPitch, midStride, w1, h1, xo1, (const int*)al1, yo1,
                       (const int*)be1, dst, dstImgPitch, dstStride, w2, h2, xo2, (const int*)al2,
                       yo2, (const int*)be2, nimg);
  return hipGetLastError();
}

// Whether every tile of the level pair fits k_pyr_resize2's windows: the
// level-l region (rows, dwords + 2 read-ahead) within PYR2_R1R x PYR2_R1W, the
// level l-1 window within PYR2_S0R x PYR2_S0W (with each group's read-ahead).
// Tables as the planner builds them (x: xofs, y: yofs per level).
int orb_k_pyr_resize2_fits(int w0, int h0, int w1, int h1, const int* xo1, const int* yo1, int w2,
                           int h2, const int* xo2, const int* yo2) {
  for (int x0 = 0; x0 < w2; x0 += PYR_TW) {
    const int xl = std::min(x0 + PYR_TW - 1, w2 - 1), xt = std::min(x0 + PYR_TW - 4, w2 - 1);
    const int X0 = x0 == 0 ? 0 : (xo2[x0] & ~3);
    const int ownX = x0 + PYR_TW >= w2 ? w1 : (xo2[x0 + PYR_TW] & ~3);
    const int X1e = std::max(std::min(xo2[xl] + 1, w1 - 1) + 1, ownX);
    const int nG1 = (X1e - X0 + 3) >> 2;
    if (X0 < 0 || ownX < X0 || 4 * nG1 > PYR2_TAB || nG1 > PYR2_R1W) return 0;
    if (((xo2[xt] - X0) >> 2) + 2 >= PYR2_R1W) return 0;  // level l+1 read-ahead
    const int c0a = xo1[X0], c0b = std::min(xo1[std::min(X0 + 4 * nG1 - 1, w1 - 1)] + 1, w0 - 1);
    const int colBase0 = c0a & ~3, nW0 = ((c0b - colBase0) >> 2) + 1;
    if (4 * ((nW0 + 3) >> 2) > PYR2_S0W) return 0;
    for (int g = 0; g < nG1; ++g) {
      const int xa = std::min(X0 + 4 * g, w1 - 1);
      if (xo1[std::min(xa + 3, w1 - 1)] - xo1[xa] > 6) return 0;  // 8 source bytes per group
      if (((xo1[xa] - colBase0) >> 2) + 2 >= PYR2_S0W) return 0;
    }
  }
  for (int y0 = 0; y0 < h2; y0 += PYR_TH) {
    const int yl = std::min(y0 + PYR_TH - 1, h2 - 1);
    const int Y0 = y0 == 0 ? 0 : std::min(std::max(yo2[y0], 0), h1 - 1);
    const int ownY = y0 + PYR_TH >= h2 ? h1 : std::min(std::max(yo2[y0 + PYR_TH], 0), h1 - 1);
    const int Y1e = std::max(std::min(std::max(yo2[yl] + 1, 0), h1 - 1) + 1, ownY);
    if (ownY < Y0 || Y1e - Y0 > PYR2_R1R) return 0;
    const int r0a = std::min(std::max(yo1[Y0], 0), h0 - 1);
    const int r0b = std::min(std::max(yo1[Y1e - 1] + 1, 0), h0 - 1);
    if (r0b - r0a + 1 > PYR2_S0R) return 0;
  }
  return 1;
}

// Dynamic LDS of k_fast_band for bands of up to `bandElems` elements (rows x
// element pitch): f16 pixels, strengths, queue, corner list, two interior
// bitmaps, per-column flags / cells, phase-B group list.
size_t orb_k_fast_band_lds(int bandElems) {
  const size_t bitBytes = 4 * (size_t)(((bandElems >> 5) + 4) & ~1);
  return (size_t)bandElems * 3 + FAST_QCAP * 2 + FAST_CORNERS * 2 + 2 * bitBytes +
         2 * (size_t)((bandElems / 7 + 15) & ~7) + 2 * ((size_t)bandElems / 28 + 8);
}

hipError_t orb_k_fast_band(const uint8_t* img0, long long img0Pitch, int img0Stride,
                           const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                           const OrbBandDesc* bands, int nbands, const OrbCellDesc* cells,
                           uint32_t* cellKeys, int32_t* cellCount, int32_t* errFlag, int nimg,
                           hipStream_t s) {
  const size_t lds = orb_k_fast_band_lds(plan->maxBandBytes);
  // each workgroup takes 2 bands (swept 1-8 in round 2), prefetching the next
  // (one band per workgroup for a frame or two per call: the grid is small and
  // the per-workgroup band chain is the latency)
  const int perWg = nimg <= 2 ? 1 : 2;
  if ((size_t)plan->maxBandBytes > (size_t)4 * FAST_LOADS * 256) return hipErrorInvalidValue;
  dim3 grid((nbands + perWg - 1) / perWg, nimg), block(256);
  hipLaunchKernelGGL(k_fast_band, grid, block, lds, s, img0, img0Pitch, img0Stride, arena,
                     arenaPitch, *plan, bands, cells, nbands, cellKeys, cellCount, errFlag);
  return hipGetLastError();
}

// k_fast_cells: LDS per workgroup for cells of at most maxRows x maxCols
// (ROI incl. the 3-px border)
// k_fast_cells stages one ROI row per lane (every ORB-SLAM2 configuration;
// the larger cells of tiny levels go to k_fast_band)
bool orb_k_fast_cells_fits(const OrbPlanDesc* plan) {
  // lane = ROI row (<= 64 rows); a row's P <= 56 bytes (+3 realign) in four 16-byte loads
  return plan->maxCellRows <= 64 && ((plan->maxCellCols + 20) & ~7) <= 56;
}

size_t orb_k_fast_cells_lds(int maxRows, int maxCols) {
  return (size_t)FC_WAVES * fc_wave_bytes(fc_tile_elems(maxRows, maxCols));
}

// cells [cellBeg, cellEnd) of every image (the level-0 cells can run beside the
// resize chain, which levels >= 1 wait for)
hipError_t orb_k_fast_cells(const uint8_t* img0, long long img0Pitch, int img0Stride,
                            const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                            const OrbCellDesc* cells, uint32_t* cellKeys, int32_t* cellCount,
                            int32_t* errFlag, int cellBeg, int cellEnd, int nimg, hipStream_t s) {
  if (cellEnd <= cellBeg) return hipSuccess;
  if (!orb_k_fast_cells_fits(plan)) return hipErrorInvalidValue;
  // LDS sized for the largest cell of the levels this launch covers (level 0's
  // side launch gets the smaller slices of its 38-row cells)
  int mr = 7, mc = 7;
  for (int l = 0; l < plan->nlevels; ++l)
    if (plan->lv[l].cellBeg < cellEnd && plan->lv[l].cellEnd > cellBeg) {
      mr = std::max(mr, plan->lv[l].cellMaxRows);
      mc = std::max(mc, plan->lv[l].cellMaxCols);
    }
  const int tileElems = fc_tile_elems(mr, mc);
  const size_t lds = orb_k_fast_cells_lds(mr, mc);
  // every W = 30 cell grid of the ORB-SLAM2 configurations has ROI widths of
  // 36-43 pixels: pitch 48 (56 without FC_TIGHT), the compile-time instance
  const bool p56 = fc_pitch(mc) == FC_CONST_PITCH;
  const void* fn = p56 ? (const void*)k_fast_cells<FC_CONST_PITCH> : (const void*)k_fast_cells<0>;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const int n = cellEnd - cellBeg;
  dim3 grid((n + FC_WAVES * FC_CPW - 1) / (FC_WAVES * FC_CPW), nimg), block(64 * FC_WAVES);
  if (p56)
    hipLaunchKernelGGL(k_fast_cells<FC_CONST_PITCH>, grid, block, lds, s, img0, img0Pitch, img0Stride, arena,
                       arenaPitch, *plan, cells, cellKeys, cellCount, tileElems, cellBeg, cellEnd,
                       errFlag);
  else
    hipLaunchKernelGGL(k_fast_cells<0>, grid, block, lds, s, img0, img0Pitch, img0Stride, arena,
                       arenaPitch, *plan, cells, cellKeys, cellCount, tileElems, cellBeg, cellEnd,
                       errFlag);
  return hipGetLastError();
}

size_t orb_k_octree_lds(int nodeCapMax, int maxCellsPerLevel, int ldsKeyCap) {
  int n2 = 1;
  while (n2 < nodeCapMax) n2 <<= 1;
  size_t b = (size_t)n2 * 8 + 2 * (size_t)nodeCapMax * sizeof(OctNode) + (size_t)nodeCapMax * 16 +
             4 * (size_t)nodeCapMax * 4 + (size_t)((maxCellsPerLevel + 3) & ~3) * 4;
  b += (size_t)ldsKeyCap * 4 + (size_t)ldsKeyCap * 2;
  return b;
}

size_t orb_k_octree_node_bytes(int nodeCapMax, int maxCellsPerLevel) {
  return orb_k_octree_lds(nodeCapMax, maxCellsPerLevel, 0);
}

hipError_t orb_k_octree(const OrbPlanDesc* plan, const int32_t* cellCount,
                        const uint32_t* cellKeys, uint32_t* gKeys, uint16_t* gNid, int ldsKeyCap,
                        int nodeCapMax, int maxCellsPerLevel, uint32_t* outKeys,
                        int32_t* outCount, int32_t* errFlag, int levelBeg, int levelEnd, int nimg,
                        uint8_t* gNodes, long long nodeStride, hipStream_t s) {
  if (levelEnd <= levelBeg || nimg <= 0) return hipSuccess;
  // global node tables (gNodes): the LDS holds the keys only
  const size_t lds = gNodes ? (size_t)ldsKeyCap * 6
                            : orb_k_octree_lds(nodeCapMax, maxCellsPerLevel, ldsKeyCap);
  // register-resident keys for a few frames per call (one workgroup per level)
  const bool reg = nimg <= 16;
  const bool gn = gNodes != nullptr;
  const void* fn = reg ? (gn ? (const void*)k_octree<true, true> : (const void*)k_octree<true, false>)
                       : (gn ? (const void*)k_octree<false, true> : (const void*)k_octree<false, false>);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  // The pass bound is never reached with the reference's own bounds (a pass
  // halves every divided node; distinct keys separate in ~12 passes, the
  // final phase adds a few).  The test build lib/variants/octree_passes2.so
  // (make testhook: -DORB_OCTREE_TEST_PASSES=2) lowers it to drive the
  // failed-image path (negative count, ORB_EDEVICE); the product has no hook.
#ifdef ORB_OCTREE_TEST_PASSES
  constexpr int maxPasses = ORB_OCTREE_TEST_PASSES;
  static_assert(ORB_OCTREE_TEST_PASSES >= 1 && ORB_OCTREE_TEST_PASSES <= OCT_MAX_PASSES, "pass bound");
#else
  constexpr int maxPasses = OCT_MAX_PASSES;
#endif
  // Batches take 256-thread workgroups: the octree alone is slower (0.150 vs
  // 0.132 ms per 512 frames) but the smaller workgroups fit better beside the
  // other lane's kernels (bench 317.0k / 316.6k vs 315.5k / 315.2k frames/s,
  // two interleaved pairs, profiles/r03_octree256.txt); 512 threads
  // was the old shape
  constexpr int bthreads = OCT_BATCH_THREADS;
  static_assert(OCT_BATCH_THREADS >= 128 && OCT_BATCH_THREADS % 64 == 0, "octree rank needs >= 128 threads");
  dim3 grid(nimg, levelEnd - levelBeg), block(reg ? OCT_REG_THREADS : bthreads);
#define ORB_OCTREE_LAUNCH(R, G)                                                                 \
  hipLaunchKernelGGL((k_octree<R, G>), grid, block, lds, s, *plan, cellCount, cellKeys, gKeys,  \
                     gNid, ldsKeyCap, nodeCapMax, maxCellsPerLevel, outKeys, outCount, errFlag, \
                     levelBeg, maxPasses, gNodes, nodeStride)
  if (reg && gn) ORB_OCTREE_LAUNCH(true, true);
  else if (reg) ORB_OCTREE_LAUNCH(true, false);
  else if (gn) ORB_OCTREE_LAUNCH(false, true);
  else ORB_OCTREE_LAUNCH(false, false);
#undef ORB_OCTREE_LAUNCH
  return hipGetLastError();
}

hipError_t orb_k_blur_levels(const uint8_t* img0, long long img0Pitch, int img0Stride,
                             const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                             const OrbTileDesc* tiles, uint8_t* blur, long long blurPitch,
                             int nimg, hipStream_t s) {
  // each workgroup blurs one tile of 8 images (swept 2-16)
  constexpr int perWg = 8;
  dim3 grid(plan->nBlurTiles, (nimg + perWg - 1) / perWg), block(256);
  hipLaunchKernelGGL(k_blur_levels, grid, block, 0, s, img0, img0Pitch, img0Stride, arena,
                     arenaPitch, *plan, tiles, blur, blurPitch, nimg);
  return hipGetLastError();
}

hipError_t orb_k_orient_desc(const uint8_t* img0, long long img0Pitch, int img0Stride,
                             const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                             const uint32_t* outKeys, const int32_t* outCount,
                             const int32_t* errFlag, orb_keypoint_t* kps, uint8_t* desc,
                             int capacity, int32_t* counts, int nimg, int levelBeg,
                             int levelEnd, hipStream_t s) {
  if (plan->slotsPerImage & 1) return hipErrorInvalidValue;
  if (levelBeg < 0 || levelEnd > plan->nlevels || levelBeg >= levelEnd) return hipErrorInvalidValue;
  const int slotBeg = plan->lv[levelBeg].outOff;
  const int slotEnd = levelEnd == plan->nlevels ? plan->slotsPerImage : plan->lv[levelEnd].outOff;
  if ((slotBeg | slotEnd) & 1) return hipErrorInvalidValue;
  // DESC_PPW keypoint pairs per wave for batches (the next pair's loads overlap
  // the current one); one pair per wave for a frame or two per call, where the
  // grid is small and the per-wave chain is the latency
  const int ppw = nimg <= 2 ? 1 : DESC_PPW;
  dim3 grid((slotEnd - slotBeg + 8 * ppw - 1) / (8 * ppw), nimg), block(256);
  if (ppw == DESC_PPW)
    hipLaunchKernelGGL(k_orient_desc<DESC_PPW>, grid, block, 0, s, img0, img0Pitch, img0Stride,
                       arena, arenaPitch, *plan, outKeys, outCount, errFlag, kps, desc, capacity,
                       counts, DESC_PPW, slotBeg, slotEnd);
  else if (ppw == 1 && DESC_SMALL_CT)
    hipLaunchKernelGGL(k_orient_desc<1>, grid, block, 0, s, img0, img0Pitch, img0Stride, arena,
                       arenaPitch, *plan, outKeys, outCount, errFlag, kps, desc, capacity, counts,
                       1, slotBeg, slotEnd);
  else
    hipLaunchKernelGGL(k_orient_desc<0>, grid, block, 0, s, img0, img0Pitch, img0Stride, arena,
                       arenaPitch, *plan, outKeys, outCount, errFlag, kps, desc, capacity, counts,
                       ppw, slotBeg, slotEnd);
  return hipGetLastError();
}

}  // extern "C"
