// matcher_kernels.hip -- gfx950 kernels of the Hamming matcher (ORBmatcher + Frame grid).
//
// Hamming distance = 4 x __popcll over the 256-bit descriptors (no MFMA: these
// are bit-count/compare kernels).  The reference matchers are sequential with
// "first-come" keypoint claims (src/ORBmatcher.cc:90-93,127), so each matcher
// is split into a data-parallel distance stage that keeps, per query, the
// first K candidates in (distance, scan order) order, and an ordered resolve
// stage that replays the sequential semantics exactly.
#include <algorithm>
#include <cmath>

#include "matcher_common.h"

// ---------------------------------------------------------- k_hamming_batch
__global__ __launch_bounds__(256) void k_hamming_batch(const uint8_t* __restrict__ a,
                                                       const uint8_t* __restrict__ b, int n,
                                                       int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = hamming256(load_desc(a + (size_t)i * 32), load_desc(b + (size_t)i * 32));
}

// ------------------------------------------------------------ k_grid_build
// Frame::AssignFeaturesToGrid + PosInGrid (src/Frame.cc:261-276, 426-436):
// cell = (round((x-minX)*invW), round((y-minY)*invH)), out-of-grid keys dropped,
// per-cell lists in ascending keypoint index.  Stored as CSR with cell index
// ix*48+iy, the order GetFeaturesInArea scans (ix outer, iy inner, :391-400).
//
// One wave per frame and 12 KB of LDS (the 3,073 cell counters): LDS counts,
// a wave scan over the cells (48 per lane, read and written as b128), then a
// stable scatter in keypoint order, 64 keys a round: lanes holding the same
// cell find each other with 12 ballots over the cell id bits, so a key's slot
// is its cell's cursor plus the same-cell lanes below it, and the group's
// highest lane advances the cursor.  The next round's keypoint fields are
// loaded while the current one scatters.  (Round 3's 256-thread form held
// 56.7 KB of LDS per frame and sorted each cell's list with one thread; beside
// the extraction kernels it waited for LDS and ran 2.3 ms per 1,024 frames.)
// `staged` (optional): the keypoints in cell order as k_proj_candidates stages
// them in LDS, {x, y, idx | octave << 24 | locked << 31, uR}, so that each of
// its workgroups copies the frame's grid with coalesced loads instead of
// gathering it through cellIdx.
#define GB_LDS_KEYS 8192  // staged copies for frames of up to this many keypoint slots
__global__ __launch_bounds__(64) void k_grid_build(const orb_keypoint_t* __restrict__ keys,
                                                   const int32_t* __restrict__ nkeys, int kpStride,
                                                   float minX, float minY, float invW, float invH,
                                                   int32_t* __restrict__ cellStart,
                                                   int32_t* __restrict__ cellIdx,
                                                   const uint8_t* __restrict__ locked,
                                                   const float* __restrict__ uright,
                                                   uint4* __restrict__ staged) {
  __shared__ __attribute__((aligned(16))) int cnt[GRID_CELLS + 4];
  const int p = blockIdx.x, lane = threadIdx.x;
  const int n = max(nkeys[p], 0);
  const orb_keypoint_t* K = keys + (size_t)p * kpStride;
  {
    int4* c4 = reinterpret_cast<int4*>(cnt);
    for (int i = lane; i < (GRID_CELLS + 4) / 4; i += 64) c4[i] = make_int4(0, 0, 0, 0);
  }
  __syncthreads();
  // counts: four keys per lane in flight
  for (int base = 0; base < n; base += 256) {
    int c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = base + 64 * j + lane;
      c[j] = k < n ? grid_cell(K[k], minX, minY, invW, invH) : -1;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (c[j] >= 0) atomicAdd(&cnt[c[j]], 1);
  }
  __syncthreads();
  // exclusive scan over 3072 cells: 48 consecutive cells per lane
  {
    constexpr int per = GRID_CELLS / 64;
    static_assert(per * 64 == GRID_CELLS && per % 4 == 0, "cells split evenly over the lanes");
    int4* c4 = reinterpret_cast<int4*>(cnt + lane * per);
    int4 v[per / 4];
    int s = 0;
#pragma unroll
    for (int i = 0; i < per / 4; ++i) {
      v[i] = c4[i];
      s += v[i].x + v[i].y + v[i].z + v[i].w;
    }
    int ex = wave_incl_scan(s) - s;
    int4* cs4 = reinterpret_cast<int4*>(cellStart + (size_t)p * (GRID_CELLS + 1));
    const bool al16 = ((uintptr_t)cs4 & 15) == 0;
    int32_t* cs = cellStart + (size_t)p * (GRID_CELLS + 1) + lane * per;
#pragma unroll
    for (int i = 0; i < per / 4; ++i) {
      const int4 e = make_int4(ex, ex + v[i].x, ex + v[i].x + v[i].y, ex + v[i].x + v[i].y + v[i].z);
      ex = e.w + v[i].w;
      c4[i] = e;
      if (al16) {
        reinterpret_cast<int4*>(cs)[i] = e;
      } else {
        cs[4 * i] = e.x;
        cs[4 * i + 1] = e.y;
        cs[4 * i + 2] = e.z;
        cs[4 * i + 3] = e.w;
      }
    }
    if (lane == 63) cellStart[(size_t)p * (GRID_CELLS + 1) + GRID_CELLS] = ex;
  }
  __syncthreads();
  int32_t* ci = cellIdx + (size_t)p * kpStride;
  const uint8_t* LK = locked ? locked + (size_t)p * kpStride : nullptr;
  const float* UR = uright ? uright + (size_t)p * kpStride : nullptr;
  uint4* sg = staged ? staged + (size_t)p * kpStride : nullptr;
  const unsigned long long ltMask = (1ull << lane) - 1ull;
  // round r's fields, loaded one round ahead
  float nx = 0.f, ny = 0.f, nu = -1.f;
  int noct = 0, nlk = 0;
  auto load = [&](int k) {
    if (k < n) {
      nx = K[k].x;
      ny = K[k].y;
      if (sg) {
        noct = K[k].octave;
        nlk = LK ? LK[k] : 0;
        nu = UR ? UR[k] : -1.0f;
      }
    }
  };
  load(lane);
  for (int base = 0; base < n; base += 64) {
    const int k = base + lane;
    const float x = nx, y = ny, u = nu;
    const int oct = noct, lk = nlk;
    load(k + 64);
    int c = -1;
    if (k < n) {
      orb_keypoint_t kp;
      kp.x = x;
      kp.y = y;
      c = grid_cell(kp, minX, minY, invW, invH);
    }
    const int id = c < 0 ? 4095 : c;
    unsigned long long peers = __ballot(1);
#pragma unroll
    for (int bit = 0; bit < 12; ++bit) {
      const unsigned long long m = __ballot((id >> bit) & 1);
      peers &= ((id >> bit) & 1) ? m : ~m;
    }
    int pos = 0;
    if (c >= 0) pos = cnt[c] + __popcll(peers & ltMask);
    __builtin_amdgcn_wave_barrier();
    if (c >= 0) {
      ci[pos] = k;
      if (sg) {
        uint4 e;
        e.x = __float_as_uint(x);
        e.y = __float_as_uint(y);
        e.z = (uint32_t)k | ((uint32_t)oct << 24) | (lk ? 0x80000000u : 0u);
        e.w = __float_as_uint(u);
        sg[pos] = e;
      }
      if ((peers >> lane) == 1ull) cnt[c] += __popcll(peers);  // highest lane of the group
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Four waves per frame for frames with many keypoint slots (C5: 4,000
// keypoints; the one-wave scatter takes 63 dependent rounds there): wave w
// takes the contiguous keys [w n / 4, (w + 1) n / 4).  Per (cell, wave) counts
// ride in u16 halves, two waves per dword (36 KB of LDS with the cell starts),
// the cell starts come from one block scan, and wave w's cursor in cell c is
// the cell's start plus the counts of waves 0..w-1 there, so the four waves
// scatter at once and the lists stay in ascending keypoint order.
#define GB4_MIN_SLOTS 1536  // frames with more keypoint slots take k_grid_build4
__global__ __launch_bounds__(256) void k_grid_build4(const orb_keypoint_t* __restrict__ keys,
                                                     const int32_t* __restrict__ nkeys, int kpStride,
                                                     float minX, float minY, float invW, float invH,
                                                     int32_t* __restrict__ cellStart,
                                                     int32_t* __restrict__ cellIdx,
                                                     const uint8_t* __restrict__ locked,
                                                     const float* __restrict__ uright,
                                                     uint4* __restrict__ staged) {
  __shared__ uint32_t c2[GRID_CELLS][2];  // waves (0, 1) and (2, 3): counts, then cursors
  __shared__ int start[GRID_CELLS];
  __shared__ int tmp[20];
  const int p = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = min(max(nkeys[p], 0), 65535);
  const int kb = (int)((long long)n * w / 4), ke = (int)((long long)n * (w + 1) / 4);
  const int half = w >> 1, sh = 16 * (w & 1);
  const orb_keypoint_t* K = keys + (size_t)p * kpStride;
  for (int i = t; i < GRID_CELLS * 2; i += 256) (&c2[0][0])[i] = 0u;
  __syncthreads();
  for (int base = kb; base < ke; base += 256) {
    int c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = base + 64 * j + lane;
      c[j] = k < ke ? grid_cell(K[k], minX, minY, invW, invH) : -1;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (c[j] >= 0) atomicAdd(&c2[c[j]][half], 1u << sh);
  }
  __syncthreads();
  {
    constexpr int per = GRID_CELLS / 256;
    static_assert(per * 256 == GRID_CELLS, "cells split evenly over the threads");
    int s = 0;
#pragma unroll
    for (int i = 0; i < per; ++i) {
      const uint32_t a = c2[t * per + i][0], b = c2[t * per + i][1];
      s += (int)((a & 0xFFFFu) + (a >> 16) + (b & 0xFFFFu) + (b >> 16));
    }
    int tot;
    int ex = block_excl_scan(s, tmp, &tot);
    int32_t* cs = cellStart + (size_t)p * (GRID_CELLS + 1);
#pragma unroll
    for (int i = 0; i < per; ++i) {
      const int c = t * per + i;
      const uint32_t a = c2[c][0], b = c2[c][1];
      const uint32_t n0 = a & 0xFFFFu, n1 = a >> 16, n2 = b & 0xFFFFu, n3 = b >> 16;
      start[c] = ex;
      cs[c] = ex;
      // wave cursors inside the cell: 0, n0, n0 + n1, n0 + n1 + n2
      c2[c][0] = (n0 << 16);
      c2[c][1] = (n0 + n1) | ((n0 + n1 + n2) << 16);
      ex += (int)(n0 + n1 + n2 + n3);
    }
    if (t == 255) cs[GRID_CELLS] = tot;
  }
  __syncthreads();
  int32_t* ci = cellIdx + (size_t)p * kpStride;
  const uint8_t* LK = locked ? locked + (size_t)p * kpStride : nullptr;
  const float* UR = uright ? uright + (size_t)p * kpStride : nullptr;
  uint4* sg = staged ? staged + (size_t)p * kpStride : nullptr;
  const unsigned long long ltMask = (1ull << lane) - 1ull;
  float nx = 0.f, ny = 0.f, nu = -1.f;
  int noct = 0, nlk = 0;
  auto load = [&](int k) {
    if (k < ke) {
      nx = K[k].x;
      ny = K[k].y;
      if (sg) {
        noct = K[k].octave;
        nlk = LK ? LK[k] : 0;
        nu = UR ? UR[k] : -1.0f;
      }
    }
  };
  load(kb + lane);
  for (int base = kb; base < ke; base += 64) {
    const int k = base + lane;
    const float x = nx, y = ny, u = nu;
    const int oct = noct, lk = nlk;
    load(k + 64);
    int c = -1;
    if (k < ke) {
      orb_keypoint_t kp;
      kp.x = x;
      kp.y = y;
      c = grid_cell(kp, minX, minY, invW, invH);
    }
    const int id = c < 0 ? 4095 : c;
    unsigned long long peers = __ballot(1);
#pragma unroll
    for (int bit = 0; bit < 12; ++bit) {
      const unsigned long long m = __ballot((id >> bit) & 1);
      peers &= ((id >> bit) & 1) ? m : ~m;
    }
    int pos = 0;
    if (c >= 0) pos = start[c] + (int)((c2[c][half] >> sh) & 0xFFFFu) + __popcll(peers & ltMask);
    __builtin_amdgcn_wave_barrier();
    if (c >= 0) {
      ci[pos] = k;
      if (sg) {
        uint4 e;
        e.x = __float_as_uint(x);
        e.y = __float_as_uint(y);
        e.z = (uint32_t)k | ((uint32_t)oct << 24) | (lk ? 0x80000000u : 0u);
        e.w = __float_as_uint(u);
        sg[pos] = e;
      }
      // the group's highest lane advances this wave's cursor (the other half
      // of the dword is another wave's: an atomic add keeps both)
      if ((peers >> lane) == 1ull) atomicAdd(&c2[c][half], (uint32_t)__popcll(peers) << sh);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ------------------------------------------ SearchByProjection(F, localMap)
// Per map point: candidate scan + first-K in (dist, scan order); counts every
// candidate that could ever be best/second (dist < 256, not pre-locked, passes
// the stereo gate).  ncand = -1 marks a point the reference skips outright.
//
// The frame's grid is staged in LDS once per workgroup: cellStart, and the
// keypoints in cell order as {x, y, idx | octave << 24 | locked << 31, uR}
// (the order GetFeaturesInArea visits them), so the scan is LDS-latency bound;
// only the descriptors of window candidates come from global memory.  Frames
// with more than PROJ_STAGE keypoints scan the global grid instead.
#ifndef PROJ_STAGE
#define PROJ_STAGE 4096  // frames with up to this many keypoints are staged (C5: 4000)
#endif

#ifndef PROJ_QB
#define PROJ_QB 4  // window candidates scored per batch of descriptor loads
#endif
#ifndef PROJ_XCD
#define PROJ_XCD 1  // XCD-contiguous workgroup order (A/B knob)
#endif
#ifndef PROJ_WG
#define PROJ_WG 512  // map points per workgroup (grid staged once per workgroup; swept 256-1024)
#endif
// DIRECT: the staged grid and the cell table are read where k_grid_build left
// them (L2-resident: 64 KB + 12 KB per C5 frame, the problem's workgroups
// share one XCD) instead of being copied into LDS by every workgroup; the
// workgroup then holds no LDS and the chip is not limited to two 1024-point
// workgroups per CU
// ncand of the projection matcher: the candidate count, with the point's
// has_obs (a claim by it locks the keypoint) in bit 30, so the resolve reads one
// word per point for both; -1 = not in view / bad
// and (bits 19-29) 1 + the slot of its candidate list (0: none, ProjParams.ovf)
#define NC_OBS 0x40000000
#define NC_SLOT_SHIFT 19
__device__ __forceinline__ int nc_count(int v) { return v < 0 ? v : (v & ((1 << NC_SLOT_SHIFT) - 1)); }
__device__ __forceinline__ bool nc_obs(int v) { return v >= 0 && (v & NC_OBS) != 0; }
__device__ __forceinline__ int nc_slot(int v) { return v < 0 ? -1 : ((v >> NC_SLOT_SHIFT) & 0x7FF) - 1; }
// problem p's list `slot` (nc_slot >= 0 only when ProjParams.ovf is set)
__device__ __forceinline__ const uint32_t* ovf_list(const ProjParams& P, int p, int slot) {
  return P.ovf + ((size_t)p * OVF_SLOTS + slot) * OVF_CAP;
}

// PPT: map points per thread (a workgroup covers WG * PPT points, the grid
// staged once for all of them)
template <int WG, bool DIRECT = false, int PPT = 1>
__global__ __launch_bounds__(WG) void k_proj_candidates(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked, int kpStride,
    const int32_t* __restrict__ nkeys, const orb_mp_track_t* __restrict__ mps,
    const uint8_t* __restrict__ mpDesc, const int32_t* __restrict__ nmps, int mpStride,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx,
    const uint4* __restrict__ stagedGrid, int stageCap, ProjParams P,
    uint32_t* __restrict__ topk, int32_t* __restrict__ ncand) {
  __shared__ int sCS[DIRECT ? 1 : GRID_CELLS + 1];
  extern __shared__ __attribute__((aligned(16))) uint4 sKp[];  // min(kpStride, PROJ_STAGE)
  __shared__ float sScale[ORB_MAX_LEVELS];
  // XCD-contiguous order: a problem's workgroups share one L2, which then
  // serves the staged grid and the frame's descriptors to all of them
  int bx, p;
#if PROJ_XCD
  xcd_swizzle(bx, p);
#else
  bx = blockIdx.x;
  p = blockIdx.y;
#endif
  const int tid = threadIdx.x;
  const int M = nmps[p], N = nkeys[p];
  if (bx * WG * PPT >= M) return;  // whole workgroup idle (uniform)
  const orb_keypoint_t* K = keys + (size_t)p * kpStride;
  const uint8_t* D = desc + (size_t)p * kpStride * 32;
  const uint8_t* LK = locked ? locked + (size_t)p * kpStride : nullptr;
  const float* UR = uright ? uright + (size_t)p * kpStride : nullptr;
  const int32_t* cs = cellStart + (size_t)p * (GRID_CELLS + 1);
  const int32_t* ci = cellIdx + (size_t)p * kpStride;
  const bool staged = DIRECT || N <= stageCap;
#pragma unroll
  for (int i = 0; i < ORB_MAX_LEVELS; ++i)
    if (tid == i) sScale[i] = P.scale[i];
  // the cell table and the cell-ordered keypoints scanned below: LDS copies,
  // or (DIRECT) the global arrays themselves
  const int* gCS = sCS;
  const uint4* gKp = sKp;
  if (DIRECT) {
    gCS = cs;
    gKp = stagedGrid + (size_t)p * kpStride;
  } else if (staged) {
    // (batches of loads issued before their stores: a load-store loop waits
    // one memory latency per iteration)
    const int nInGrid = cs[GRID_CELLS];
    constexpr int CSB = (GRID_CELLS + 1 + WG - 1) / WG;
    int csv[CSB];
#pragma unroll
    for (int k = 0; k < CSB; ++k) csv[k] = cs[min(tid + k * WG, GRID_CELLS)];
#pragma unroll
    for (int k = 0; k < CSB; ++k)
      if (tid + k * WG <= GRID_CELLS) sCS[tid + k * WG] = csv[k];
    if (stagedGrid) {
      const uint4* sg = stagedGrid + (size_t)p * kpStride;
      for (int j0 = 0; j0 < nInGrid; j0 += 4 * WG) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = sg[min(j0 + k * WG + tid, nInGrid - 1)];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (j0 + k * WG + tid < nInGrid) sKp[j0 + k * WG + tid] = v[k];
      }
    } else {
    for (int j = tid; j < nInGrid; j += WG) {
      const int idx = ci[j];
      const orb_keypoint_t kp = K[idx];
      uint4 e;
      e.x = __float_as_uint(kp.x);
      e.y = __float_as_uint(kp.y);
      e.z = (uint32_t)idx | ((uint32_t)kp.octave << 24) | ((LK && LK[idx]) ? 0x80000000u : 0u);
      e.w = __float_as_uint(UR ? UR[idx] : -1.0f);
      sKp[j] = e;
    }
    }
  }
  __syncthreads();
  for (int pk = 0; pk < PPT; ++pk) {
  const int m = (bx * PPT + pk) * WG + tid;
  if (m >= M) break;
  const size_t mg = (size_t)p * mpStride + m;
  const orb_mp_track_t mp = mps[mg];
  if (!mp.in_view || mp.bad) {
    ncand[mg] = -1;
    continue;
  }
  const int lvl = mp.level;
  float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:135-141)
  if (P.th != 1.0f) r *= P.th;
  const float rs = r * sScale[lvl];
  const ulonglong4 q = load_desc(mpDesc + mg * 32);
  Top4 top;
  int count = 0;
  auto visit = [&](int idx, int oct, bool lockd, float ur) {
    if (lockd) return;
    if (ur > 0) {
      const float er = fabsf(mp.proj_xr - ur);
      if (er > rs) return;
    }
    const int dist = hamming256(q, load_desc(D + (size_t)idx * 32));
    if (dist >= 256) return;  // can never become best or second
    ++count;
    top.insert(pack_cand(idx, dist, oct), dist);
  };
  // GetFeaturesInArea (src/Frame.cc:368-424) over the staged grid: fn(idx |
  // octave << 24) for every window keypoint passing the level, lock and stereo
  // tests, in scan order
  auto walk = [&](auto&& fn) {
    const float x = mp.proj_x, y = mp.proj_y;
    const int nMinCellX = max(0, (int)floorf((x - P.minX - rs) * P.invW));
    const int nMaxCellX = min(ORB_GRID_COLS - 1, (int)ceilf((x - P.minX + rs) * P.invW));
    const int nMinCellY = max(0, (int)floorf((y - P.minY - rs) * P.invH));
    const int nMaxCellY = min(ORB_GRID_ROWS - 1, (int)ceilf((y - P.minY + rs) * P.invH));
    if (nMinCellX >= ORB_GRID_COLS || nMaxCellX < 0 || nMinCellY >= ORB_GRID_ROWS || nMaxCellY < 0)
      return;
    const int minL = lvl - 1, maxL = lvl;
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
      for (int iy = nMinCellY; iy <= nMaxCellY; ++iy) {
        const int c = ix * ORB_GRID_ROWS + iy;
        const int e = gCS[c + 1];
        for (int j = gCS[c]; j < e; ++j) {
          const uint4 E = gKp[j];
          const int oct = (int)((E.z >> 24) & 0x7Fu);
          if (oct < minL || oct > maxL) continue;
          const float dx = __uint_as_float(E.x) - x, dy = __uint_as_float(E.y) - y;
          if (!(fabsf(dx) < rs && fabsf(dy) < rs) || (E.z >> 31) != 0) continue;
          const float ur = __uint_as_float(E.w);
          if (ur > 0 && fabsf(mp.proj_xr - ur) > rs) continue;
          fn((E.z & 0xFFFFFFu) | ((uint32_t)oct << 24));
        }
      }
    }
  };
  if (staged) {
    // Window candidates that pass the lock and stereo tests queue up (scan order) and
    // are scored PROJ_QB at a time, so their descriptor loads overlap.
    // the queue lives in registers (qe[k] written through selects, no LDS:
    // C5's staged frame already takes 76 KB of LDS per workgroup)
    int nq = 0;
    uint32_t qe[PROJ_QB];
#pragma unroll
    for (int k = 0; k < PROJ_QB; ++k) qe[k] = 0;
    auto flush = [&](int cnt) {
      ulonglong4 dd[PROJ_QB];
#pragma unroll
      for (int k = 0; k < PROJ_QB; ++k)
        dd[k] = load_desc(D + (size_t)((k < cnt ? qe[k] : qe[0]) & 0xFFFFFFu) * 32);
#pragma unroll
      for (int k = 0; k < PROJ_QB; ++k) {
        if (k >= cnt) break;
        const int dist = hamming256(q, dd[k]);
        if (dist >= 256) continue;  // can never become best or second
        ++count;
        top.insert(pack_cand((int)(qe[k] & 0xFFFFFFu), dist, (int)(qe[k] >> 24)), dist);
      }
    };
    walk([&](uint32_t qv) {
#pragma unroll
      for (int k = 0; k < PROJ_QB; ++k) qe[k] = nq == k ? qv : qe[k];
      if (++nq == PROJ_QB) {
        flush(PROJ_QB);
        nq = 0;
      }
    });
    if (nq) flush(nq);
  } else {
    for_features_in_area(K, cs, ci, P, mp.proj_x, mp.proj_y, rs, lvl - 1, lvl,
                         [&](int idx, const orb_keypoint_t& kp) {
                           visit(idx, kp.octave, LK && LK[idx], UR ? UR[idx] : -1.0f);
                         });
  }
  top.store(topk + mg * TOPK);
  // more candidates than the top-K holds: the whole list, in scan order, for
  // the resolves' re-scan (a second walk of the window; rare: C4's maps have
  // at most 4-6 candidates per point)
  int slot = -1;
  if (count > TOPK && count <= OVF_CAP && P.ovf) {
    slot = ovf_alloc(P.ovfCtr + p, P.gen);
    if (slot >= OVF_SLOTS) slot = -1;
  }
  if (slot >= 0) {
    uint32_t* lst = P.ovf + ((size_t)p * OVF_SLOTS + slot) * OVF_CAP;
    int n = 0;
    auto put = [&](int idx, int oct) {
      const int dist = hamming256(q, load_desc(D + (size_t)idx * 32));
      if (dist < 256 && n < OVF_CAP) lst[n++] = pack_cand(idx, dist, oct);
    };
    if (staged)
      walk([&](uint32_t qv) { put((int)(qv & 0xFFFFFFu), (int)(qv >> 24)); });
    else
      for_features_in_area(K, cs, ci, P, mp.proj_x, mp.proj_y, rs, lvl - 1, lvl,
                           [&](int idx, const orb_keypoint_t& kp) {
                             if ((LK && LK[idx]) || (UR && UR[idx] > 0 && fabsf(mp.proj_xr - UR[idx]) > rs))
                               return;
                             put(idx, kp.octave);
                           });
  }
  ncand[mg] = count | (mp.has_obs ? NC_OBS : 0) | ((slot + 1) << NC_SLOT_SHIFT);
  }
}

// Sequential-semantics resolve, one workgroup per problem, speculatively a
// window of map points at a time: every lane evaluates its point against the claims made so
// far; lane i's result stands unless an earlier lane of the same window claims
// (and locks) a keypoint among the top-K entries lane i looked at.  The longest
// conflict-free prefix is committed, the window restarts after it.  A point
// whose top-K ran dry (more than K candidates, too many claimed) is re-scanned
// exactly once it is first in its window.
__device__ __forceinline__ bool lock_test(const uint32_t* bm, int idx) {
  return (bm[idx >> 5] >> (idx & 31)) & 1u;
}

// A window is 64 * NW points (NW waves of one workgroup per problem): every
// thread evaluates its point, claims are resolved across the whole window in
// LDS (earliest claiming thread per keypoint), and the longest conflict-free
// prefix over all waves is committed.  NW = 1 is one wave per problem; wider
// windows cut the number of sequential rounds for large local maps.

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_proj_resolve(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked,
    const int32_t* __restrict__ nkeys, int kpStride, const orb_mp_track_t* __restrict__ mps,
    const uint8_t* __restrict__ mpDesc, const int32_t* __restrict__ nmps, int mpStride,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, ProjParams P,
    const uint32_t* __restrict__ topk, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ kpMatch, int32_t* __restrict__ nmatches) {
  constexpr int W = 64 * NW, CHUNK = 256 * NW;
  // LDS: lock bitmap (1 bit / keypoint), earliest claiming thread per keypoint
  // of the current window, and a prefetched chunk of per-point resolve inputs
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ uint4 cTop[CHUNK];
  __shared__ int cN[CHUNK];
  __shared__ uint8_t cObs[CHUNK];
  __shared__ int sFirst[NW], sCount[NW];
  __shared__ int sSlow;
  const int p = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = nkeys[p], M = nmps[p];
  const int words = (kpStride + 31) >> 5;
  uint32_t* bm = dyn;
  int* claimBy = (int*)(dyn + ((words + 3) & ~3));
  for (int i = t; i < words; i += W) bm[i] = 0u;
  for (int i = t; i < kpStride; i += W) claimBy[i] = W;
  int32_t* km = kpMatch + (size_t)p * kpStride;
  for (int i = t; i < n; i += W) km[i] = -1;
  __syncthreads();
  const float nnratio = P.nnratio;
  const size_t pbase = (size_t)p * mpStride;
  int matches = 0;  // this wave's committed accepts
  int start = 0;
  int cb = -CHUNK;  // first point held in the LDS chunk
  while (start < M) {
    if (start + W > cb + CHUNK && cb + CHUNK < M) {  // slide the chunk to `start`
      cb = start;
      __syncthreads();
      for (int j = t; j < CHUNK; j += W) {
        const int m = cb + j;
        if (m < M) {
          cTop[j] = *reinterpret_cast<const uint4*>(topk + (pbase + m) * TOPK);
          const int v = ncand[pbase + m];
          cN[j] = v;  // raw: count, obs, list slot
          cObs[j] = nc_obs(v);
        }
      }
      __syncthreads();
    }
    const int m = start + t;
    const bool active = m < M;
    int nc = -1, ncRaw = -1;
    uint32_t e[TOPK];
    bool hasObs = false;
    if (active) {
      const int j = m - cb;
      ncRaw = cN[j];
      nc = nc_count(ncRaw);
      const uint4 t4 = cTop[j];
      e[0] = t4.x; e[1] = t4.y; e[2] = t4.z; e[3] = t4.w;
      hasObs = cObs[j] != 0;
    }
    // evaluate against the current locks
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    int consumed = 0, found = 0;
    if (nc > 0) {
      const int avail = nc < TOPK ? nc : TOPK;
      for (int j = 0; j < avail && found < 2; ++j) {
        ++consumed;
        const int idx = cand_idx(e[j]);
        if (lock_test(bm, idx)) continue;
        if (found == 0) {
          bestDist = cand_dist(e[j]);
          bestLevel = cand_oct(e[j]);
          bestIdx = idx;
        } else {
          bestDist2 = cand_dist(e[j]);
          bestLevel2 = cand_oct(e[j]);
        }
        ++found;
      }
    }
    const bool slow = nc > TOPK && found < 2;
    const int slowSlot = nc_slot(ncRaw);
    bool accept = false;
    if (nc > 0 && !slow && bestDist <= 100)
      accept = !(bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2);
    const bool locks = accept && hasObs;
    // conflict: an earlier thread of this window locks a keypoint this one looked at
    if (locks) atomicMin(&claimBy[bestIdx], t);
    __syncthreads();
    bool conflict = false;
    for (int q = 0; q < consumed; ++q) conflict |= claimBy[cand_idx(e[q])] < t;
    const unsigned long long bad = __ballot(active && (conflict || (slow && t > 0)));
    if (lane == 0) sFirst[wv] = bad ? wv * 64 + (int)__builtin_ctzll(bad) : W;
    if (t == 0) sSlow = active && slow;
    __syncthreads();
    if (locks) claimBy[bestIdx] = W;
    int commit = W;
#pragma unroll
    for (int i = 0; i < NW; ++i) commit = min(commit, sFirst[i]);
    if (sSlow) {
      // exact re-scan of the first point of the window, thread 0, current locks
      if (t == 0 && slowSlot >= 0) {  // the point's candidate list (scan order)
        const uint32_t* lst = ovf_list(P, p, slowSlot);
        int bd = 256, bl = -1, bd2 = 256, bl2 = -1, bi = -1;
        for (int j = 0; j < nc; ++j) {
          const uint32_t ce = lst[j];
          const int idx = cand_idx(ce);
          if (lock_test(bm, idx)) continue;
          const int dist = cand_dist(ce);
          if (dist < bd) {
            bd2 = bd; bd = dist; bl2 = bl; bl = cand_oct(ce); bi = idx;
          } else if (dist < bd2) {
            bl2 = cand_oct(ce); bd2 = dist;
          }
        }
        if (bd <= 100 && !(bl == bl2 && (float)bd > nnratio * (float)bd2)) {
          atomicMax(&km[bi], m);
          if (cObs[m - cb]) bm[bi >> 5] |= 1u << (bi & 31);
          ++matches;
        }
      } else if (t == 0) {
        const size_t mg = pbase + m;
        const orb_mp_track_t mp = mps[mg];
        const int lvl = mp.level;
        float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;
        if (P.th != 1.0f) r *= P.th;
        const float rs = r * P.scale[lvl];
        const orb_keypoint_t* K = keys + (size_t)p * kpStride;
        const uint8_t* D = desc + (size_t)p * kpStride * 32;
        const uint8_t* LK = locked ? locked + (size_t)p * kpStride : nullptr;
        const float* UR = uright ? uright + (size_t)p * kpStride : nullptr;
        const ulonglong4 qd = load_desc(mpDesc + mg * 32);
        int bd = 256, bl = -1, bd2 = 256, bl2 = -1, bi = -1;
        for_features_in_area(K, cellStart + (size_t)p * (GRID_CELLS + 1),
                             cellIdx + (size_t)p * kpStride, P, mp.proj_x, mp.proj_y, rs,
                             lvl - 1, lvl, [&](int idx, const orb_keypoint_t& kp) {
                               if ((LK && LK[idx]) || lock_test(bm, idx)) return;
                               if (UR && UR[idx] > 0) {
                                 const float er = fabsf(mp.proj_xr - UR[idx]);
                                 if (er > r * P.scale[lvl]) return;
                               }
                               const int dist = hamming256(qd, load_desc(D + (size_t)idx * 32));
                               if (dist < bd) {
                                 bd2 = bd; bd = dist; bl2 = bl; bl = kp.octave; bi = idx;
                               } else if (dist < bd2) {
                                 bl2 = kp.octave; bd2 = dist;
                               }
                             });
        if (bd <= 100 && !(bl == bl2 && (float)bd > nnratio * (float)bd2)) {
          atomicMax(&km[bi], m);
          if (mp.has_obs) bm[bi >> 5] |= 1u << (bi & 31);
          ++matches;
        }
      }
      commit = 1;
    } else {
      if (t < commit && accept) {
        atomicMax(&km[bestIdx], m);
        if (locks) atomicOr(&bm[bestIdx >> 5], 1u << (bestIdx & 31));
      }
      matches += __popcll(__ballot(t < commit && accept));
    }
    __syncthreads();  // this round's locks before the next window's evaluation
    start += commit;
  }
  if (lane == 0) sCount[wv] = matches;
  __syncthreads();
  if (t == 0) {
    int tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) tot += sCount[i];
    nmatches[p] = tot;
  }
}


// Barrier ordering LDS only: global stores and atomics still in flight (the
// fire-and-forget kpMatch updates, the next window's prefetch) are not waited
// for, unlike __syncthreads().
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The exact scan of a point whose top-K ran dry (more than K candidates, too
// many of them taken): GetFeaturesInArea under the same "taken" test.  Not
// inlined: its global loads would otherwise sit inside k_proj_resolve_fp's
// round loop, and the compiler's wait for them at the loop head (one vmcnt
// counter, in order) also waited for the next windows' inputs in flight; as
// a call the waits stay on the (rare: never in C5) path that takes it.
__device__ __noinline__ int fp_slow(int m, const int* cur, const orb_mp_track_t* mpp,
                                    const uint8_t* mpd, const orb_keypoint_t* K, const uint8_t* D,
                                    const uint8_t* LK, const float* UR, const int32_t* cs,
                                    const int32_t* ci, const ProjParams P, const uint32_t* lst,
                                    int nl) {
  // (P by value: a reference would put the caller's copy in scratch memory
  // and every fp_choose would read nnratio from there)
  if (lst) {  // the point's candidate list (scan order; static tests applied)
    uint32_t e[OVF_CAP];
#pragma unroll
    for (int j = 0; j < OVF_CAP; j += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(lst + j);
      e[j] = v.x; e[j + 1] = v.y; e[j + 2] = v.z; e[j + 3] = v.w;
    }
    // every claim read issued before any is used (entries past nl read entry
    // 0's keypoint and are ignored): one memory round trip
    int cv[OVF_CAP];
#pragma unroll
    for (int j = 0; j < OVF_CAP; ++j) cv[j] = cur[cand_idx(j < nl ? e[j] : e[0])];
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
#pragma unroll
    for (int j = 0; j < OVF_CAP; ++j) {
      if (j >= nl || cv[j] < m) continue;
      const int dist = cand_dist(e[j]);
      if (dist < bestDist) {
        bestDist2 = bestDist; bestDist = dist;
        bestLevel2 = bestLevel; bestLevel = cand_oct(e[j]); bestIdx = cand_idx(e[j]);
      } else if (dist < bestDist2) {
        bestLevel2 = cand_oct(e[j]); bestDist2 = dist;
      }
    }
    const bool accept = bestIdx >= 0 && bestDist <= 100 &&
                        !(bestLevel == bestLevel2 && (float)bestDist > P.nnratio * (float)bestDist2);
    return accept ? bestIdx : -1;
  }
  const orb_mp_track_t mp = *mpp;
  const int lvl = mp.level;
  float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;
  if (P.th != 1.0f) r *= P.th;
  const float rs = r * P.scale[lvl];
  const ulonglong4 qd = load_desc(mpd);
  int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
  for_features_in_area(K, cs, ci, P, mp.proj_x, mp.proj_y, rs, lvl - 1, lvl,
                       [&](int idx, const orb_keypoint_t& kp) {
                         if ((LK && LK[idx]) || cur[idx] < m) return;
                         if (UR && UR[idx] > 0) {
                           const float er = fabsf(mp.proj_xr - UR[idx]);
                           if (er > rs) return;
                         }
                         const int dist = hamming256(qd, load_desc(D + (size_t)idx * 32));
                         if (dist < bestDist) {
                           bestDist2 = bestDist; bestDist = dist;
                           bestLevel2 = bestLevel; bestLevel = kp.octave; bestIdx = idx;
                         } else if (dist < bestDist2) {
                           bestLevel2 = kp.octave; bestDist2 = dist;
                         }
                       });
  const bool accept = bestIdx >= 0 && bestDist <= 100 &&
                      !(bestLevel == bestLevel2 && (float)bestDist > P.nnratio * (float)bestDist2);
  return accept ? bestIdx : -1;
}

// One point's SearchByProjection decision (src/ORBmatcher.cc:83-132) with
// "keypoint k taken before point m" = cur[k] < m (committed locks are -1,
// claims of the current window hold the claiming point): the keypoint it
// takes, or -1.
__device__ __forceinline__ int fp_choose(const uint32_t (&e)[TOPK], int nc, int m, const int* cur,
                                         const orb_mp_track_t* mpp, const uint8_t* mpd,
                                         const orb_keypoint_t* K, const uint8_t* D,
                                         const uint8_t* LK, const float* UR, const int32_t* cs,
                                         const int32_t* ci, const ProjParams& P,
                                         const uint32_t* lst) {
  int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
  int found = 0;
  const int avail = nc < TOPK ? nc : TOPK;
  // every claim read issued before any is used (unused slots read entry 0's
  // keypoint again): one memory round trip, not one per candidate -- the
  // claims are LDS in k_proj_resolve_fp but global memory in k_proj_jacobi
  int cv[TOPK];
#pragma unroll
  for (int j = 0; j < TOPK; ++j) cv[j] = cur[cand_idx(j < avail ? e[j] : e[0])];
  bool taken[TOPK];
#pragma unroll
  for (int j = 0; j < TOPK; ++j) taken[j] = j < avail ? cv[j] < m : true;
#pragma unroll
  for (int j = 0; j < TOPK; ++j) {
    const bool use = found < 2 && !taken[j];
    if (use && found == 0) {
      bestDist = cand_dist(e[j]); bestLevel = cand_oct(e[j]); bestIdx = cand_idx(e[j]);
    } else if (use) {
      bestDist2 = cand_dist(e[j]); bestLevel2 = cand_oct(e[j]);
    }
    found += use ? 1 : 0;
  }
  // top-K ran dry: exact scan of the point's area under the same locks
  if (nc > TOPK && found < 2) return fp_slow(m, cur, mpp, mpd, K, D, LK, UR, cs, ci, P, lst, nc);
  const bool accept = bestIdx >= 0 && bestDist <= 100 &&
                      !(bestLevel == bestLevel2 && (float)bestDist > P.nnratio * (float)bestDist2);
  return accept ? bestIdx : -1;
}

// Fixed-point resolve for large local maps: a window of 1024 points (one per
// thread) is iterated to the sequential result instead of being committed
// prefix by prefix.  Each round every point re-decides with "taken" = a
// committed lock or a claim by an earlier point of the window in the previous
// round's choices, and claims (atomicMin of its index) the keypoint it locks.
// The sequential result is the unique fixed point (the smallest point whose
// choice differs from it sees a correct claim set and becomes correct next
// round), so the loop ends after at most one round per point; C5 windows
// settle in 2.2 rounds on average (tools/r04/c5_stats.cpp: the deepest claim
// chain of a 1024-point window is 0.5 on average, 2 at most, and no C5 point
// ever needs more than its top 4 candidates).  Claims are double-buffered
// (round r reads buffer (r-1)&1, writes r&1); a committed lock is -1 in both
// buffers.  Every memory access of the window loop is LDS: the inputs of the
// windows two and three ahead are loaded while the current one iterates
// (FP_AHEAD), and the keypoint -> point result (kpMatch) is kept in LDS and
// written out once at the end, so no wait on a global access (loads, or the
// kpMatch atomics, which share the in-order vmcnt counter with the loads on
// gfx9) sits inside the loop; rounds synchronise on LDS only.
#ifndef FP_AHEAD
#define FP_AHEAD 2  // windows of inputs in flight ahead of the current one (1 or 2)
#endif
#ifndef FP_DEBUG
#define FP_DEBUG 0  // diagnostic build: per-window rounds and clock stamps of problem 0
#endif
#if FP_DEBUG
// [0] windows, then per window: rounds, cycles (s_memtime) at its end
__device__ unsigned long long g_fp_dbg[2 + 2 * 256];
extern "C" hipError_t orb_k_fp_debug(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fp_dbg), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif
// PPT points per thread: a window of T * PPT points
template <int T, int PPT = 1>
__global__ __launch_bounds__(T) void k_proj_resolve_fp(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked,
    const int32_t* __restrict__ nkeys, int kpStride, const orb_mp_track_t* __restrict__ mps,
    const uint8_t* __restrict__ mpDesc, const int32_t* __restrict__ nmps, int mpStride,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, ProjParams P,
    const uint32_t* __restrict__ topk, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ kpMatch, int32_t* __restrict__ nmatches,
    const int32_t* __restrict__ done, long long doneStride) {
  constexpr int NOCLAIM = 0x7FFFFFFF;
  // 2 x kpStride claims, kpStride kpMatch
  extern __shared__ __attribute__((aligned(16))) int claims[];
  __shared__ int sCount[T / 64];
  __shared__ int sChanged[2];
  const int p = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // after the Jacobi rounds (k_proj_jacobi): only problems they left unsettled
  if (done && done[(long long)p * doneStride] != 0) return;
  const int n = nkeys[p], M = nmps[p];
  int* skm = claims + 2 * kpStride;
  if (t < 2) sChanged[t] = 0;
  for (int i = t; i < 2 * kpStride; i += T) claims[i] = NOCLAIM;
  for (int i = t; i < n; i += T) skm[i] = -1;
  const size_t pbase = (size_t)p * mpStride;
  const orb_keypoint_t* K = keys + (size_t)p * kpStride;
  const uint8_t* D = desc + (size_t)p * kpStride * 32;
  const uint8_t* LK = locked ? locked + (size_t)p * kpStride : nullptr;
  const float* UR = uright ? uright + (size_t)p * kpStride : nullptr;
  const int32_t* cs = cellStart + (size_t)p * (GRID_CELLS + 1);
  const int32_t* ci = cellIdx + (size_t)p * kpStride;
  int matches = 0;
  // inputs of the windows ahead (A: next, B: the one after)
  struct In {
    uint4 e;
    int nc;  // count | NC_OBS
  };
  // issued by every lane on every path (index clamped, the count masked
  // after the wait): the compiler then counts the loads in flight exactly and
  // waits for a window's inputs only, not for the later windows' too
  auto load = [&](In& in, int m) {
    const size_t mg = pbase + (size_t)max(0, min(m, M - 1));
    in.e = *reinterpret_cast<const uint4*>(topk + mg * TOPK);
    in.nc = ncand[mg];
  };
  constexpr int W = T * PPT;  // points per window
  In inA[PPT], inB[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) load(inA[k], k * T + t);
#if FP_AHEAD > 1
  asm volatile("" ::: "memory");  // A's loads all issue before B's (in-order counts)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < PPT; ++k) load(inB[k], W + k * T + t);
#endif
  __syncthreads();  // LDS reset before any window's claims
  int round = 0;  // global round counter: buffer parity and change flags
#if FP_DEBUG
  int dbgW = 0;
  if (p == 0 && t == 0) g_fp_dbg[1] = __builtin_amdgcn_s_memtime();
#endif
  // one window: its inputs leave `in` (loaded FP_AHEAD windows earlier) and
  // `in` is reloaded with the inputs FP_AHEAD windows on
  auto window = [&](int start, In (&in)[PPT]) {
    uint32_t e[PPT][TOPK];
    int nc[PPT], prev[PPT], acc[PPT];
    const uint32_t* lst[PPT];
    bool obs[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int m = start + k * T + t;
      e[k][0] = in[k].e.x; e[k][1] = in[k].e.y; e[k][2] = in[k].e.z; e[k][3] = in[k].e.w;
      nc[k] = m < M ? nc_count(in[k].nc) : -1;
      const int sl = m < M ? nc_slot(in[k].nc) : -1;
      lst[k] = sl >= 0 ? ovf_list(P, p, sl) : nullptr;
      obs[k] = m < M && nc_obs(in[k].nc);
      prev[k] = -1;  // this point's claim in the previous round
      acc[k] = -1;
    }
    while (true) {
      const int* cur = claims + ((round + 1) & 1) * kpStride;
      int* nxt = claims + (round & 1) * kpStride;
      bool changed = false;
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const int m = start + k * T + t;
        acc[k] = nc[k] > 0 ? fp_choose(e[k], nc[k], m, cur, mps + pbase + m, mpDesc + (pbase + m) * 32,
                                       K, D, LK, UR, cs, ci, P, lst[k])
                           : -1;
        const int claim = obs[k] ? acc[k] : -1;
        if (claim >= 0) atomicMin(&nxt[claim], m);
        changed |= claim != prev[k];
      }
      if (__ballot(changed) != 0ull && lane == 0) sChanged[round & 1] = 1;
      lds_barrier();
      const bool any = sChanged[round & 1] != 0;
      if (t == 0) sChanged[(round + 1) & 1] = 0;  // next written after the barrier below
      // cur is not read any more: drop these points' claims of the previous
      // round from it, it collects the next round's claims
#pragma unroll
      for (int k = 0; k < PPT; ++k)
        if (prev[k] >= 0) claims[((round + 1) & 1) * kpStride + prev[k]] = NOCLAIM;
      ++round;
      if (!any) break;  // (uniform) claims stable: the window is at its fixed point
#pragma unroll
      for (int k = 0; k < PPT; ++k) prev[k] = obs[k] ? acc[k] : -1;
      lds_barrier();
    }
    // commit: the final claims become committed locks in both buffers
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      if (acc[k] >= 0) {
        atomicMax(&skm[acc[k]], start + k * T + t);
        if (obs[k]) {
          claims[acc[k]] = -1;
          claims[kpStride + acc[k]] = -1;
        }
        ++matches;
      }
    }
    // reloaded only now, when this window's inputs are dead: the loads land in
    // the registers they came from (no copy, so no wait for them before the
    // window that uses them)
#pragma unroll
    for (int k = 0; k < PPT; ++k) load(in[k], start + FP_AHEAD * W + k * T + t);
    lds_barrier();
#if FP_DEBUG
    if (p == 0 && t == 0 && dbgW < 256) {
      g_fp_dbg[2 + 2 * dbgW] = (unsigned long long)round;
      g_fp_dbg[3 + 2 * dbgW] = __builtin_amdgcn_s_memtime();
      g_fp_dbg[0] = (unsigned long long)(dbgW + 1);
    }
    ++dbgW;
#endif
  };
#if FP_AHEAD > 1
  for (int start = 0; start < M; start += 2 * W) {
    window(start, inA);
    window(start + W, inB);  // (past M: one round in which nothing changes)
  }
#else
  for (int start = 0; start < M; start += W) window(start, inA);
#endif
  int32_t* km = kpMatch + (size_t)p * kpStride;
  for (int i = t; i < n; i += T) km[i] = skm[i];
  matches = wave_sum(matches);
  if (lane == 0) sCount[wv] = matches;
  __syncthreads();
  if (t == 0) {
    int tot = 0;
#pragma unroll
    for (int i = 0; i < T / 64; ++i) tot += sCount[i];
    nmatches[p] = tot;
  }
}


// Jacobi resolve for large local maps (C5: 16 problems x 50,000 points): the
// fixed-point iteration of k_proj_resolve_fp taken over a whole problem at
// once and spread over the chip, one launch per round.  Round r: every point
// m re-decides with "keypoint k taken" = claims_{r-1}[k] < m (the smallest
// point that claimed k with observations in round r-1), stores its decision,
// and claims its locking choice in claims_r (atomicMin).  The sequential
// result is the unique fixed point (point 0 decides alone; point m's decision
// depends only on earlier points'), so once a round changes no claim its
// decisions are final: the next launch commits them (kpMatch = the last
// accepting point, atomicMax) and marks the problem done.  Three claim
// buffers rotate (round r reads r-1, writes r, clears r+1, which round r-2
// wrote and round r-1 read).  The launch sequence is fixed (rounds 0..R-1, a
// commit-only launch R, then k_proj_resolve_fp for the problems not done), so
// the result is exact however many rounds a problem needs.
// Scratch per problem: flags[0..R) "round r changed a claim", flags[R] done,
// three claim buffers of kpStride, the decisions (mpStride).
__host__ __device__ inline long long jacobi_claims_off() { return 64; }
__host__ __device__ inline long long jacobi_stride(int kpStride, int mpStride) {
  return (jacobi_claims_off() + 3LL * kpStride + mpStride + 63) & ~63LL;
}
#define JAC_T 256
__global__ __launch_bounds__(JAC_T) void k_proj_jacobi_init(int32_t* __restrict__ scr, long long stride,
                                                         int kpStride, int R,
                                                         const int32_t* __restrict__ nkeys,
                                                         int32_t* __restrict__ kpMatch,
                                                         int32_t* __restrict__ nmatches) {
  const int p = blockIdx.y, i = blockIdx.x * JAC_T + threadIdx.x;
  int32_t* S = scr + (long long)p * stride;
  if (i <= R) S[i] = 0;
  if (i < 3 * kpStride) S[jacobi_claims_off() + i] = 0x7FFFFFFF;
  if (i < kpStride && i < nkeys[p]) kpMatch[(long long)p * kpStride + i] = -1;
  if (i == 0) nmatches[p] = 0;
}

// PPT points per thread (m = (blockIdx.x * PPT + k) * JAC_T + t): C5's 16 x
// 50,000 points in 784 workgroups, every one resident at once.  Every global
// read a round needs (the problem's flags, the points' counts, top-K and
// previous decisions) is issued before any of them is used, so a workgroup
// pays one memory latency, then the claim reads, then the stores.
#ifndef JAC_PPT
#define JAC_PPT 4
#endif
template <int PPT>
__global__ __launch_bounds__(JAC_T) void k_proj_jacobi(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked,
    int kpStride, const orb_mp_track_t* __restrict__ mps,
    const uint8_t* __restrict__ mpDesc, const int32_t* __restrict__ nmps, int mpStride,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, ProjParams P,
    const uint32_t* __restrict__ topk, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ kpMatch, int32_t* __restrict__ nmatches, int32_t* __restrict__ scr,
    long long stride, int r, int R) {
  __shared__ int sCnt[JAC_T / 64];
  const int p = blockIdx.y, t = threadIdx.x, lane = t & 63;
  const int M = nmps[p];
  int32_t* S = scr + (long long)p * stride;
  int32_t* claims = S + jacobi_claims_off();
  int32_t* dec = claims + 3LL * kpStride;
  const size_t pbase = (size_t)p * mpStride;
  // every load up front (indices clamped: no branch between them)
  const int done = S[R];
  const int prevChanged = r >= 1 ? S[r - 1] : 1;
  int ncv[PPT], old[PPT];
  uint4 q[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int m = (blockIdx.x * PPT + k) * JAC_T + t;
    const size_t mg = pbase + (size_t)max(0, min(m, M - 1));
    ncv[k] = ncand[mg];
    q[k] = *reinterpret_cast<const uint4*>(topk + mg * TOPK);
    old[k] = r > 0 ? dec[mg - pbase] : -1;
  }
  // S[R] = the launch that committed the problem, + 1: an earlier launch's
  // commit ends the problem; a commit by another workgroup of this launch
  // does not (this workgroup's points are still to be committed)
  if (done != 0 && done != r + 1) return;
  if (r >= 1 && prevChanged == 0) {
    // round r-1 changed no claim: its decisions are the sequential result
    int c = 0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int m = (blockIdx.x * PPT + k) * JAC_T + t;
      const int acc = m < M ? old[k] : -1;
      if (acc >= 0) atomicMax(&kpMatch[(size_t)p * kpStride + acc], m);
      c += __popcll(__ballot(acc >= 0));
    }
    if (lane == 0) sCnt[t >> 6] = c;
    __syncthreads();
    if (t == 0) {
      int tot = 0;
#pragma unroll
      for (int i = 0; i < JAC_T / 64; ++i) tot += sCnt[i];
      if (tot) atomicAdd(&nmatches[p], tot);
      S[R] = r + 1;
    }
    return;
  }
  if (r >= R) return;  // commit-only launch, problem still changing: k_proj_resolve_fp
  const int* cur = claims + (long long)((r + 2) % 3) * kpStride;
  int* nxt = claims + (long long)(r % 3) * kpStride;
  int* clr = claims + (long long)((r + 1) % 3) * kpStride;
  for (int i = blockIdx.x * JAC_T + t; i < kpStride; i += gridDim.x * JAC_T) clr[i] = 0x7FFFFFFF;
  bool changed = false;
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int m = (blockIdx.x * PPT + k) * JAC_T + t;
    if (m >= M) continue;
    const int nc = nc_count(ncv[k]);
    const bool hasObs = nc_obs(ncv[k]);
    int acc = -1;
    if (nc > 0) {
      const uint32_t e[TOPK] = {q[k].x, q[k].y, q[k].z, q[k].w};
      const int sl = nc_slot(ncv[k]);
      acc = fp_choose(e, nc, m, cur, mps + pbase + m, mpDesc + (pbase + m) * 32,
                      keys + (size_t)p * kpStride, desc + (size_t)p * kpStride * 32,
                      locked ? locked + (size_t)p * kpStride : nullptr,
                      uright ? uright + (size_t)p * kpStride : nullptr,
                      cellStart + (size_t)p * (GRID_CELLS + 1), cellIdx + (size_t)p * kpStride, P,
                      sl >= 0 ? ovf_list(P, p, sl) : nullptr);
    }
    dec[m] = acc;
    const bool obs = acc >= 0 && hasObs;
    if (obs) atomicMin(&nxt[acc], m);
    const int oldClaim = (old[k] >= 0 && hasObs) ? old[k] : -1;
    changed |= (obs ? acc : -1) != oldClaim;
  }
  if (__ballot(changed) != 0ull && lane == 0) S[r] = 1;
}

// ------------------------------------------------------------ host launchers
extern "C" {

hipError_t orb_k_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hamming_batch, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

// k_grid_build4 (four waves) for frames with more keypoint slots than
// GB4_MIN_SLOTS and for calls of a few frames (the one-wave build's serial
// scatter is the latency of a one-frame call: 20 us of its 70 us
// SearchByProjection, profiles/r05_latency.txt); the one-wave k_grid_build
// for batches of small frames, where a wave per frame fills the chip
#define GB4_FEW 16
static bool grid4(int kpStride, int nproblems) {
  return kpStride < 65536 && (kpStride > GB4_MIN_SLOTS || nproblems <= GB4_FEW);
}

hipError_t orb_k_grid_build(const orb_keypoint_t* keys, const int32_t* nkeys, int kpStride,
                            float minX, float minY, float invW, float invH, int32_t* cellStart,
                            int32_t* cellIdx, int nproblems, hipStream_t s) {
  if (grid4(kpStride, nproblems))
    hipLaunchKernelGGL(k_grid_build4, dim3(nproblems), dim3(256), 0, s, keys, nkeys, kpStride, minX,
                       minY, invW, invH, cellStart, cellIdx, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL(k_grid_build, dim3(nproblems), dim3(64), 0, s, keys, nkeys, kpStride, minX,
                       minY, invW, invH, cellStart, cellIdx, nullptr, nullptr, nullptr);
  return hipGetLastError();
}

// grid + the cell-ordered staging copy for k_proj_candidates (16 B per
// keypoint slot); returns hipErrorNotSupported beyond GB_LDS_KEYS keypoint slots
hipError_t orb_k_grid_build_staged(const orb_keypoint_t* keys, const int32_t* nkeys,
                                   const uint8_t* locked, const float* uright, int kpStride,
                                   float minX, float minY, float invW, float invH,
                                   int32_t* cellStart, int32_t* cellIdx, void* staged,
                                   int nproblems, hipStream_t s) {
  if (kpStride > GB_LDS_KEYS) return hipErrorNotSupported;
  if (grid4(kpStride, nproblems))
    hipLaunchKernelGGL(k_grid_build4, dim3(nproblems), dim3(256), 0, s, keys, nkeys, kpStride, minX,
                       minY, invW, invH, cellStart, cellIdx, locked, uright, (uint4*)staged);
  else
    hipLaunchKernelGGL(k_grid_build, dim3(nproblems), dim3(64), 0, s, keys, nkeys, kpStride, minX,
                       minY, invW, invH, cellStart, cellIdx, locked, uright, (uint4*)staged);
  return hipGetLastError();
}

int orb_k_grid_stage_max(void) { return GB_LDS_KEYS; }

// Compile-time variants of the candidate scan (tools/build_variant.sh; the
// default build instantiates only the defaults):
//   PROJ_DIRECT 1     scan the staged grid in global memory (no LDS copy)
//   PROJ_PPT_LARGE 2  two map points per thread for large maps
#ifndef PROJ_DIRECT
#define PROJ_DIRECT 0
#endif
#ifndef PROJ_PPT_LARGE
#define PROJ_PPT_LARGE 1
#endif
#ifndef PROJ_PPT_SMALL
#define PROJ_PPT_SMALL 1  // map points per thread of the candidate scan for maps under PROJ_LARGE_MAP
#endif
// large problems (C5: 4,000 keypoints staged = 64 KB of LDS per workgroup,
// 50,000 points) take 1024-point workgroups: half the staging per point
#define PROJ_LARGE_MAP 20000

hipError_t orb_k_proj_candidates(const orb_keypoint_t* keys, const uint8_t* desc,
                                 const float* uright, const uint8_t* locked, int kpStride,
                                 const int32_t* nkeys, const orb_mp_track_t* mps,
                                 const uint8_t* mpDesc,
                                 const int32_t* nmps, int mpStride, int mpMax,
                                 const int32_t* cellStart, const int32_t* cellIdx,
                                 const void* stagedGrid, const void* params, uint32_t* topk,
                                 int32_t* ncand, int nproblems, hipStream_t s) {
  const ProjParams P = *(const ProjParams*)params;
  if (mpMax <= 0 || nproblems <= 0) return hipSuccess;
  // dynamic LDS: the staged keypoints of a frame, sized to the key capacity
  const int stageCap = std::min(kpStride, PROJ_STAGE);
  const bool large = stageCap > 2048 && mpMax >= PROJ_LARGE_MAP;
  const bool direct = PROJ_DIRECT && stagedGrid;
  const size_t lds = direct ? 0 : (size_t)stageCap * sizeof(uint4);
  const void* fn;
  dim3 grid;
  int wg;
  if (large) {
    constexpr int ppt = PROJ_DIRECT ? 1 : PROJ_PPT_LARGE;
    fn = direct ? (const void*)k_proj_candidates<1024, true> : (const void*)k_proj_candidates<1024, false, ppt>;
    grid = dim3((mpMax + 1024 * (direct ? 1 : ppt) - 1) / (1024 * (direct ? 1 : ppt)), nproblems);
    wg = 1024;
  } else {
    fn = direct ? (const void*)k_proj_candidates<PROJ_WG, true>
                : (const void*)k_proj_candidates<PROJ_WG, false, PROJ_PPT_SMALL>;
    const int per = PROJ_WG * (direct ? 1 : PROJ_PPT_SMALL);
    grid = dim3((mpMax + per - 1) / per, nproblems);
    wg = PROJ_WG;
  }
  if (lds > 65536 - (GRID_CELLS + 1) * 4 - 64) {  // with the static grid table
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const uint4* sg = (const uint4*)stagedGrid;
  if (large && direct)
    hipLaunchKernelGGL((k_proj_candidates<1024, true>), grid, dim3(wg), lds, s, keys, desc, uright,
                       locked, kpStride, nkeys, mps, mpDesc, nmps, mpStride, cellStart, cellIdx, sg,
                       stageCap, P, topk, ncand);
  else if (large)
    hipLaunchKernelGGL((k_proj_candidates<1024, false, PROJ_PPT_LARGE>), grid, dim3(wg), lds, s, keys,
                       desc, uright, locked, kpStride, nkeys, mps, mpDesc, nmps, mpStride, cellStart,
                       cellIdx, sg, stageCap, P, topk, ncand);
  else if (direct)
    hipLaunchKernelGGL((k_proj_candidates<PROJ_WG, true>), grid, dim3(wg), lds, s, keys, desc, uright,
                       locked, kpStride, nkeys, mps, mpDesc, nmps, mpStride, cellStart, cellIdx, sg,
                       stageCap, P, topk, ncand);
  else
    hipLaunchKernelGGL((k_proj_candidates<PROJ_WG, false, PROJ_PPT_SMALL>), grid, dim3(wg), lds, s, keys,
                       desc, uright, locked, kpStride, nkeys, mps, mpDesc, nmps, mpStride, cellStart,
                       cellIdx, sg, stageCap, P, topk, ncand);
  return hipGetLastError();
}

// ---------------------------------------------------------------- resolve
// SearchByProjection's first-come claims (src/ORBmatcher.cc:90-93,127) are
// resolved in map-point order by one of three exact schedules (DESIGN.md
// §4.2); the caller's schedule (orb_matcher_set_resolve) picks among them and
// ORB_RESOLVE_AUTO picks by shape:
//  * k_proj_resolve<NW> (prefix windows, NW waves per problem): batches of
//    small local maps.  >= 128 problems (the headline's 1024-frame launches,
//    run beside the next launch's extraction) take one wave per problem: the
//    longer per-problem chain is hidden and the extraction keeps the CU slots
//    (bench 306.5k vs 304.9k frames/s with four, profiles/r03_resolve_nw.txt);
//    9-127 problems four waves; maps of 20,000+ points whose fixed-point claim
//    buffers do not fit in LDS eight.
//  * k_proj_resolve_fp (1024-point windows iterated to their fixed point): maps
//    of 20,000+ points (C5: 33.9k -> 40.3k problems/s over 512-point prefix
//    windows), and calls of at most RESOLVE_FP_FEW problems at any map size
//    (the drop-in's one frame: one 5,000-point map in 5 windows instead of 20
//    prefix windows, SearchByProjection 0.239 -> 0.197 ms, profiles/r04_step10.txt).
//  * k_proj_jacobi rounds over the whole chip, then k_proj_resolve_fp for any
//    problem not settled (only on request: the rounds compete with a
//    concurrent extraction for every CU, profiles/r04_c5_stages.txt).
#ifndef RESOLVE_FP_T
#define RESOLVE_FP_T 1024  // threads of k_proj_resolve_fp (RESOLVE_FP_W / T points per thread)
#endif
#ifndef RESOLVE_FP_W
#define RESOLVE_FP_W 1024  // points per window of k_proj_resolve_fp (A/B knob)
#endif
#define RESOLVE_FP_MIN_MAP 20000
#define RESOLVE_FP_FEW 8
#ifndef RESOLVE_AUTO_FP
#define RESOLVE_AUTO_FP 0  // 1: every call takes the fixed-point kernel (A/B knob)
#endif
#ifndef RESOLVE_W1_MIN
#define RESOLVE_W1_MIN 128  // calls of at least this many problems take k_proj_resolve<1> (A/B knob)
#endif
#define RESOLVE_FP_LDS_MAX (160 * 1024 - 1024)

int orb_k_proj_resolve_kernel(int nproblems, int kpStride, int mpStride, int schedule) {
  const bool fpFits = (size_t)kpStride * 12 <= RESOLVE_FP_LDS_MAX;  // claims x 2 + kpMatch
  if (fpFits) {
    if (schedule == ORB_RESOLVE_JACOBI) return ORB_RESOLVE_KERNEL_JACOBI;
    if (schedule == ORB_RESOLVE_FIXED_POINT) return ORB_RESOLVE_KERNEL_FIXED_POINT;
    if (schedule == ORB_RESOLVE_AUTO && (mpStride >= RESOLVE_FP_MIN_MAP || nproblems <= RESOLVE_FP_FEW ||
                                         RESOLVE_AUTO_FP))
      return ORB_RESOLVE_KERNEL_FIXED_POINT;
  }
  if (mpStride >= RESOLVE_FP_MIN_MAP) return ORB_RESOLVE_KERNEL_PREFIX_W8;
  return nproblems >= RESOLVE_W1_MIN ? ORB_RESOLVE_KERNEL_PREFIX_W1 : ORB_RESOLVE_KERNEL_PREFIX_W4;
}

// bytes of Jacobi-resolve scratch for n problems (0 unless that schedule runs)
size_t orb_k_proj_jacobi_bytes(int kpStride, int mpStride, int nproblems, int schedule) {
  if (orb_k_proj_resolve_kernel(nproblems, kpStride, mpStride, schedule) != ORB_RESOLVE_KERNEL_JACOBI)
    return 0;
  return (size_t)jacobi_stride(kpStride, mpStride) * 4 * (size_t)nproblems;
}

hipError_t orb_k_proj_resolve(const orb_keypoint_t* keys, const uint8_t* desc,
                              const float* uright, const uint8_t* locked, const int32_t* nkeys,
                              int kpStride, const orb_mp_track_t* mps, const uint8_t* mpDesc,
                              const int32_t* nmps, int mpStride, const int32_t* cellStart,
                              const int32_t* cellIdx, const void* params, const uint32_t* topk,
                              const int32_t* ncand, int32_t* kpMatch, int32_t* nmatches,
                              int nproblems, int schedule, int jacobiRounds, int32_t* jacScratch,
                              hipStream_t s) {
  const ProjParams P = *(const ProjParams*)params;
  if (nproblems <= 0) return hipSuccess;
  const int kern = orb_k_proj_resolve_kernel(nproblems, kpStride, mpStride, schedule);
  if (kern == ORB_RESOLVE_KERNEL_FIXED_POINT || kern == ORB_RESOLVE_KERNEL_JACOBI) {
    const size_t ldsFp = (size_t)kpStride * 12;
    if (ldsFp > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute((const void*)k_proj_resolve_fp<RESOLVE_FP_T, RESOLVE_FP_W / RESOLVE_FP_T>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsFp);
      if (e != hipSuccess) return e;
    }
    const int32_t* done = nullptr;
    long long doneStride = 0;
    if (kern == ORB_RESOLVE_KERNEL_JACOBI) {
      if (!jacScratch) return hipErrorInvalidValue;
      const int R = std::max(1, std::min(48, jacobiRounds));
      const long long js = jacobi_stride(kpStride, mpStride);
      const int initN = std::max(3 * kpStride, R + 1);
      hipLaunchKernelGGL(k_proj_jacobi_init, dim3((initN + JAC_T - 1) / JAC_T, nproblems), dim3(JAC_T),
                         0, s, jacScratch, js, kpStride, R, nkeys, kpMatch, nmatches);
      // (an empty map stride still launches one workgroup per problem: a grid of x = 0 is invalid)
      const dim3 g((std::max(mpStride, 1) + JAC_T * JAC_PPT - 1) / (JAC_T * JAC_PPT), nproblems);
      for (int r = 0; r <= R; ++r)
        hipLaunchKernelGGL(k_proj_jacobi<JAC_PPT>, g, dim3(JAC_T), 0, s, keys, desc, uright, locked,
                           kpStride, mps, mpDesc, nmps, mpStride, cellStart, cellIdx, P, topk, ncand,
                           kpMatch, nmatches, jacScratch, js, r, R);
      done = jacScratch + R;
      doneStride = js;
    }
    hipLaunchKernelGGL((k_proj_resolve_fp<RESOLVE_FP_T, RESOLVE_FP_W / RESOLVE_FP_T>), dim3(nproblems), dim3(RESOLVE_FP_T),
                       ldsFp, s, keys, desc,
                       uright, locked, nkeys, kpStride, mps, mpDesc, nmps, mpStride, cellStart,
                       cellIdx, P, topk, ncand, kpMatch, nmatches, done, doneStride);
    return hipGetLastError();
  }
  const size_t words = (size_t)((kpStride + 31) / 32);
  const size_t lds = ((words + 3) & ~(size_t)3) * 4 + (size_t)kpStride * 4;
  if (kern == ORB_RESOLVE_KERNEL_PREFIX_W8)
    hipLaunchKernelGGL(k_proj_resolve<8>, dim3(nproblems), dim3(512), lds, s, keys, desc, uright,
                       locked, nkeys, kpStride, mps, mpDesc, nmps, mpStride, cellStart, cellIdx,
                       P, topk, ncand, kpMatch, nmatches);
  else if (kern == ORB_RESOLVE_KERNEL_PREFIX_W1)
    hipLaunchKernelGGL(k_proj_resolve<1>, dim3(nproblems), dim3(64), lds, s, keys, desc, uright,
                       locked, nkeys, kpStride, mps, mpDesc, nmps, mpStride, cellStart, cellIdx,
                       P, topk, ncand, kpMatch, nmatches);
  else
    hipLaunchKernelGGL(k_proj_resolve<4>, dim3(nproblems), dim3(256), lds, s, keys, desc, uright,
                       locked, nkeys, kpStride, mps, mpDesc, nmps, mpStride, cellStart, cellIdx,
                       P, topk, ncand, kpMatch, nmatches);
  return hipGetLastError();
}

size_t orb_k_proj_params_size(void) { return sizeof(ProjParams); }

// bytes of the candidate-list pool (ProjParams.ovf) of n problems
size_t orb_k_proj_ovf_bytes(int nproblems) {
  return (size_t)std::max(nproblems, 1) * OVF_SLOTS * OVF_CAP * 4;
}


}  // extern "C"

// ==================================================== Frame::ComputeStereoMatches
// src/Frame.cc:516-704.  One wave per left keypoint:
//  1. candidates = right keypoints whose row band [floor(y-2s), ceil(y+2s)]
//     contains int(vL), octave within +-1, uR in [uL - maxD, uL]; the lanes
//     scan the right keypoints strided and reduce (dist, iR) -> first minimum
//     (the reference scans vRowIndices[vL] in ascending iR, strict <).
//  2. 11x11 SAD (patch minus its centre) at the left octave for the 11 shifts,
//     parabola sub-pixel, disparity window, depth = bf / disparity.
// k_stereo_prune then drops matches whose SAD >= 1.5*1.4*median (:690-703).
struct StereoParams {
  int nLevels;
  float bf, fx;
  int w[ORB_MAX_LEVELS], h[ORB_MAX_LEVELS];
  int strideL[ORB_MAX_LEVELS], strideR[ORB_MAX_LEVELS];
  float scale[ORB_MAX_LEVELS], invScale[ORB_MAX_LEVELS];
};

struct StereoPairLevels {
  const uint8_t* L[ORB_MAX_LEVELS];
  const uint8_t* R[ORB_MAX_LEVELS];
};

// vRowIndices (src/Frame.cc:531-550) as CSR per pair: row yi lists every right
// keypoint whose band [floor(y - 2 s), ceil(y + 2 s)] contains it (s = the
// keypoint's scale factor).  One workgroup per pair, LDS row counters.  The
// order inside a row is free: the match is the lexicographic (distance, iR)
// minimum, which is the reference's first minimum in ascending iR.
__global__ __launch_bounds__(1024) void k_stereo_rows(const orb_keypoint_t* __restrict__ rkeys,
                                                      const int32_t* __restrict__ nright,
                                                      int kpStride, StereoParams P,
                                                      int32_t* __restrict__ rowStart,
                                                      int32_t* __restrict__ rowIdx, int rowCap) {
  extern __shared__ int cnt[];  // rows + 1
  __shared__ int tmp[17];
  const int pair = blockIdx.x, t = threadIdx.x, T = blockDim.x;
  const int H = P.h[0], NR = nright[pair];
  const orb_keypoint_t* K = rkeys + (size_t)pair * kpStride;
  for (int i = t; i <= H; i += T) cnt[i] = 0;
  __syncthreads();
  auto band = [&](const orb_keypoint_t& kp, int* lo, int* hi) {
    const float r = 2.0f * P.scale[kp.octave];
    *lo = max((int)floorf(kp.y - r), 0);
    *hi = min((int)ceilf(kp.y + r), H - 1);
  };
  for (int iR = t; iR < NR; iR += T) {
    int lo, hi;
    band(K[iR], &lo, &hi);
    for (int yi = lo; yi <= hi; ++yi) atomicAdd(&cnt[yi], 1);
  }
  __syncthreads();
  {  // exclusive scan of the H + 1 counters, a chunk per thread
    const int n = H + 1, per = (n + T - 1) / T, b = min(t * per, n), e = min(b + per, n);
    int sum = 0;
    for (int i = b; i < e; ++i) sum += cnt[i];
    int total;
    int ex = block_excl_scan(sum, tmp, &total);
    for (int i = b; i < e; ++i) {
      const int v = cnt[i];
      cnt[i] = ex;
      ex += v;
    }
    __syncthreads();
  }
  int32_t* rs = rowStart + (size_t)pair * (H + 1);
  for (int i = t; i <= H; i += T) rs[i] = cnt[i];
  __syncthreads();
  // entry j of the pair's row lists: iR | octave << 24, and the keypoint's x
  // in the parallel float array rx (the match's candidate filter then needs
  // no load of the keypoint record)
  int32_t* ri = rowIdx + (size_t)pair * 2 * rowCap;
  float* rx = reinterpret_cast<float*>(ri + rowCap);
  for (int iR = t; iR < NR; iR += T) {
    const orb_keypoint_t kp = K[iR];
    int lo, hi;
    band(kp, &lo, &hi);
    const int e = iR | (kp.octave << 24);
    for (int yi = lo; yi <= hi; ++yi) {
      const int pos = atomicAdd(&cnt[yi], 1);
      if (pos < rowCap) {
        ri[pos] = e;
        rx[pos] = kp.x;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_stereo_match(
    const orb_keypoint_t* __restrict__ lkeys, const uint8_t* __restrict__ ldesc,
    const int32_t* __restrict__ nleft, const orb_keypoint_t* __restrict__ rkeys,
    const uint8_t* __restrict__ rdesc, const int32_t* __restrict__ nright, int kpStride,
    const StereoPairLevels* __restrict__ pyr, StereoParams P, float* __restrict__ uRight,
    float* __restrict__ depth, int32_t* __restrict__ sad, const int32_t* __restrict__ rowStart,
    const int32_t* __restrict__ rowIdx, int rowCap) {
  const int pair = blockIdx.y, lane = threadIdx.x & 63;
  const int iL = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int NL = nleft[pair], NR = nright[pair];
  if (iL >= NL) return;
  const size_t base = (size_t)pair * kpStride;
  const orb_keypoint_t kpL = lkeys[base + iL];
  float ur = -1.0f, dp = -1.0f;
  int sadOut = -1;
  const float mb = P.bf / P.fx;
  const float minZ = mb, minD = 0.f, maxD = P.bf / minZ;
  const int levelL = kpL.octave;
  const float vL = kpL.y, uL = kpL.x;
  const int row = (int)vL;  // vRowIndices[vL]: float -> size_t truncation
  const float minU = uL - maxD, maxU = uL - minD;
  int bestDist = 1 << 30, bestIdx = 1 << 30;
  float bestX = 0.f;
  (void)NR;
  if (maxU >= 0 && row >= 0 && row < P.h[0]) {
    const ulonglong4 dL = load_desc(ldesc + (base + iL) * 32);
    // vCandidates = vRowIndices[vL]: the right keypoints whose band holds the row
    const int32_t* rs = rowStart + (size_t)pair * (P.h[0] + 1);
    const int32_t* ri = rowIdx + (size_t)pair * 2 * rowCap;
    const float* rx = reinterpret_cast<const float*>(ri + rowCap);
    const int jEnd = min(rs[row + 1], rowCap);
    for (int j = rs[row] + lane; j < jEnd; j += 64) {
      const int e = ri[j];
      const float uR = rx[j];
      const int iR = e & 0xFFFFFF, octR = e >> 24;
      if (octR < levelL - 1 || octR > levelL + 1) continue;
      if (!(uR >= minU && uR <= maxU)) continue;
      const int dist = hamming256(dL, load_desc(rdesc + (base + iR) * 32));
      // (distance, iR) order: a row list holds its entries in no particular order
      if (dist < bestDist || (dist == bestDist && iR < bestIdx)) { bestDist = dist; bestIdx = iR; bestX = uR; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int od = __shfl_xor(bestDist, o, 64), oi = __shfl_xor(bestIdx, o, 64);
    const float ox = __shfl_xor(bestX, o, 64);
    if (od < bestDist || (od == bestDist && oi < bestIdx)) { bestDist = od; bestIdx = oi; bestX = ox; }
  }
  // bestDist starts at TH_HIGH=100 in the reference; accept below (100+50)/2
  if (maxU >= 0 && bestDist < 75) {
    const float uR0 = bestX;
    const float sf = P.invScale[levelL];
    const float scaleduL = round_half_away(kpL.x * sf);
    const float scaledvL = round_half_away(kpL.y * sf);
    const float scaleduR0 = round_half_away(uR0 * sf);
    const int w = 5, L = 5;
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    if (!(iniu < 0 || endu >= P.w[levelL])) {
      const uint8_t* IL = pyr[pair].L[levelL];
      const uint8_t* IR = pyr[pair].R[levelL];
      const int sL = P.strideL[levelL], sR = P.strideR[levelL];
      const int y0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
      const int cL = IL[(long long)(y0 + w) * sL + xl0 + w];
      // lane p < 121 (two rounds) owns patch pixel (yy, xx): its left value
      // once, and the 11 right values it meets over the 11 shifts, which are
      // consecutive bytes of one right row (four dword loads, realigned); the
      // shifts' right centres come from lanes 0..10.  Per-shift SADs are
      // < 121 * 255 < 2^16, so two share a word through the wave reduction.
      const int xrb = (int)scaleduR0 - L - w;  // right patch column of shift -L
      const int cRv = lane < 2 * L + 1 ? (int)IR[(long long)(y0 + w) * sR + xrb + w + lane] : 0;
      uint32_t acc[11];
      // |(l - cL) - (r - cR_k)| as one v_sad_u16 on values biased by 256
      // (both in [1, 511]); the right byte and its shift's bias in one add
      uint32_t rbias[11];
#pragma unroll
      for (int k = 0; k < 11; ++k) {
        acc[k] = 0u;
        rbias[k] = (uint32_t)(256 - __builtin_amdgcn_readlane(cRv, k));
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int p = lane + 64 * q;
        if (p < 121) {
          const int yy = p / 11, xx = p - yy * 11;
          const uint32_t ab = (uint32_t)((int)IL[(long long)(y0 + yy) * sL + xl0 + xx] - cL + 256);
          const uint8_t* rrow = IR + (long long)(y0 + yy) * sR + xrb + xx;
          const uintptr_t ra = (uintptr_t)rrow;
          const uint32_t* rw = reinterpret_cast<const uint32_t*>(ra & ~(uintptr_t)3);
          const uint32_t shb = (uint32_t)(ra & 3);
          uint32_t wv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) wv[k] = rw[k];
          uint32_t bw[3];
#pragma unroll
          for (int k = 0; k < 3; ++k) bw[k] = __builtin_amdgcn_alignbyte(wv[k + 1], wv[k], shb);
#pragma unroll
          for (int k = 0; k < 11; ++k) {
            const uint32_t bb = ((bw[k >> 2] >> (8 * (k & 3))) & 0xFFu) + rbias[k];
            acc[k] = __builtin_amdgcn_sad_u16(ab, bb, acc[k]);
          }
        }
      }
      int dists[11];
#pragma unroll
      for (int k = 0; k < 11; k += 2) {
        const int packed = (int)(acc[k] | (k + 1 < 11 ? acc[k + 1] << 16 : 0u));
        const int sum = wave_sum(packed);
        dists[k] = sum & 0xFFFF;
        if (k + 1 < 11) dists[k + 1] = (int)((uint32_t)sum >> 16);
      }
      int bestSad = 2147483647, bestinc = 0;
#pragma unroll
      for (int inc = -L; inc <= L; ++inc)
        if ((float)dists[inc + L] < (float)bestSad) { bestSad = dists[inc + L]; bestinc = inc; }
      if (bestinc != -L && bestinc != L) {
        const float dist1 = (float)dists[L + bestinc - 1], dist2 = (float)dists[L + bestinc],
                    dist3 = (float)dists[L + bestinc + 1];
        const float deltaR = __fdiv_rn(dist1 - dist3, 2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (!(deltaR < -1 || deltaR > 1)) {
          float bestuR = P.scale[levelL] * ((float)scaleduR0 + (float)bestinc + deltaR);
          float disparity = uL - bestuR;
          if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
              disparity = 0.01f;
              bestuR = (float)((double)uL - 0.01);
            }
            dp = __fdiv_rn(P.bf, disparity);
            ur = bestuR;
            sadOut = bestSad;
          }
        }
      }
    }
  }
  if (lane == 0) {
    uRight[base + iL] = ur;
    depth[base + iL] = dp;
    sad[base + iL] = sadOut;
  }
}

// 64 / G left keypoints per wave (lane group h = lanes G h .. G h + G - 1
// takes keypoint (64 / G) w + h): the same steps as k_stereo_match, with the
// candidate reduction, the right centres and the SAD sums kept inside each
// group.  The kernel is a chain of dependent loads per keypoint (row band,
// candidates, descriptors, then the patches), so its cost beside the
// extraction is the wave slots it holds: C3's stereo match 0.535 ms per 256
// pairs with one keypoint per wave, 0.445 with two, 0.412 with four
// (profiles/r05_stereo.txt); G = 16 is the smallest group that holds the 11
// shifts' right centres.
// sum over the G-lane group (G = 32 or 16) a lane belongs to
template <int G>
__device__ __forceinline__ int stereo_group_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);  // row_mirror
  if (G == 32) v += __builtin_amdgcn_ds_swizzle(v, 0x401F);        // lane ^ 16
  return v;
}
template <int G>
__global__ __launch_bounds__(256) void k_stereo_match2(
    const orb_keypoint_t* __restrict__ lkeys, const uint8_t* __restrict__ ldesc,
    const int32_t* __restrict__ nleft, const orb_keypoint_t* __restrict__ rkeys,
    const uint8_t* __restrict__ rdesc, const int32_t* __restrict__ nright, int kpStride,
    const StereoPairLevels* __restrict__ pyr, StereoParams P, float* __restrict__ uRight,
    float* __restrict__ depth, int32_t* __restrict__ sad, const int32_t* __restrict__ rowStart,
    const int32_t* __restrict__ rowIdx, int rowCap) {
  constexpr int KPW = 64 / G;  // keypoints per wave
  const int pair = blockIdx.y, lane = threadIdx.x & 63, half = lane / G, hl = lane & (G - 1);
  const int iL = (blockIdx.x * 4 + (threadIdx.x >> 6)) * KPW + half;
  const int NL = nleft[pair];
  const bool live = iL < NL;
  if (__ballot(live) == 0ull) return;  // (wave-uniform)
  const size_t base = (size_t)pair * kpStride;
  const orb_keypoint_t kpL = lkeys[base + (live ? iL : 0)];
  float ur = -1.0f, dp = -1.0f;
  int sadOut = -1;
  const float mb = P.bf / P.fx;
  const float minZ = mb, minD = 0.f, maxD = P.bf / minZ;
  const int levelL = kpL.octave;
  const float vL = kpL.y, uL = kpL.x;
  const int row = (int)vL;  // vRowIndices[vL]: float -> size_t truncation
  const float minU = uL - maxD, maxU = uL - minD;
  int bestDist = 1 << 30, bestIdx = 1 << 30;
  float bestX = 0.f;  // the best candidate's x (from the row list)
  const bool scan = live && maxU >= 0 && row >= 0 && row < P.h[0];
  if (scan) {
    const ulonglong4 dL = load_desc(ldesc + (base + iL) * 32);
    const int32_t* rs = rowStart + (size_t)pair * (P.h[0] + 1);
    const int32_t* ri = rowIdx + (size_t)pair * 2 * rowCap;
    const float* rx = reinterpret_cast<const float*>(ri + rowCap);
    const int jEnd = min(rs[row + 1], rowCap);
    for (int j = rs[row] + hl; j < jEnd; j += G) {
      const int e = ri[j];
      const float uR = rx[j];
      const int iR = e & 0xFFFFFF, octR = e >> 24;
      if (octR < levelL - 1 || octR > levelL + 1) continue;
      if (!(uR >= minU && uR <= maxU)) continue;
      const int dist = hamming256(dL, load_desc(rdesc + (base + iR) * 32));
      // (distance, iR) order: a row list holds its entries in no particular order
      if (dist < bestDist || (dist == bestDist && iR < bestIdx)) { bestDist = dist; bestIdx = iR; bestX = uR; }
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) {  // inside the group
    const int od = __shfl_xor(bestDist, o, 64), oi = __shfl_xor(bestIdx, o, 64);
    const float ox = __shfl_xor(bestX, o, 64);
    if (od < bestDist || (od == bestDist && oi < bestIdx)) { bestDist = od; bestIdx = oi; bestX = ox; }
  }
  const bool matched = scan && bestDist < 75;  // uniform within the half
  float scaleduR0 = 0.f;
  bool patch = false;
  const int w = 5, L = 5;
  const uint8_t* IL = nullptr;
  const uint8_t* IR = nullptr;
  int sL = 0, sR = 0, y0 = 0, xl0 = 0, xrb = 0;
  if (matched) {
    const float uR0 = bestX;
    const float sf = P.invScale[levelL];
    scaleduR0 = round_half_away(uR0 * sf);
    const float scaleduL = round_half_away(kpL.x * sf);
    const float scaledvL = round_half_away(kpL.y * sf);
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    patch = !(iniu < 0 || endu >= P.w[levelL]);
    IL = pyr[pair].L[levelL];
    IR = pyr[pair].R[levelL];
    sL = P.strideL[levelL];
    sR = P.strideR[levelL];
    y0 = (int)scaledvL - w;
    xl0 = (int)scaleduL - w;
    xrb = (int)scaleduR0 - L - w;  // right patch column of shift -L
  }
  if (__ballot(patch) != 0ull) {  // (wave-uniform: the cross-lane steps below need both halves)
    const int cL = patch ? (int)IL[(long long)(y0 + w) * sL + xl0 + w] : 0;
    // the half's lanes 0..10 load its shifts' right centres; every lane of
    // the half takes them by a lane shuffle inside the half
    const int cRv = (patch && hl < 2 * L + 1) ? (int)IR[(long long)(y0 + w) * sR + xrb + w + hl] : 0;
    uint32_t acc[11], rbias[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) {
      acc[k] = 0u;
      rbias[k] = (uint32_t)(256 - __shfl(cRv, (lane & ~(G - 1)) + k, 64));
    }
    if (patch) {
#pragma unroll
      for (int q = 0; q < (121 + G - 1) / G; ++q) {
        const int p = hl + G * q;
        if (p < 121) {
          const int yy = p / 11, xx = p - yy * 11;
          const uint32_t ab = (uint32_t)((int)IL[(long long)(y0 + yy) * sL + xl0 + xx] - cL + 256);
          const uint8_t* rrow = IR + (long long)(y0 + yy) * sR + xrb + xx;
          const uintptr_t ra = (uintptr_t)rrow;
          const uint32_t* rw = reinterpret_cast<const uint32_t*>(ra & ~(uintptr_t)3);
          const uint32_t shb = (uint32_t)(ra & 3);
          uint32_t wv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) wv[k] = rw[k];
          uint32_t bw[3];
#pragma unroll
          for (int k = 0; k < 3; ++k) bw[k] = __builtin_amdgcn_alignbyte(wv[k + 1], wv[k], shb);
#pragma unroll
          for (int k = 0; k < 11; ++k) {
            const uint32_t bb = ((bw[k >> 2] >> (8 * (k & 3))) & 0xFFu) + rbias[k];
            acc[k] = __builtin_amdgcn_sad_u16(ab, bb, acc[k]);
          }
        }
      }
    }
    int dists[11];
#pragma unroll
    for (int k = 0; k < 11; k += 2) {
      const int packed = (int)(acc[k] | (k + 1 < 11 ? acc[k + 1] << 16 : 0u));
      const int sum = stereo_group_sum<G>(packed);
      dists[k] = sum & 0xFFFF;
      if (k + 1 < 11) dists[k + 1] = (int)((uint32_t)sum >> 16);
    }
    if (patch) {
      int bestSad = 2147483647, bestinc = 0;
#pragma unroll
      for (int inc = -L; inc <= L; ++inc)
        if ((float)dists[inc + L] < (float)bestSad) { bestSad = dists[inc + L]; bestinc = inc; }
      if (bestinc != -L && bestinc != L) {
        const float dist1 = (float)dists[L + bestinc - 1], dist2 = (float)dists[L + bestinc],
                    dist3 = (float)dists[L + bestinc + 1];
        const float deltaR = __fdiv_rn(dist1 - dist3, 2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (!(deltaR < -1 || deltaR > 1)) {
          float bestuR = P.scale[levelL] * ((float)scaleduR0 + (float)bestinc + deltaR);
          float disparity = uL - bestuR;
          if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
              disparity = 0.01f;
              bestuR = (float)((double)uL - 0.01);
            }
            dp = __fdiv_rn(P.bf, disparity);
            ur = bestuR;
            sadOut = bestSad;
          }
        }
      }
    }
  }
  if (live && hl == 0) {
    uRight[base + iL] = ur;
    depth[base + iL] = dp;
    sad[base + iL] = sadOut;
  }
}

#ifndef STEREO_KPW
#define STEREO_KPW 4  // left keypoints per wave of the stereo match: 4 (16-lane groups), 2, or 1 (k_stereo_match)
#endif

// Median-based outlier rejection: k-th smallest SAD by bisection on the value
// (k = V/2 of the V valid matches, == vDistIdx[size/2] after the sort), then
// every match with SAD >= 1.5*1.4*median is reset to -1.  One block per pair.
__global__ __launch_bounds__(256) void k_stereo_prune(const int32_t* __restrict__ nleft,
                                                      int kpStride, float* __restrict__ uRight,
                                                      float* __restrict__ depth,
                                                      const int32_t* __restrict__ sad) {
  __shared__ int tmp[17];
  const int pair = blockIdx.x, t = threadIdx.x;
  const int NL = nleft[pair];
  const size_t base = (size_t)pair * kpStride;
  int c = 0;
  for (int i = t; i < NL; i += 256) c += sad[base + i] >= 0;
  int V;
  block_excl_scan(c, tmp, &V);
  if (V == 0) return;  // the reference indexes an empty vector here (undefined)
  const int k = V / 2;
  int lo = 0, hi = 1 << 20;  // smallest v with count(sad <= v) > k
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    int cnt = 0;
    for (int i = t; i < NL; i += 256) {
      const int s = sad[base + i];
      cnt += (s >= 0 && s <= mid);
    }
    int tot;
    block_excl_scan(cnt, tmp, &tot);
    if (tot > k) hi = mid; else lo = mid + 1;
  }
  const float median = (float)lo;
  const float thDist = 1.5f * 1.4f * median;
  for (int i = t; i < NL; i += 256) {
    const int s = sad[base + i];
    if (s >= 0 && !((float)s < thDist)) {
      uRight[base + i] = -1.0f;
      depth[base + i] = -1.0f;
    }
  }
}

extern "C" size_t orb_k_stereo_params_size(void) { return sizeof(StereoParams); }

// Row-index scratch of orb_k_stereo: ints per pair for the row starts and for
// the row lists (every right keypoint listed in each row of its band).
extern "C" void orb_k_stereo_scratch(const void* params, int kpStride, size_t* startInts,
                                     size_t* idxInts) {
  const StereoParams& P = *(const StereoParams*)params;
  float smax = 1.f;
  for (int l = 0; l < P.nLevels; ++l) smax = std::max(smax, P.scale[l]);
  *startInts = (size_t)P.h[0] + 1;
  // entries (iR | octave << 24) and their keypoints' x, two arrays
  *idxInts = 2 * (size_t)kpStride * (size_t)(std::ceil(4.0 * smax) + 3.0);
}

extern "C" hipError_t orb_k_stereo(const orb_keypoint_t* lkeys, const uint8_t* ldesc,
                                   const int32_t* nleft, const orb_keypoint_t* rkeys,
                                   const uint8_t* rdesc, const int32_t* nright, int kpStride,
                                   int maxLeft, const void* pyr, const void* params,
                                   float* uRight, float* depth, int32_t* sad, int npairs,
                                   int32_t* rowStart, int32_t* rowIdx, hipStream_t s) {
  if (npairs <= 0 || maxLeft <= 0) return hipSuccess;
  const StereoParams P = *(const StereoParams*)params;
  size_t startInts, idxInts;
  orb_k_stereo_scratch(params, kpStride, &startInts, &idxInts);
  const size_t rowsLds = ((size_t)P.h[0] + 1) * sizeof(int);
  if (rowsLds > 64 * 1024) return hipErrorInvalidValue;  // images up to 16k rows
  hipLaunchKernelGGL(k_stereo_rows, dim3(npairs), dim3(1024), rowsLds, s, rkeys, nright,
                     kpStride, P, rowStart, rowIdx, (int)(idxInts / 2));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (STEREO_KPW == 4)
    hipLaunchKernelGGL(k_stereo_match2<16>, dim3((maxLeft + 15) / 16, npairs), dim3(256), 0, s, lkeys,
                       ldesc, nleft, rkeys, rdesc, nright, kpStride,
                       (const StereoPairLevels*)pyr, P, uRight, depth, sad, rowStart, rowIdx,
                       (int)(idxInts / 2));
  else if (STEREO_KPW == 2)
    hipLaunchKernelGGL(k_stereo_match2<32>, dim3((maxLeft + 7) / 8, npairs), dim3(256), 0, s, lkeys,
                       ldesc, nleft, rkeys, rdesc, nright, kpStride,
                       (const StereoPairLevels*)pyr, P, uRight, depth, sad, rowStart, rowIdx,
                       (int)(idxInts / 2));
  else
    hipLaunchKernelGGL(k_stereo_match, dim3((maxLeft + 3) / 4, npairs), dim3(256), 0, s, lkeys,
                       ldesc, nleft, rkeys, rdesc, nright, kpStride,
                       (const StereoPairLevels*)pyr, P, uRight, depth, sad, rowStart, rowIdx,
                       (int)(idxInts / 2));
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_stereo_prune, dim3(npairs), dim3(256), 0, s, nleft, kpStride, uRight,
                     depth, sad);
  return hipGetLastError();
}


// ============================== SearchByProjection(CurrentFrame, LastFrame)
// src/ORBmatcher.cc:1460-1619.  k_frame_candidates: per last-frame point, the
// first K candidates in (distance, scan order).  k_frame_resolve: one wave per
// problem replays the sequential loop (first-come locks by points with
// observations), then the rotation histogram filter.
struct FrameProjParams {
  float minX, maxX, minY, maxY, invW, invH;
  float fx, fy, cx, cy, bf;
  float th;
  int fwd, bwd, checkOri;
  float scale[ORB_MAX_LEVELS];
};

__global__ __launch_bounds__(256) void k_frame_candidates(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked,
    const orb_last_mp_t* __restrict__ last, const uint8_t* __restrict__ lastDesc, int nlast,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, FrameProjParams F,
    uint32_t* __restrict__ topk, int32_t* __restrict__ ncand) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nlast) return;
  const orb_last_mp_t L = last[i];
  ncand[i] = -1;
  if (!L.valid) return;
  const float invzc = L.invzc;
  if (invzc < 0) return;
  const float u = F.fx * L.xc * invzc + F.cx;
  const float v = F.fy * L.yc * invzc + F.cy;
  if (u < F.minX || u > F.maxX) return;
  if (v < F.minY || v > F.maxY) return;
  const int o = L.last_octave;
  const float radius = F.th * F.scale[o];
  ProjParams P;
  P.minX = F.minX; P.minY = F.minY; P.invW = F.invW; P.invH = F.invH;
  int minL, maxL;
  if (F.fwd) { minL = o; maxL = -1; }
  else if (F.bwd) { minL = 0; maxL = o; }
  else { minL = o - 1; maxL = o + 1; }
  const ulonglong4 q = load_desc(lastDesc + (size_t)i * 32);
  Top4 top;
  int count = 0;
  for_features_in_area(keys, cellStart, cellIdx, P, u, v, radius, minL, maxL,
                       [&](int idx, const orb_keypoint_t& kp) {
                         if (locked && locked[idx]) return;
                         if (uright && uright[idx] > 0) {
                           const float ur = u - F.bf * invzc;
                           const float er = fabsf(ur - uright[idx]);
                           if (er > radius) return;
                         }
                         const int dist = hamming256(q, load_desc(desc + (size_t)idx * 32));
                         if (dist >= 256) return;
                         ++count;
                         top.insert(pack_cand(idx, dist, kp.octave), dist);
                       });
  top.store(topk + (size_t)i * TOPK);
  ncand[i] = count;
}

__global__ __launch_bounds__(64) void k_frame_resolve(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked, int nkeys,
    const orb_last_mp_t* __restrict__ last, const uint8_t* __restrict__ lastDesc, int nlast,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, FrameProjParams F,
    const uint32_t* __restrict__ topk, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ kpMatch, int32_t* __restrict__ nmatches) {
  // LDS: in-call lock bits, earliest claiming lane of the window, the last
  // point assigned to each keypoint, the accepted keypoint of each point
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ int hist[32];
  const int lane = threadIdx.x;
  const int words = (nkeys + 31) >> 5;
  const int wpad = (words + 3) & ~3, npad = (nkeys + 3) & ~3;
  uint32_t* bm = dyn;
  int* claimBy = (int*)(dyn + wpad);
  int* lastWriter = claimBy + npad;
  int* accIdx = lastWriter + npad;
  for (int i = lane; i < words; i += 64) bm[i] = 0u;
  for (int i = lane; i < nkeys; i += 64) { claimBy[i] = 64; lastWriter[i] = -1; }
  if (lane < 32) hist[lane] = 0;
  __syncthreads();
  int start = 0;
  while (start < nlast) {
    const int m = start + lane;
    const bool active = m < nlast;
    int nc = -1;
    uint32_t e[TOPK];
    bool hasObs = false;
    if (active) {
      nc = ncand[m];
      for (int j = 0; j < TOPK; ++j) e[j] = topk[(size_t)m * TOPK + j];
      hasObs = last[m].has_obs != 0;
    }
    int best = -1, bestDist = 256, consumed = 0;
    if (nc > 0) {
      const int avail = nc < TOPK ? nc : TOPK;
      for (int j = 0; j < avail; ++j) {
        ++consumed;
        if (lock_test(bm, cand_idx(e[j]))) continue;
        best = cand_idx(e[j]);
        bestDist = cand_dist(e[j]);
        break;
      }
    }
    const bool slow = nc > TOPK && best < 0;
    const bool accept = !slow && best >= 0 && bestDist <= 100;
    const bool locks = accept && hasObs;
    if (locks) atomicMin(&claimBy[best], lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bool conflict = false;
    for (int q = 0; q < consumed; ++q) conflict |= claimBy[cand_idx(e[q])] < lane;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (locks) claimBy[best] = 64;
    const unsigned long long bad = __ballot(active && (conflict || (slow && lane > 0)));
    const unsigned long long slowFirst = __ballot(lane == 0 && active && slow);
    int commit = bad ? (int)__builtin_ctzll(bad) : 64;
    if (slowFirst) {
      if (lane == 0) {  // exact re-scan against the current locks
        const orb_last_mp_t L = last[m];
        const float invzc = L.invzc;
        const float u = F.fx * L.xc * invzc + F.cx;
        const float v = F.fy * L.yc * invzc + F.cy;
        const int o = L.last_octave;
        const float radius = F.th * F.scale[o];
        ProjParams P;
        P.minX = F.minX; P.minY = F.minY; P.invW = F.invW; P.invH = F.invH;
        int minL, maxL;
        if (F.fwd) { minL = o; maxL = -1; }
        else if (F.bwd) { minL = 0; maxL = o; }
        else { minL = o - 1; maxL = o + 1; }
        const ulonglong4 q = load_desc(lastDesc + (size_t)m * 32);
        int bd = 256, bi = -1;
        for_features_in_area(keys, cellStart, cellIdx, P, u, v, radius, minL, maxL,
                             [&](int idx, const orb_keypoint_t& kp) {
                               if ((locked && locked[idx]) || lock_test(bm, idx)) return;
                               if (uright && uright[idx] > 0) {
                                 const float ur = u - F.bf * invzc;
                                 if (fabsf(ur - uright[idx]) > radius) return;
                               }
                               const int dist = hamming256(q, load_desc(desc + (size_t)idx * 32));
                               if (dist < bd) { bd = dist; bi = idx; }
                             });
        accIdx[m] = -1;
        if (bd <= 100) {
          accIdx[m] = bi;
          atomicMax(&lastWriter[bi], m);
          if (hasObs) bm[bi >> 5] |= 1u << (bi & 31);
          if (F.checkOri) atomicAdd(&hist[rot_bin(L.last_angle - keys[bi].angle)], 1);
        }
      }
      commit = 1;
    } else {
      if (active && lane < commit) {
        accIdx[m] = accept ? best : -1;
        if (accept) {
          atomicMax(&lastWriter[best], m);
          if (locks) atomicOr(&bm[best >> 5], 1u << (best & 31));
          if (F.checkOri) atomicAdd(&hist[rot_bin(last[m].last_angle - keys[best].angle)], 1);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    start += commit;
  }
  // rotation filter: records of the bins outside the top 3 are undone
  int ind1 = -1, ind2 = -1, ind3 = -1;
  if (F.checkOri) three_maxima(hist, ind1, ind2, ind3);
  uint32_t* cleared = bm;  // reuse: bit set = keypoint reset to NULL by the filter
  for (int i = lane; i < words; i += 64) cleared[i] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int removed = 0, accepted = 0;
  for (int m = lane; m < nlast; m += 64) {
    const int bi = accIdx[m];
    if (bi < 0) continue;
    ++accepted;
    if (!F.checkOri) continue;
    const int b = rot_bin(last[m].last_angle - keys[bi].angle);
    if (b != ind1 && b != ind2 && b != ind3) {
      ++removed;
      atomicOr(&cleared[bi >> 5], 1u << (bi & 31));
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // kpMatch: MapPoint id assigned by this call, -1 untouched, -2 reset to NULL
  for (int i = lane; i < nkeys; i += 64) {
    const int wr = lastWriter[i];
    if ((cleared[i >> 5] >> (i & 31)) & 1u) kpMatch[i] = -2;
    else kpMatch[i] = wr >= 0 ? last[wr].mp_id : -1;
  }
  const int acc = wave_sum(accepted), rem = wave_sum(removed);
  if (lane == 0) *nmatches = acc - rem;
}

extern "C" size_t orb_k_frame_params_size(void) { return sizeof(FrameProjParams); }

extern "C" hipError_t orb_k_frame_proj(const orb_keypoint_t* keys, const uint8_t* desc,
                                       const float* uright, const uint8_t* locked, int nkeys,
                                       const orb_last_mp_t* last, const uint8_t* lastDesc,
                                       int nlast, const int32_t* cellStart,
                                       const int32_t* cellIdx, const void* params,
                                       uint32_t* topk, int32_t* ncand, int32_t* kpMatch,
                                       int32_t* nmatches, hipStream_t s) {
  const FrameProjParams F = *(const FrameProjParams*)params;
  if (nlast > 0) {
    hipLaunchKernelGGL(k_frame_candidates, dim3((nlast + 255) / 256), dim3(256), 0, s, keys,
                       desc, uright, locked, last, lastDesc, nlast, cellStart, cellIdx, F, topk,
                       ncand);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const size_t words = (size_t)((nkeys + 31) / 32);
  const size_t lds = (((words + 3) & ~(size_t)3) + 2 * (((size_t)nkeys + 3) & ~(size_t)3) +
                      (size_t)std::max(nlast, 1)) * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_frame_resolve,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_frame_resolve, dim3(1), dim3(64), lds, s, keys, desc, uright, locked,
                     nkeys, last, lastDesc, nlast, cellStart, cellIdx, F, topk, ncand, kpMatch,
                     nmatches);
  return hipGetLastError();
}

// ====================================== SearchByBoW(KeyFrame*, Frame&, ...)
// src/ORBmatcher.cc:164-306.  A frame feature belongs to exactly one vocabulary
// node, and claims (vpMapPointMatches[realIdxF]) only ever involve features of
// the node being matched, so nodes are independent: one wave per KeyFrame
// node finds its Frame node by binary search and replays the node's loop
// sequentially, lanes sharing the brute-force distance scan.  k_bow_finish
// applies the rotation histogram filter.
__global__ __launch_bounds__(256) void k_bow_match(
    const uint8_t* __restrict__ kfDesc, const float* __restrict__ kfAngle,
    const int32_t* __restrict__ kfMp, const uint8_t* __restrict__ kfBad, int kfNodes,
    const uint32_t* __restrict__ kfNodeIds, const int32_t* __restrict__ kfOffs,
    const uint32_t* __restrict__ kfFeats, const uint8_t* __restrict__ fDesc,
    const float* __restrict__ fAngle, int fNodes, const uint32_t* __restrict__ fNodeIds,
    const int32_t* __restrict__ fOffs, const uint32_t* __restrict__ fFeats, float nnratio,
    int nF, const int32_t* __restrict__ fMp, const uint8_t* __restrict__ fBad, int thLow,
    int32_t* __restrict__ accF) {
  // per-wave LDS bitmap of the frame features this wave's node has claimed
  extern __shared__ __attribute__((aligned(16))) uint32_t claimBits[];
  const int lane = threadIdx.x & 63;
  const int a = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int words = (nF + 31) >> 5;
  uint32_t* claimed = claimBits + (threadIdx.x >> 6) * words;
  for (int i = lane; i < words; i += 64) claimed[i] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (a >= kfNodes) return;
  const uint32_t id = kfNodeIds[a];
  int lo = 0, hi = fNodes;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (fNodeIds[mid] < id) lo = mid + 1; else hi = mid;
  }
  const bool found = lo < fNodes && fNodeIds[lo] == id;
  for (int p = kfOffs[a]; p < kfOffs[a + 1]; ++p) {
    accF[p] = -1;
    if (!found) continue;
    const int realIdxKF = (int)kfFeats[p];
    if (kfMp[realIdxKF] < 0) continue;
    if (kfBad && kfBad[realIdxKF]) continue;
    const ulonglong4 dKF = load_desc(kfDesc + (size_t)realIdxKF * 32);
    const int fb = fOffs[lo], fe = fOffs[lo + 1];
    // per-lane first-two in (dist, position) order, then a wave merge
    int d1 = 256, q1 = 1 << 30, d2 = 256, q2 = 1 << 30;
    for (int q = fb + lane; q < fe; q += 64) {
      const int realIdxF = (int)fFeats[q];
      if ((claimed[realIdxF >> 5] >> (realIdxF & 31)) & 1u) continue;
      if (fMp && (fMp[realIdxF] < 0 || (fBad && fBad[realIdxF]))) continue;  // KF-KF (:628-632)
      const int dist = hamming256(dKF, load_desc(fDesc + (size_t)realIdxF * 32));
      if (dist < d1) { d2 = d1; q2 = q1; d1 = dist; q1 = q; }
      else if (dist < d2) { d2 = dist; q2 = q; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int od1 = __shfl_xor(d1, o, 64), oq1 = __shfl_xor(q1, o, 64);
      const int od2 = __shfl_xor(d2, o, 64), oq2 = __shfl_xor(q2, o, 64);
      // merge two sorted pairs by (dist, position)
      const bool mineFirst = d1 < od1 || (d1 == od1 && q1 < oq1);
      int n1d, n1q, c1d, c1q, c2d, c2q;
      if (mineFirst) { n1d = d1; n1q = q1; c1d = d2; c1q = q2; c2d = od1; c2q = oq1; }
      else { n1d = od1; n1q = oq1; c1d = od2; c1q = oq2; c2d = d1; c2q = q1; }
      const bool c1First = c1d < c2d || (c1d == c2d && c1q < c2q);
      d1 = n1d; q1 = n1q;
      d2 = c1First ? c1d : c2d;
      q2 = c1First ? c1q : c2q;
    }
    // TH_LOW: <= 50 against a Frame (:239), < 50 between KeyFrames (:650)
    if (d1 <= thLow && (float)d1 < nnratio * (float)d2) {
      const int realIdxF = (int)fFeats[q1];
      if (lane == 0) {
        claimed[realIdxF >> 5] |= 1u << (realIdxF & 31);
        accF[p] = realIdxF;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Output: against a Frame (fMp == NULL) fMatch[f] = the KeyFrame keypoint's
// MapPoint id; between KeyFrames fMatch[kf keypoint] = the matched KF2
// keypoint's MapPoint id (vpMatches12).  Rotation-filtered matches stay -1.
__global__ __launch_bounds__(256) void k_bow_finish(
    int nKfFeats, const uint32_t* __restrict__ kfFeats, const float* __restrict__ kfAngle,
    const float* __restrict__ fAngle, int checkOri, const int32_t* __restrict__ accF,
    const int32_t* __restrict__ kfMp, const int32_t* __restrict__ fMp,
    int32_t* __restrict__ fMatch, int32_t* __restrict__ nmatches) {
  __shared__ int hist[32];
  __shared__ int tmp[17];
  const int t = threadIdx.x;
  if (t < 32) hist[t] = 0;
  __syncthreads();
  int acc = 0;
  for (int p = t; p < nKfFeats; p += 256) {
    const int f = accF[p];
    if (f < 0) continue;
    ++acc;
    if (checkOri) atomicAdd(&hist[rot_bin(kfAngle[kfFeats[p]] - fAngle[f])], 1);
  }
  __syncthreads();
  int ind1 = -1, ind2 = -1, ind3 = -1;
  if (checkOri) three_maxima(hist, ind1, ind2, ind3);
  int removed = 0;
  for (int p = t; p < nKfFeats; p += 256) {
    const int f = accF[p];
    if (f < 0) continue;
    if (checkOri) {
      const int b = rot_bin(kfAngle[kfFeats[p]] - fAngle[f]);
      if (b != ind1 && b != ind2 && b != ind3) {
        ++removed;
        continue;
      }
    }
    const int k = (int)kfFeats[p];
    if (fMp) fMatch[k] = fMp[f];
    else fMatch[f] = kfMp[k];
  }
  int totA, totR;
  block_excl_scan(acc, tmp, &totA);
  block_excl_scan(removed, tmp, &totR);
  if (t == 0) *nmatches = totA - totR;
}

extern "C" hipError_t orb_k_bow(const uint8_t* kfDesc, const float* kfAngle, const int32_t* kfMp,
                                const uint8_t* kfBad, int kfNodes, const uint32_t* kfNodeIds,
                                const int32_t* kfOffs, const uint32_t* kfFeats, int nKfFeats,
                                const uint8_t* fDesc, const float* fAngle, int fNodes,
                                const uint32_t* fNodeIds, const int32_t* fOffs,
                                const uint32_t* fFeats, int nF, const int32_t* fMp,
                                const uint8_t* fBad, int thLow, float nnratio, int checkOri,
                                int32_t* fMatch, int32_t* accF, int32_t* nmatches,
                                hipStream_t s) {
  if (kfNodes > 0) {
    const size_t lds = 4 * (size_t)((nF + 31) / 32) * 4;
    if (lds > 65536) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_bow_match, dim3((kfNodes + 3) / 4), dim3(256), lds, s, kfDesc, kfAngle,
                       kfMp, kfBad, kfNodes, kfNodeIds, kfOffs, kfFeats, fDesc, fAngle, fNodes,
                       fNodeIds, fOffs, fFeats, nnratio, nF, fMp, fBad, thLow, accF);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_bow_finish, dim3(1), dim3(256), 0, s, nKfFeats, kfFeats, kfAngle, fAngle,
                     checkOri, accF, kfMp, fMp, fMatch, nmatches);
  return hipGetLastError();
}

// ================================================================ k_frustum
// Tracking::SearchLocalPoints' frustum pass (src/Tracking.cc:1360-1377):
// Frame::isInFrustum (src/Frame.cc:303-366) + MapPoint::PredictScale
// (src/MapPoint.cc:435-450), one thread per map point, one grid row per
// problem.  Pinned arithmetic (oracle/orb_oracle.cpp frustum_one):
//   Pc = Rcw*P + tcw       float, left-to-right dot, then + t (cv::gemm 3x3 path)
//   dist = cv::norm(P-Ow)  double sum of squares, double sqrt, to float
//   viewCos = PO.dot(Pn)/dist   double dot / double(dist), to float
//   level = ceil(logf(maxDist/dist) / logScale) with logf pinned to pinned_log
struct FrustumParams {
  float fx, fy, cx, cy, bf;
  float minX, maxX, minY, maxY;
  float cosLimit, logScale;
  int nLevels;
};

__global__ __launch_bounds__(256) void k_frustum(const orb_map_point_t* __restrict__ mps,
                                                 const int32_t* __restrict__ nmps, int mpStride,
                                                 const orb_pose_t* __restrict__ poses,
                                                 FrustumParams fp,
                                                 orb_mp_track_t* __restrict__ tracks,
                                                 int32_t* __restrict__ nInView) {
  const int p = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int M = nmps[p];
  bool in = false;
  if (i < M) {
    const orb_map_point_t mp = mps[(long long)p * mpStride + i];
    const orb_pose_t& T = poses[p];
    orb_mp_track_t tr;
    tr.proj_x = tr.proj_y = tr.proj_xr = tr.view_cos = 0.f;
    tr.level = 0;
    tr.bad = mp.bad;
    tr.has_obs = mp.has_obs;
    tr._pad = 0;
    if (!mp.seen && !mp.bad) {
      const float P0 = mp.pos[0], P1 = mp.pos[1], P2 = mp.pos[2];
      const float X = ((T.rcw[0] * P0 + T.rcw[1] * P1) + T.rcw[2] * P2) + T.tcw[0];
      const float Y = ((T.rcw[3] * P0 + T.rcw[4] * P1) + T.rcw[5] * P2) + T.tcw[1];
      const float Z = ((T.rcw[6] * P0 + T.rcw[7] * P1) + T.rcw[8] * P2) + T.tcw[2];
      if (!(Z < 0.0f)) {
        const float invz = __fdiv_rn(1.0f, Z);
        const float u = fp.fx * X * invz + fp.cx;
        const float v = fp.fy * Y * invz + fp.cy;
        if (!(u < fp.minX || u > fp.maxX) && !(v < fp.minY || v > fp.maxY)) {
          const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
          const float O0 = P0 - T.ow[0], O1 = P1 - T.ow[1], O2 = P2 - T.ow[2];
          const double ss = (((double)O0 * O0) + (double)O1 * O1) + (double)O2 * O2;
          const float dist = (float)__dsqrt_rn(ss);
          if (!(dist < minD || dist > maxD)) {
            const double dot = (((double)O0 * mp.normal[0]) + (double)O1 * mp.normal[1]) +
                               (double)O2 * mp.normal[2];
            const float viewCos = (float)(dot / (double)dist);
            if (!(viewCos < fp.cosLimit)) {
              const float ratio = __fdiv_rn(mp.max_distance, dist);
              const float lr = (float)pinned_log((double)ratio);
              const float q = ceilf(__fdiv_rn(lr, fp.logScale));
              int lvl;
              if (q < 0.f) lvl = 0;
              else if (q >= (float)fp.nLevels) lvl = fp.nLevels - 1;
              else lvl = (int)q;
              tr.proj_x = u;
              tr.proj_y = v;
              tr.proj_xr = u - fp.bf * invz;
              tr.view_cos = viewCos;
              tr.level = lvl;
              in = true;
            }
          }
        }
      }
    }
    tr.in_view = in ? 1 : 0;
    tracks[(long long)p * mpStride + i] = tr;
  }
  const int c = __popcll(__ballot(in));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&nInView[p], c);
}

extern "C" size_t orb_k_frustum_params_size(void) { return sizeof(FrustumParams); }

extern "C" hipError_t orb_k_frustum(const orb_map_point_t* mps, const int32_t* nmps, int mpStride,
                         int mpMax, const orb_pose_t* poses, const void* params,
                         orb_mp_track_t* tracks, int32_t* nInView, int nproblems, hipStream_t s) {
  hipError_t e = hipMemsetAsync(nInView, 0, sizeof(int32_t) * nproblems, s);
  if (e != hipSuccess) return e;
  if (mpMax <= 0) return hipSuccess;
  const FrustumParams fp = *static_cast<const FrustumParams*>(params);
  hipLaunchKernelGGL(k_frustum, dim3((mpMax + 255) / 256, nproblems), dim3(256), 0, s, mps, nmps,
                     mpStride, poses, fp, tracks, nInView);
  return hipGetLastError();
}
