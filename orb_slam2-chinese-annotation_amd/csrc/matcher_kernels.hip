// matcher_kernels.hip -- gfx950 kernels of the Hamming matcher (ORBmatcher + Frame grid).
//
// Hamming distance = 4 x __popcll over the 256-bit descriptors (no MFMA: these
// are bit-count/compare kernels).  The reference matchers are sequential with
// "first-come" keypoint claims (src/ORBmatcher.cc:90-93,127), so each matcher
// is split into a data-parallel distance stage that keeps, per query, the
// first K candidates in (distance, scan order) order, and an ordered resolve
// stage that replays the sequential semantics exactly.
#include "orb_device.h"
#include "../../include/orb_abi.h"

#define GRID_CELLS (ORB_GRID_COLS * ORB_GRID_ROWS)
#define TOPK 4

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
// One wave per frame.
__device__ __forceinline__ int grid_cell(const orb_keypoint_t& k, float minX, float minY,
                                         float invW, float invH) {
  const int px = (int)round_half_away((k.x - minX) * invW);
  const int py = (int)round_half_away((k.y - minY) * invH);
  if (px < 0 || px >= ORB_GRID_COLS || py < 0 || py >= ORB_GRID_ROWS) return -1;
  return px * ORB_GRID_ROWS + py;
}

__global__ __launch_bounds__(64) void k_grid_build(const orb_keypoint_t* __restrict__ keys,
                                                   const int32_t* __restrict__ nkeys, int kpStride,
                                                   float minX, float minY, float invW, float invH,
                                                   int32_t* __restrict__ cellStart,
                                                   int32_t* __restrict__ cellIdx) {
  __shared__ int cnt[GRID_CELLS + 1];
  const int p = blockIdx.x, lane = threadIdx.x;
  const int n = nkeys[p];
  const orb_keypoint_t* K = keys + (size_t)p * kpStride;
  for (int i = lane; i <= GRID_CELLS; i += 64) cnt[i] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  for (int k = lane; k < n; k += 64) {
    const int c = grid_cell(K[k], minX, minY, invW, invH);
    if (c >= 0) atomicAdd(&cnt[c], 1);
  }
  __syncthreads();
  // exclusive scan over 3072 cells: 48 consecutive cells per lane
  {
    const int per = GRID_CELLS / 64;
    int s = 0;
    for (int i = 0; i < per; ++i) s += cnt[lane * per + i];
    int ex = wave_incl_scan(s) - s;
    for (int i = 0; i < per; ++i) {
      const int v = cnt[lane * per + i];
      cnt[lane * per + i] = ex;
      ex += v;
    }
    if (lane == 63) cnt[GRID_CELLS] = ex;
  }
  __syncthreads();
  int32_t* cs = cellStart + (size_t)p * (GRID_CELLS + 1);
  for (int i = lane; i <= GRID_CELLS; i += 64) cs[i] = cnt[i];
  __syncthreads();
  // stable scatter in keypoint order, 64 keys at a time; lanes holding the same
  // cell find each other with 12 ballots over the cell id bits
  int32_t* ci = cellIdx + (size_t)p * kpStride;
  const unsigned long long ltMask = (1ull << lane) - 1ull;
  for (int base = 0; base < n; base += 64) {
    const int k = base + lane;
    int c = k < n ? grid_cell(K[k], minX, minY, invW, invH) : -1;
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
      if ((peers >> lane) == 1ull) cnt[c] += __popcll(peers);  // highest lane of the group
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ------------------------------------------ SearchByProjection(F, localMap)
struct ProjParams {
  float minX, minY, invW, invH;
  float th, nnratio;
  int nLevels;
  float scale[ORB_MAX_LEVELS];
};

// Top-K entry: keypoint index (19b) | distance (9b) << 19 | octave (4b) << 28.
__device__ __forceinline__ uint32_t pack_cand(int idx, int dist, int oct) {
  return (uint32_t)idx | ((uint32_t)dist << 19) | ((uint32_t)oct << 28);
}
__device__ __forceinline__ int cand_idx(uint32_t e) { return (int)(e & 0x7FFFFu); }
__device__ __forceinline__ int cand_dist(uint32_t e) { return (int)((e >> 19) & 0x1FFu); }
__device__ __forceinline__ int cand_oct(uint32_t e) { return (int)(e >> 28); }

// Visit, in GetFeaturesInArea order (src/Frame.cc:368-424), every keypoint of
// the window that passes the level and |dx|,|dy| < r tests.
template <typename F>
__device__ __forceinline__ void for_features_in_area(const orb_keypoint_t* K,
                                                     const int32_t* cs, const int32_t* ci,
                                                     const ProjParams& P, float x, float y,
                                                     float r, int minLevel, int maxLevel,
                                                     F&& visit) {
  const int nMinCellX = max(0, (int)floorf((x - P.minX - r) * P.invW));
  if (nMinCellX >= ORB_GRID_COLS) return;
  const int nMaxCellX = min(ORB_GRID_COLS - 1, (int)ceilf((x - P.minX + r) * P.invW));
  if (nMaxCellX < 0) return;
  const int nMinCellY = max(0, (int)floorf((y - P.minY - r) * P.invH));
  if (nMinCellY >= ORB_GRID_ROWS) return;
  const int nMaxCellY = min(ORB_GRID_ROWS - 1, (int)ceilf((y - P.minY + r) * P.invH));
  if (nMaxCellY < 0) return;
  const bool checkLevels = (minLevel > 0) || (maxLevel >= 0);
  for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
    for (int iy = nMinCellY; iy <= nMaxCellY; ++iy) {
      const int c = ix * ORB_GRID_ROWS + iy;
      const int e = cs[c + 1];
      for (int j = cs[c]; j < e; ++j) {
        const int idx = ci[j];
        const orb_keypoint_t& kp = K[idx];
        if (checkLevels) {
          if (kp.octave < minLevel) continue;
          if (maxLevel >= 0 && kp.octave > maxLevel) continue;
        }
        const float dx = kp.x - x, dy = kp.y - y;
        if (fabsf(dx) < r && fabsf(dy) < r) visit(idx, kp);
      }
    }
  }
}

// Per map point: candidate scan + first-K in (dist, scan order); counts every
// candidate that could ever be best/second (dist < 256, not pre-locked, passes
// the stereo gate).  ncand = -1 marks a point the reference skips outright.
__global__ __launch_bounds__(256) void k_proj_candidates(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked, int kpStride,
    const orb_mp_track_t* __restrict__ mps, const uint8_t* __restrict__ mpDesc,
    const int32_t* __restrict__ nmps, int mpStride, const int32_t* __restrict__ cellStart,
    const int32_t* __restrict__ cellIdx, ProjParams P, uint32_t* __restrict__ topk,
    int32_t* __restrict__ ncand) {
  const int p = blockIdx.y;
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nmps[p]) return;
  const size_t mg = (size_t)p * mpStride + m;
  const orb_mp_track_t mp = mps[mg];
  if (!mp.in_view || mp.bad) {
    ncand[mg] = -1;
    return;
  }
  const int lvl = mp.level;
  float r = (double)mp.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:135-141)
  if (P.th != 1.0f) r *= P.th;
  const float rs = r * P.scale[lvl];
  const orb_keypoint_t* K = keys + (size_t)p * kpStride;
  const uint8_t* D = desc + (size_t)p * kpStride * 32;
  const uint8_t* LK = locked ? locked + (size_t)p * kpStride : nullptr;
  const float* UR = uright ? uright + (size_t)p * kpStride : nullptr;
  const int32_t* cs = cellStart + (size_t)p * (GRID_CELLS + 1);
  const int32_t* ci = cellIdx + (size_t)p * kpStride;
  const ulonglong4 q = load_desc(mpDesc + mg * 32);
  uint32_t top[TOPK];
  int ntop = 0, count = 0;
  for_features_in_area(K, cs, ci, P, mp.proj_x, mp.proj_y, rs, lvl - 1, lvl,
                       [&](int idx, const orb_keypoint_t& kp) {
                         if (LK && LK[idx]) return;
                         if (UR && UR[idx] > 0) {
                           const float er = fabsf(mp.proj_xr - UR[idx]);
                           if (er > r * P.scale[lvl]) return;
                         }
                         const int dist = hamming256(q, load_desc(D + (size_t)idx * 32));
                         if (dist >= 256) return;  // can never become best or second
                         ++count;
                         // stable insertion: after existing entries with equal distance
                         int pos = ntop;
                         while (pos > 0 && cand_dist(top[pos - 1]) > dist) --pos;
                         if (pos >= TOPK) return;
                         const int last = ntop < TOPK ? ntop : TOPK - 1;
                         for (int j = last; j > pos; --j) top[j] = top[j - 1];
                         top[pos] = pack_cand(idx, dist, kp.octave);
                         if (ntop < TOPK) ++ntop;
                       });
  for (int j = 0; j < TOPK; ++j) topk[mg * TOPK + j] = j < ntop ? top[j] : 0xFFFFFFFFu;
  ncand[mg] = count;
}

// Sequential-semantics resolve, one wave per problem, speculatively 64 map
// points at a time: every lane evaluates its point against the claims made so
// far; lane i's result stands unless an earlier lane of the same window claims
// (and locks) a keypoint among the top-K entries lane i looked at.  The longest
// conflict-free prefix is committed, the window restarts after it.  A point
// whose top-K ran dry (more than K candidates, too many claimed) is re-scanned
// exactly once it is first in its window.
__device__ __forceinline__ bool lock_test(const uint32_t* bm, int idx) {
  return (bm[idx >> 5] >> (idx & 31)) & 1u;
}

#define RES_CHUNK 256

__global__ __launch_bounds__(64) void k_proj_resolve(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const uint8_t* __restrict__ locked,
    const int32_t* __restrict__ nkeys, int kpStride, const orb_mp_track_t* __restrict__ mps,
    const uint8_t* __restrict__ mpDesc, const int32_t* __restrict__ nmps, int mpStride,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, ProjParams P,
    const uint32_t* __restrict__ topk, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ kpMatch, int32_t* __restrict__ nmatches) {
  // LDS: lock bitmap (1 bit / keypoint), earliest claiming lane per keypoint
  // of the current window, and a prefetched chunk of per-point resolve inputs
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ uint4 cTop[RES_CHUNK];
  __shared__ int cN[RES_CHUNK];
  __shared__ uint8_t cObs[RES_CHUNK];
  const int p = blockIdx.x, lane = threadIdx.x;
  const int n = nkeys[p], M = nmps[p];
  const int words = (kpStride + 31) >> 5;
  uint32_t* bm = dyn;
  int* claimBy = (int*)(dyn + ((words + 3) & ~3));
  for (int i = lane; i < words; i += 64) bm[i] = 0u;
  for (int i = lane; i < kpStride; i += 64) claimBy[i] = 64;
  int32_t* km = kpMatch + (size_t)p * kpStride;
  for (int i = lane; i < n; i += 64) km[i] = -1;
  __syncthreads();
  const float nnratio = P.nnratio;
  const size_t pbase = (size_t)p * mpStride;
  int matches = 0;
  int start = 0;
  int cb = -RES_CHUNK;  // first point held in the LDS chunk
  while (start < M) {
    if (start + 64 > cb + RES_CHUNK && cb + RES_CHUNK < M) {  // slide the chunk to `start`
      cb = start;
      __syncthreads();
      for (int j = lane; j < RES_CHUNK; j += 64) {
        const int m = cb + j;
        if (m < M) {
          cTop[j] = *reinterpret_cast<const uint4*>(topk + (pbase + m) * TOPK);
          cN[j] = ncand[pbase + m];
          cObs[j] = mps[pbase + m].has_obs;
        }
      }
      __syncthreads();
    }
    const int m = start + lane;
    const bool active = m < M;
    int nc = -1;
    uint32_t e[TOPK];
    bool hasObs = false;
    if (active) {
      const int j = m - cb;
      nc = cN[j];
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
    bool accept = false;
    if (nc > 0 && !slow && bestDist <= 100)
      accept = !(bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2);
    const bool locks = accept && hasObs;
    // conflict: an earlier lane of this window locks a keypoint this lane looked at
    if (locks) atomicMin(&claimBy[bestIdx], lane);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bool conflict = false;
    for (int q = 0; q < consumed; ++q) conflict |= claimBy[cand_idx(e[q])] < lane;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (locks) claimBy[bestIdx] = 64;
    const unsigned long long bad = __ballot(active && (conflict || (slow && lane > 0)));
    const unsigned long long slowFirst = __ballot(lane == 0 && active && slow);
    int commit = bad ? (int)__builtin_ctzll(bad) : 64;
    if (slowFirst) {
      // exact re-scan of the first point of the window, lane 0, current locks
      if (lane == 0) {
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
      if (lane < commit && accept) {
        atomicMax(&km[bestIdx], m);
        if (locks) atomicOr(&bm[bestIdx >> 5], 1u << (bestIdx & 31));
      }
      matches += __popcll(__ballot(lane < commit && accept));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    start += commit;
  }
  if (lane == 0) nmatches[p] = matches;
}

// ------------------------------------------------------------ host launchers
extern "C" {

hipError_t orb_k_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hamming_batch, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

hipError_t orb_k_grid_build(const orb_keypoint_t* keys, const int32_t* nkeys, int kpStride,
                            float minX, float minY, float invW, float invH, int32_t* cellStart,
                            int32_t* cellIdx, int nproblems, hipStream_t s) {
  hipLaunchKernelGGL(k_grid_build, dim3(nproblems), dim3(64), 0, s, keys, nkeys, kpStride, minX,
                     minY, invW, invH, cellStart, cellIdx);
  return hipGetLastError();
}

hipError_t orb_k_proj_candidates(const orb_keypoint_t* keys, const uint8_t* desc,
                                 const float* uright, const uint8_t* locked, int kpStride,
                                 const orb_mp_track_t* mps, const uint8_t* mpDesc,
                                 const int32_t* nmps, int mpStride, int mpMax,
                                 const int32_t* cellStart, const int32_t* cellIdx,
                                 const void* params, uint32_t* topk, int32_t* ncand,
                                 int nproblems, hipStream_t s) {
  const ProjParams P = *(const ProjParams*)params;
  if (mpMax <= 0 || nproblems <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_proj_candidates, dim3((mpMax + 255) / 256, nproblems), dim3(256), 0, s,
                     keys, desc, uright, locked, kpStride, mps, mpDesc, nmps, mpStride, cellStart,
                     cellIdx, P, topk, ncand);
  return hipGetLastError();
}

hipError_t orb_k_proj_resolve(const orb_keypoint_t* keys, const uint8_t* desc,
                              const float* uright, const uint8_t* locked, const int32_t* nkeys,
                              int kpStride, const orb_mp_track_t* mps, const uint8_t* mpDesc,
                              const int32_t* nmps, int mpStride, const int32_t* cellStart,
                              const int32_t* cellIdx, const void* params, const uint32_t* topk,
                              const int32_t* ncand, int32_t* kpMatch, int32_t* nmatches,
                              int nproblems, hipStream_t s) {
  const ProjParams P = *(const ProjParams*)params;
  if (nproblems <= 0) return hipSuccess;
  const size_t words = (size_t)((kpStride + 31) / 32);
  const size_t lds = ((words + 3) & ~(size_t)3) * 4 + (size_t)kpStride * 4;
  hipLaunchKernelGGL(k_proj_resolve, dim3(nproblems), dim3(64), lds, s, keys, desc, uright,
                     locked, nkeys, kpStride, mps, mpDesc, nmps, mpStride, cellStart, cellIdx, P,
                     topk, ncand, kpMatch, nmatches);
  return hipGetLastError();
}

size_t orb_k_proj_params_size(void) { return sizeof(ProjParams); }

}  // extern "C"
