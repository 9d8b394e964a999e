// mapping_kernels.hip -- gfx950 kernels of the matcher callers widened from
// ORBmatcher::SearchForInitialization (monocular map
// initialisation) and MapPoint::ComputeDistinctiveDescriptors (LocalMapping /
// Tracking descriptor refresh).  Both are Hamming bit-count work: VALU
// (v_bcnt) and wave ballots, no MFMA.
#include <algorithm>
#include <climits>

#include "matcher_common.h"

// ================================================= SearchForInitialization
// src/ORBmatcher.cc:429-577.  For each level-0 keypoint i1 of F1 (in order):
// the level-0 F2 keypoints in the window around vbPrevMatched[i1], skipping
// those already matched at a distance <= this one (vMatchedDistance), best /
// second-best (first minimum in scan order), accept if best <= TH_LOW and
// best < second * nnratio, stealing the F2 keypoint from its previous owner.
//
// k_init_prep (one workgroup per problem): the level-0 F1 queries in order,
// and the level-0 F2 keypoints in grid-scan order (the CSR order of the Frame
// grid: GetFeaturesInArea visits cells ix-major, iy-minor, ascending index,
// so any window's scan order is this order restricted to the window).
// k_init_candidates (thread per query): the staged F2 list and descriptors in
// LDS, each query tests every entry against its cell range and |dx|,|dy| < r
// -- the same set GetFeaturesInArea returns, in the same order -- and keeps
// every candidate (up to INIT_LIST, packed idx|dist) and the first INIT_TOPK
// in (distance, scan order).
// k_init_resolve (one wave per problem): speculative in-order resolve of 64
// consecutive queries at a time.  vMatchedDistance only decreases, so a
// query's surviving candidates only shrink; its (best, second) stays exact
// unless an earlier query of the same batch accepts one of those two
// keypoints.  Lanes up to the first such conflict commit together (no two
// committed lanes then accept the same keypoint); a query whose top-K list ran
// out of survivors is resolved exactly by the whole wave from its full list.
#define INIT_TOPK 16
#define INIT_LIST 256
#define INIT_STAGE 1536  // F2 level-0 keypoints staged in LDS (48 B each)
#define INIT_WG 256

struct InitParams {
  float minX, minY, invW, invH;
  float r, nnratio;
  int checkOri;
};

// staged F2 keypoint: position, grid cell (ix << 16 | iy), original index
struct InitKey {
  float x, y;
  uint32_t cell;
  int32_t idx;
};

template <int K>
struct TopKReg {
  uint32_t t[K];
  __device__ __forceinline__ TopKReg() {
#pragma unroll
    for (int j = 0; j < K; ++j) t[j] = 0xFFFFFFFFu;
  }
  // stable sorted insertion after equal distances (same network as Top4)
  __device__ __forceinline__ void insert(uint32_t e, int d) {
    bool b[K];
#pragma unroll
    for (int j = 0; j < K; ++j) b[j] = cand_dist(t[j]) > d;
#pragma unroll
    for (int j = K - 1; j > 0; --j) t[j] = b[j - 1] ? t[j - 1] : (b[j] ? e : t[j]);
    t[0] = b[0] ? e : t[0];
  }
};

__global__ __launch_bounds__(INIT_WG) void k_init_prep(
    const orb_keypoint_t* __restrict__ keys1, const int32_t* __restrict__ n1s,
    const orb_keypoint_t* __restrict__ keys2, int kpStride, const float* __restrict__ prev,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, InitParams P,
    int32_t* __restrict__ qList, int32_t* __restrict__ qOrder, int32_t* __restrict__ nQ,
    InitKey* __restrict__ stage, int32_t* __restrict__ nStage) {
  __shared__ int tmp[17];
  const int p = blockIdx.x, t = threadIdx.x;
  const size_t base = (size_t)p * kpStride;
  const int N1 = n1s[p];
  int total = 0, off = 0;
  for (int c0 = 0; c0 < N1; c0 += INIT_WG) {  // level-0 queries, :449-451
    const int i = c0 + t;
    const bool keep = i < N1 && keys1[base + i].octave == 0;
    const int ex = block_excl_scan(keep ? 1 : 0, tmp, &total);
    if (keep) qList[base + off + ex] = i;
    off += total;
  }
  if (t == 0) nQ[p] = off;
  // processing order for k_init_candidates: queries bucketed by the grid
  // column of their window centre, so a wave's windows overlap and it scans
  // one narrow range of the staged list (results still go to slot k)
  __shared__ int colCnt[ORB_GRID_COLS];
  const int nq = off;
  if (t < ORB_GRID_COLS) colCnt[t] = 0;
  __syncthreads();
  for (int k = t; k < nq; k += INIT_WG) {
    const float x = prev[(base + qList[base + k]) * 2];
    const int b = min(ORB_GRID_COLS - 1, max(0, (int)floorf((x - P.minX) * P.invW)));
    atomicAdd(&colCnt[b], 1);
  }
  __syncthreads();
  if (t < 64) {
    const int v = colCnt[t];
    colCnt[t] = wave_incl_scan(v) - v;
  }
  __syncthreads();
  for (int k = t; k < nq; k += INIT_WG) {
    const float x = prev[(base + qList[base + k]) * 2];
    const int b = min(ORB_GRID_COLS - 1, max(0, (int)floorf((x - P.minX) * P.invW)));
    qOrder[base + atomicAdd(&colCnt[b], 1)] = k;
  }
  const int32_t* cs = cellStart + (size_t)p * (GRID_CELLS + 1);
  const int32_t* ci = cellIdx + base;
  const orb_keypoint_t* K2 = keys2 + base;
  const int M = cs[GRID_CELLS];
  off = 0;
  for (int c0 = 0; c0 < M; c0 += INIT_WG) {  // GetFeaturesInArea(.., 0, 0) level filter
    const int pos = c0 + t;
    int idx = -1;
    orb_keypoint_t k;
    if (pos < M) {
      idx = ci[pos];
      k = K2[idx];
    }
    const bool keep = idx >= 0 && k.octave == 0;
    const int ex = block_excl_scan(keep ? 1 : 0, tmp, &total);
    if (keep) {
      const int c = grid_cell(k, P.minX, P.minY, P.invW, P.invH);
      InitKey e;
      e.x = k.x;
      e.y = k.y;
      e.cell = ((uint32_t)(c / ORB_GRID_ROWS) << 16) | (uint32_t)(c % ORB_GRID_ROWS);
      e.idx = idx;
      stage[base + off + ex] = e;
    }
    off += total;
  }
  if (t == 0) nStage[p] = off;
}

// Cell range of GetFeaturesInArea (src/Frame.cc:376-389); false = empty.
__device__ __forceinline__ bool init_window(const InitParams& P, float x, float y, int& x0,
                                            int& x1, int& y0, int& y1) {
  x0 = max(0, (int)floorf((x - P.minX - P.r) * P.invW));
  if (x0 >= ORB_GRID_COLS) return false;
  x1 = min(ORB_GRID_COLS - 1, (int)ceilf((x - P.minX + P.r) * P.invW));
  if (x1 < 0) return false;
  y0 = max(0, (int)floorf((y - P.minY - P.r) * P.invH));
  if (y0 >= ORB_GRID_ROWS) return false;
  y1 = min(ORB_GRID_ROWS - 1, (int)ceilf((y - P.minY + P.r) * P.invH));
  if (y1 < 0) return false;
  return true;
}

__global__ __launch_bounds__(INIT_WG) void k_init_candidates(
    const uint8_t* __restrict__ desc1, const uint8_t* __restrict__ desc2,
    const orb_keypoint_t* __restrict__ keys2, int kpStride, const float* __restrict__ prev,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, InitParams P,
    const int32_t* __restrict__ qList, const int32_t* __restrict__ qOrder,
    const int32_t* __restrict__ nQ, const InitKey* __restrict__ stage,
    const int32_t* __restrict__ nStage, uint32_t* __restrict__ topk,
    uint32_t* __restrict__ list, int32_t* __restrict__ ncand) {
  __shared__ __attribute__((aligned(16))) InitKey sKey[INIT_STAGE];
  __shared__ __attribute__((aligned(16))) ulonglong4 sDesc[INIT_STAGE];
  const int p = blockIdx.y, t = threadIdx.x;
  const int nq = nQ[p];
  if ((int)(blockIdx.x * INIT_WG) >= nq) return;  // uniform
  const size_t base = (size_t)p * kpStride;
  const int ns = nStage[p];
  const bool staged = ns <= INIT_STAGE;
  if (staged) {
    for (int j = t; j < ns; j += INIT_WG) {
      const InitKey e = stage[base + j];
      sKey[j] = e;
      sDesc[j] = load_desc(desc2 + (base + e.idx) * 32);
    }
  }
  __syncthreads();
  const int r = blockIdx.x * INIT_WG + t;
  if (r >= nq) return;
  const int k = qOrder[base + r];
  const int i1 = qList[base + k];
  const size_t qs = base + k;
  const ulonglong4 d1 = load_desc(desc1 + (base + i1) * 32);
  const float2 c = *reinterpret_cast<const float2*>(prev + (base + i1) * 2);
  TopKReg<INIT_TOPK> top;
  uint32_t* L = list + qs * INIT_LIST;
  int count = 0;
  auto visit = [&](int idx, int dist) {
    const uint32_t e = pack_cand(idx, dist, 0);
    if (count < INIT_LIST) L[count] = e;
    ++count;
    top.insert(e, dist);
  };
  if (staged) {
    int x0, x1, y0, y1;
    if (init_window(P, c.x, c.y, x0, x1, y0, y1)) {
      // entries are in cell order (ix-major): columns x0..x1 are one range
      const uint32_t lo = ((uint32_t)x0 << 16), hi = ((uint32_t)(x1 + 1) << 16);
      int jb = 0;
      for (int w = ns; w > 0;) {  // first entry with cell >= lo
        const int h = w >> 1;
        if (sKey[jb + h].cell < lo) { jb += h + 1; w -= h + 1; } else w = h;
      }
      int je = jb;
      for (int w = ns - jb; w > 0;) {  // first entry with cell >= hi
        const int h = w >> 1;
        if (sKey[je + h].cell < hi) { je += h + 1; w -= h + 1; } else w = h;
      }
      for (int j = jb; j < je; ++j) {
        const InitKey e = sKey[j];
        const int iy = (int)(e.cell & 0xFFFFu);
        if (iy < y0 || iy > y1) continue;
        const float dx = e.x - c.x, dy = e.y - c.y;
        if (fabsf(dx) < P.r && fabsf(dy) < P.r) visit(e.idx, hamming256(d1, sDesc[j]));
      }
    }
  } else {
    ProjParams G;
    G.minX = P.minX; G.minY = P.minY; G.invW = P.invW; G.invH = P.invH;
    const uint8_t* D2 = desc2 + base * 32;
    for_features_in_area(keys2 + base, cellStart + (size_t)p * (GRID_CELLS + 1), cellIdx + base,
                         G, c.x, c.y, P.r, 0, 0, [&](int idx, const orb_keypoint_t&) {
                           visit(idx, hamming256(d1, load_desc(D2 + (size_t)idx * 32)));
                         });
  }
  uint4* T = reinterpret_cast<uint4*>(topk + qs * INIT_TOPK);
#pragma unroll
  for (int j = 0; j < INIT_TOPK / 4; ++j)
    T[j] = make_uint4(top.t[4 * j], top.t[4 * j + 1], top.t[4 * j + 2], top.t[4 * j + 3]);
  ncand[qs] = count;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(64) void k_init_resolve(
    const orb_keypoint_t* __restrict__ keys1, const uint8_t* __restrict__ desc1,
    const int32_t* __restrict__ n1s, const orb_keypoint_t* __restrict__ keys2,
    const uint8_t* __restrict__ desc2, const int32_t* __restrict__ n2s, int kpStride,
    float* __restrict__ prev, const int32_t* __restrict__ cellStart,
    const int32_t* __restrict__ cellIdx, InitParams P, const int32_t* __restrict__ qList,
    const int32_t* __restrict__ nQ, const uint32_t* __restrict__ topk,
    const uint32_t* __restrict__ list, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ m12, int32_t* __restrict__ nmatches) {
  // LDS: vMatchedDistance, vnMatches21 (owner), earliest claiming lane of the
  // batch per F2 keypoint, and the F2 keypoint each i1 accepted (even if it
  // was stolen later: its histogram entry stays, :524-527)
  extern __shared__ __attribute__((aligned(16))) int sm[];
  __shared__ int hist[32];
  const int p = blockIdx.x, lane = threadIdx.x;
  const int N1 = n1s[p], N2 = n2s[p], NQ = nQ[p];
  const int n2pad = (N2 + 3) & ~3;
  int* vMD = sm;
  int* owner = vMD + n2pad;
  int* claimBy = owner + n2pad;
  int* acc = claimBy + n2pad;
  const size_t base = (size_t)p * kpStride;
  const orb_keypoint_t* K1 = keys1 + base;
  const orb_keypoint_t* K2 = keys2 + base;
  for (int i = lane; i < N2; i += 64) { vMD[i] = INT_MAX; owner[i] = -1; claimBy[i] = 64; }
  for (int i = lane; i < N1; i += 64) acc[i] = -1;
  if (lane < 32) hist[lane] = 0;
  __syncthreads();
  int start = 0;
  while (start < NQ) {
    const int k = start + lane;
    const bool active = k < NQ;
    int i1 = -1, nc = 0;
    if (active) {
      i1 = qList[base + k];
      nc = ncand[base + k];
    }
    int b1 = INT_MAX, b2 = INT_MAX, bi = -1, si = -1, found = 0;
    if (nc > 0) {
      const uint4* T = reinterpret_cast<const uint4*>(topk + (base + k) * INIT_TOPK);
      uint32_t e[INIT_TOPK];
#pragma unroll
      for (int j = 0; j < INIT_TOPK / 4; ++j) {
        const uint4 v = T[j];
        e[4 * j] = v.x; e[4 * j + 1] = v.y; e[4 * j + 2] = v.z; e[4 * j + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < INIT_TOPK; ++j) {
        if (j < nc && found < 2) {
          const int i2 = cand_idx(e[j]), d = cand_dist(e[j]);
          if (vMD[i2] > d) {
            if (found == 0) { b1 = d; bi = i2; }
            else { b2 = d; si = i2; }
            ++found;
          }
        }
      }
    }
    const bool slow = found < 2 && nc > INIT_TOPK;
    const bool accept =
        !slow && bi >= 0 && b1 <= 50 && (float)b1 < (float)b2 * P.nnratio;  // :488-492
    if (accept) atomicMin(&claimBy[bi], lane);
    wave_sync_lds();
    const bool conflict = (bi >= 0 && claimBy[bi] < lane) || (si >= 0 && claimBy[si] < lane);
    wave_sync_lds();
    if (accept) claimBy[bi] = 64;
    const unsigned long long bad = __ballot(active && (conflict || slow));
    const int commit = bad ? (int)__builtin_ctzll(bad) : 64;
    // lanes before the first bad one commit; their keypoints are distinct
    if (active && lane < commit && accept) {
      owner[bi] = i1;  // a previous owner (earlier batch) loses the keypoint
      vMD[bi] = b1;
      acc[i1] = bi;
    }
    int advance = commit;
    if (commit < 64 && ((__ballot(slow) >> commit) & 1ull)) {
      // the first bad query ran out of top-K survivors: resolve it exactly,
      // wave-wide, from its full candidate list against the updated state
      wave_sync_lds();
      const int q1 = __builtin_amdgcn_readlane(i1, commit);
      const int ncq = __builtin_amdgcn_readlane(nc, commit);
      const int qk = start + commit;
      int eb1 = INT_MAX, eb2 = INT_MAX, ebi = -1;
      if (ncq <= INIT_LIST) {
        const uint32_t* Lq = list + (base + qk) * INIT_LIST;
        uint32_t k1 = 0xFFFFFFFFu, k2 = 0xFFFFFFFFu;  // (dist << 8 | position)
        for (int c0 = 0; c0 < ncq; c0 += 64) {
          const int pos = c0 + lane;
          uint32_t key = 0xFFFFFFFFu;
          if (pos < ncq) {
            const uint32_t e = Lq[pos];
            if (vMD[cand_idx(e)] > cand_dist(e)) key = ((uint32_t)cand_dist(e) << 8) | pos;
          }
          const uint32_t m1 = wave_min_u32(key);
          const uint32_t m2 = wave_min_u32(key == m1 ? 0xFFFFFFFFu : key);
          // merge the sorted pairs (k1, k2) and (m1, m2)
          const uint32_t lo = min(k1, m1), hi = max(k1, m1);
          k2 = min(hi, min(k2, m2));
          k1 = lo;
        }
        if (k1 != 0xFFFFFFFFu) { eb1 = (int)(k1 >> 8); ebi = cand_idx(Lq[k1 & 255u]); }
        if (k2 != 0xFFFFFFFFu) eb2 = (int)(k2 >> 8);
      } else if (lane == 0) {  // more than INIT_LIST candidates: rescan the window
        ProjParams G;
        G.minX = P.minX; G.minY = P.minY; G.invW = P.invW; G.invH = P.invH;
        const ulonglong4 d1 = load_desc(desc1 + (base + q1) * 32);
        const float2 c = *reinterpret_cast<const float2*>(prev + (base + q1) * 2);
        for_features_in_area(K2, cellStart + (size_t)p * (GRID_CELLS + 1), cellIdx + base, G,
                             c.x, c.y, P.r, 0, 0, [&](int idx, const orb_keypoint_t&) {
                               const int d =
                                   hamming256(d1, load_desc(desc2 + (base + idx) * 32));
                               if (vMD[idx] <= d) return;
                               if (d < eb1) { eb2 = eb1; eb1 = d; ebi = idx; }
                               else if (d < eb2) eb2 = d;
                             });
      }
      eb1 = __builtin_amdgcn_readfirstlane(eb1);
      eb2 = __builtin_amdgcn_readfirstlane(eb2);
      ebi = __builtin_amdgcn_readfirstlane(ebi);
      if (lane == 0 && ebi >= 0 && eb1 <= 50 && (float)eb1 < (float)eb2 * P.nnratio) {
        owner[ebi] = q1;
        vMD[ebi] = eb1;
        acc[q1] = ebi;
      }
      advance = commit + 1;
    }
    wave_sync_lds();
    start += advance;
  }
  // rotation histogram over every acceptance, ComputeThreeMaxima, filter
  if (P.checkOri)
    for (int i = lane; i < N1; i += 64) {
      const int a = acc[i];
      if (a >= 0) atomicAdd(&hist[rot_bin(K1[i].angle - K2[a].angle)], 1);
    }
  wave_sync_lds();
  int ind1 = -1, ind2 = -1, ind3 = -1;
  if (P.checkOri) three_maxima(hist, ind1, ind2, ind3);
  int n = 0;
  for (int i = lane; i < N1; i += 64) {
    const int a = acc[i];
    int m = (a >= 0 && owner[a] == i) ? a : -1;
    if (m >= 0 && P.checkOri) {
      const int b = rot_bin(K1[i].angle - K2[a].angle);
      if (b != ind1 && b != ind2 && b != ind3) m = -1;
    }
    m12[base + i] = m;
    if (m >= 0) {  // vbPrevMatched[i1] = F2.mvKeysUn[i2].pt, :571-574
      *reinterpret_cast<float2*>(prev + (base + i) * 2) = make_float2(K2[m].x, K2[m].y);
      ++n;
    }
  }
  n = wave_sum(n);
  if (lane == 0) nmatches[p] = n;
}

extern "C" size_t orb_k_init_params_size(void) { return sizeof(InitParams); }
extern "C" size_t orb_k_init_list_len(void) { return INIT_LIST; }
extern "C" size_t orb_k_init_topk(void) { return INIT_TOPK; }
extern "C" size_t orb_k_init_key_size(void) { return sizeof(InitKey); }

// LDS bytes of k_init_resolve for a problem stride (both frames <= kpStride).
extern "C" size_t orb_k_init_lds(int kpStride) {
  const size_t pad = ((size_t)kpStride + 3) & ~(size_t)3;
  return (3 * pad + pad) * 4;
}

// scratch: qList/qOrder/ncand [P][kpStride] int, nQ/nStage [P] int, stage [P][kpStride]
// InitKey, topk [P][kpStride][INIT_TOPK], list [P][kpStride][INIT_LIST] u32.
extern "C" hipError_t orb_k_search_init(const orb_keypoint_t* keys1, const uint8_t* desc1,
                                        const int32_t* n1, const orb_keypoint_t* keys2,
                                        const uint8_t* desc2, const int32_t* n2, int kpStride,
                                        float* prev, const int32_t* cellStart,
                                        const int32_t* cellIdx, const void* params,
                                        int32_t* qList, int32_t* qOrder, int32_t* nQ,
                                        void* stage,
                                        int32_t* nStage, uint32_t* topk, uint32_t* list,
                                        int32_t* ncand, int32_t* m12, int32_t* nmatches,
                                        int nproblems, hipStream_t s) {
  if (nproblems <= 0) return hipSuccess;
  const InitParams P = *(const InitParams*)params;
  InitKey* st = static_cast<InitKey*>(stage);
  hipLaunchKernelGGL(k_init_prep, dim3(nproblems), dim3(INIT_WG), 0, s, keys1, n1, keys2,
                     kpStride, prev, cellStart, cellIdx, P, qList, qOrder, nQ, st, nStage);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_init_candidates, dim3((kpStride + INIT_WG - 1) / INIT_WG, nproblems),
                     dim3(INIT_WG), 0, s, desc1, desc2, keys2, kpStride, prev, cellStart, cellIdx,
                     P, qList, qOrder, nQ, st, nStage, topk, list, ncand);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds = orb_k_init_lds(kpStride);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536) {
    e = hipFuncSetAttribute((const void*)k_init_resolve,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_init_resolve, dim3(nproblems), dim3(64), lds, s, keys1, desc1, n1, keys2,
                     desc2, n2, kpStride, prev, cellStart, cellIdx, P, qList, nQ, topk, list,
                     ncand, m12, nmatches);
  return hipGetLastError();
}

// ======================================= MapPoint::ComputeDistinctiveDescriptors
// src/MapPoint.cc:250-326.  One wave per MapPoint: lane j holds observation
// descriptor j; for each row i (broadcast by readlane) the wave computes
// D[i][j] and finds the row median vDists[(N-1)/2] as the smallest v with
// #{j : D[i][j] <= v} > (N-1)/2 -- a 9-step bisection over [0, 256] on ballot
// counts, no sort.  The first row with the smallest median wins (strict <).
// Lists longer than 64 recompute each 64-column chunk per bisection step.
__device__ __forceinline__ ulonglong4 readlane_desc(const ulonglong4& v, int lane) {
  ulonglong4 r;
  const unsigned long long* a = &v.x;
  unsigned long long* o = &r.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)a[k], lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(a[k] >> 32), lane);
    o[k] = ((unsigned long long)hi << 32) | lo;
  }
  return r;
}

__global__ __launch_bounds__(256) void k_distinctive(const int32_t* __restrict__ offs,
                                                     const uint8_t* __restrict__ desc, int nmp,
                                                     int32_t* __restrict__ best,
                                                     uint8_t* __restrict__ out) {
  const int w = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  const int lane = threadIdx.x & 63;
  if (w >= nmp) return;
  const int b = offs[w], n = offs[w + 1] - b;
  if (n <= 0) {
    if (lane == 0) best[w] = -1;
    return;
  }
  const int k = (n - 1) >> 1;  // (size_t)(0.5 * (N - 1))
  const uint8_t* D = desc + (size_t)b * 32;
  int bestMed = INT_MAX, bestIdx = 0;
  if (n <= 64) {
    const ulonglong4 dj = load_desc(D + (size_t)min(lane, n - 1) * 32);
    for (int i = 0; i < n; ++i) {
      const int d = lane < n ? hamming256(readlane_desc(dj, i), dj) : 1024;
      int lo = 0, hi = 256;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (__popcll(__ballot(d <= mid)) > k) hi = mid;
        else lo = mid + 1;
      }
      if (lo < bestMed) { bestMed = lo; bestIdx = i; }
    }
  } else {
    for (int i = 0; i < n; ++i) {
      const ulonglong4 di = load_desc(D + (size_t)i * 32);
      int lo = 0, hi = 256;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        int cnt = 0;
        for (int c0 = 0; c0 < n; c0 += 64) {
          const int j = c0 + lane;
          const int d = j < n ? hamming256(di, load_desc(D + (size_t)j * 32)) : 1024;
          cnt += __popcll(__ballot(d <= mid));
        }
        if (cnt > k) hi = mid;
        else lo = mid + 1;
      }
      if (lo < bestMed) { bestMed = lo; bestIdx = i; }
    }
  }
  if (lane == 0) best[w] = bestIdx;
  if (out && lane < 8)
    reinterpret_cast<uint32_t*>(out + (size_t)w * 32)[lane] =
        reinterpret_cast<const uint32_t*>(D + (size_t)bestIdx * 32)[lane];
}

extern "C" hipError_t orb_k_distinctive(const int32_t* offs, const uint8_t* desc, int nmp,
                                        int32_t* best, uint8_t* out, hipStream_t s) {
  if (nmp <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_distinctive, dim3((nmp + 3) / 4), dim3(256), 0, s, offs, desc, nmp, best,
                     out);
  return hipGetLastError();
}
