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
// k_init_candidates (thread per i1): the window scan against the initial
// state -- every candidate in scan order (up to INIT_LIST, packed idx|dist)
// and the first INIT_TOPK in (distance, scan order).
// k_init_resolve (one wave per problem): speculative in-order resolve of 64
// consecutive i1 at a time.  vMatchedDistance only decreases, so a query's
// surviving candidates only shrink; its (best, second) stays exact unless an
// earlier query of the same batch accepts one of those two keypoints.  Lanes
// up to the first such conflict commit together (no two committed lanes then
// accept the same keypoint); a query whose top-K list ran out of survivors
// is resolved exactly by the whole wave from its full candidate list.
#define INIT_TOPK 8
#define INIT_LIST 256

struct InitParams {
  float minX, minY, invW, invH;
  float r, nnratio;
  int checkOri;
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

__global__ __launch_bounds__(256) void k_init_candidates(
    const orb_keypoint_t* __restrict__ keys1, const uint8_t* __restrict__ desc1,
    const int32_t* __restrict__ n1, const orb_keypoint_t* __restrict__ keys2,
    const uint8_t* __restrict__ desc2, int kpStride, const float* __restrict__ prev,
    const int32_t* __restrict__ cellStart, const int32_t* __restrict__ cellIdx, InitParams P,
    uint32_t* __restrict__ topk, uint32_t* __restrict__ list, int32_t* __restrict__ ncand) {
  const int p = blockIdx.y;
  const int i1 = blockIdx.x * 256 + threadIdx.x;
  if (i1 >= n1[p]) return;
  const size_t q = (size_t)p * kpStride + i1;
  const orb_keypoint_t k1 = keys1[q];
  if (k1.octave > 0) {  // :449-451
    ncand[q] = 0;
    return;
  }
  ProjParams G;
  G.minX = P.minX; G.minY = P.minY; G.invW = P.invW; G.invH = P.invH;
  const ulonglong4 d1 = load_desc(desc1 + q * 32);
  const float2 c = *reinterpret_cast<const float2*>(prev + q * 2);
  TopKReg<INIT_TOPK> top;
  uint32_t* L = list + q * INIT_LIST;
  int count = 0;
  const orb_keypoint_t* K2 = keys2 + (size_t)p * kpStride;
  const uint8_t* D2 = desc2 + (size_t)p * kpStride * 32;
  for_features_in_area(K2, cellStart + (size_t)p * (GRID_CELLS + 1),
                       cellIdx + (size_t)p * kpStride, G, c.x, c.y, P.r, 0, 0,
                       [&](int idx, const orb_keypoint_t&) {
                         const int dist = hamming256(d1, load_desc(D2 + (size_t)idx * 32));
                         const uint32_t e = pack_cand(idx, dist, 0);
                         if (count < INIT_LIST) L[count] = e;
                         ++count;
                         top.insert(e, dist);
                       });
  uint4* T = reinterpret_cast<uint4*>(topk + q * INIT_TOPK);
#pragma unroll
  for (int j = 0; j < INIT_TOPK / 4; ++j)
    T[j] = make_uint4(top.t[4 * j], top.t[4 * j + 1], top.t[4 * j + 2], top.t[4 * j + 3]);
  ncand[q] = count;
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
    const int32_t* __restrict__ cellIdx, InitParams P, const uint32_t* __restrict__ topk,
    const uint32_t* __restrict__ list, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ m12, int32_t* __restrict__ nmatches) {
  // LDS: vMatchedDistance, vnMatches21 (owner), earliest claiming lane of the
  // batch per F2 keypoint, and the F2 keypoint each i1 accepted (even if it
  // was stolen later: its histogram entry stays, :524-527)
  extern __shared__ __attribute__((aligned(16))) int sm[];
  __shared__ int hist[32];
  const int p = blockIdx.x, lane = threadIdx.x;
  const int N1 = n1s[p], N2 = n2s[p];
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
  while (start < N1) {
    const int i1 = start + lane;
    const bool active = i1 < N1;
    const int nc = active ? ncand[base + i1] : 0;
    int b1 = INT_MAX, b2 = INT_MAX, bi = -1, si = -1, found = 0;
    if (nc > 0) {
      const uint4* T = reinterpret_cast<const uint4*>(topk + (base + i1) * INIT_TOPK);
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
    int commit = bad ? (int)__builtin_ctzll(bad) : 64;
    if (commit == 0) {
      // lane 0 (i1 = start) needs its full candidate list: exact, wave-wide
      const int q1 = start;
      const int ncq = __builtin_amdgcn_readfirstlane(ncand[base + q1]);
      int eb1 = INT_MAX, eb2 = INT_MAX, ebi = -1;
      if (ncq <= INIT_LIST) {
        const uint32_t* Lq = list + (base + q1) * INIT_LIST;
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
      commit = 1;
    } else if (active && lane < commit && accept) {
      owner[bi] = i1;  // a previous owner (earlier batch) loses the keypoint
      vMD[bi] = b1;
      acc[i1] = bi;
    }
    wave_sync_lds();
    start += commit;
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

// LDS bytes of k_init_resolve for a problem stride (both frames <= kpStride).
extern "C" size_t orb_k_init_lds(int kpStride) {
  const size_t pad = ((size_t)kpStride + 3) & ~(size_t)3;
  return (3 * pad + pad) * 4;
}

extern "C" hipError_t orb_k_search_init(const orb_keypoint_t* keys1, const uint8_t* desc1,
                                        const int32_t* n1, const orb_keypoint_t* keys2,
                                        const uint8_t* desc2, const int32_t* n2, int kpStride,
                                        float* prev, const int32_t* cellStart,
                                        const int32_t* cellIdx, const void* params,
                                        uint32_t* topk, uint32_t* list, int32_t* ncand,
                                        int32_t* m12, int32_t* nmatches, int nproblems,
                                        hipStream_t s) {
  if (nproblems <= 0) return hipSuccess;
  const InitParams P = *(const InitParams*)params;
  hipLaunchKernelGGL(k_init_candidates, dim3((kpStride + 255) / 256, nproblems), dim3(256), 0, s,
                     keys1, desc1, n1, keys2, desc2, kpStride, prev, cellStart, cellIdx, P, topk,
                     list, ncand);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds = orb_k_init_lds(kpStride);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536) {
    e = hipFuncSetAttribute((const void*)k_init_resolve,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_init_resolve, dim3(nproblems), dim3(64), lds, s, keys1, desc1, n1, keys2,
                     desc2, n2, kpStride, prev, cellStart, cellIdx, P, topk, list, ncand, m12,
                     nmatches);
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
