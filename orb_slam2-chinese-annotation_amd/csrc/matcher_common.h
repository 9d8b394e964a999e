// matcher_common.h -- device helpers shared by the matcher kernels: the Frame
// grid cell rule, GetFeaturesInArea, packed candidates with the register top-K,
// and ORBmatcher's rotation histogram (bin rule + ComputeThreeMaxima).
#pragma once
#include "orb_device.h"
#include "../../include/orb_abi.h"

#define GRID_CELLS (ORB_GRID_COLS * ORB_GRID_ROWS)
#define TOPK 4

__device__ __forceinline__ int grid_cell(const orb_keypoint_t& k, float minX, float minY,
                                         float invW, float invH) {
  const int px = (int)round_half_away((k.x - minX) * invW);
  const int py = (int)round_half_away((k.y - minY) * invH);
  if (px < 0 || px >= ORB_GRID_COLS || py < 0 || py >= ORB_GRID_ROWS) return -1;
  return px * ORB_GRID_ROWS + py;
}

// Candidate lists of the map points with more than TOPK candidates: the
// resolves' exact re-scan of such a point (its top-K ran dry: too many of its
// candidates taken) reads the list instead of walking the grid -- one thread's
// chain of dependent grid, keypoint and descriptor loads (15-30 us per point,
// the whole workgroup waiting on it: one-frame SearchByProjection 40-150 us
// instead of 21 us on the frames that had one, profiles/r06_dropin.txt).
// k_proj_candidates writes the list of a point with TOPK < count <= OVF_CAP
// (its window candidates that pass the level, lock and stereo tests, in scan
// order, packed as the top-K entries) into one of OVF_SLOTS lists per problem;
// a point past OVF_CAP or beyond the slots keeps the grid re-scan.
#define OVF_CAP 16
#define OVF_SLOTS 512
struct ProjParams {
  float minX, minY, invW, invH;
  float th, nnratio;
  int nLevels;
  float scale[ORB_MAX_LEVELS];
  uint32_t* ovf;     // OVF_SLOTS x OVF_CAP entries per problem, or null (no lists)
  uint32_t* ovfCtr;  // per problem: the call's gen << 20 | slots taken
  uint32_t gen;      // 1..4095, a new value per call (no reset of ovfCtr needed)
};

// A list slot of problem counter `ctr` for the call `gen`: the first
// allocation of a call finds another call's tag and restarts the count.
__device__ __forceinline__ int ovf_alloc(uint32_t* ctr, uint32_t gen) {
  uint32_t v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (true) {
    const uint32_t n = (v >> 20) == gen ? v + 1u : ((gen << 20) | 1u);
    const uint32_t old = atomicCAS(ctr, v, n);
    if (old == v) return (int)(n & 0xFFFFFu) - 1;
    v = old;
  }
}

// Top-K entry: keypoint index (19b) | distance (9b) << 19 | octave (4b) << 28.
__device__ __forceinline__ uint32_t pack_cand(int idx, int dist, int oct) {
  return (uint32_t)idx | ((uint32_t)dist << 19) | ((uint32_t)oct << 28);
}
__device__ __forceinline__ int cand_idx(uint32_t e) { return (int)(e & 0x7FFFFu); }
__device__ __forceinline__ int cand_dist(uint32_t e) { return (int)((e >> 19) & 0x1FFu); }
__device__ __forceinline__ int cand_oct(uint32_t e) { return (int)(e >> 28); }

// First TOPK (= 4) candidates in (dist, scan order), kept in registers: a
// stable sorted insertion (after equal distances) as a branch-free network.
// Empty slots are 0xFFFFFFFF, whose distance field (511) exceeds any real one.
struct Top4 {
  uint32_t t0 = 0xFFFFFFFFu, t1 = 0xFFFFFFFFu, t2 = 0xFFFFFFFFu, t3 = 0xFFFFFFFFu;
  __device__ __forceinline__ void insert(uint32_t e, int d) {
    const bool b0 = cand_dist(t0) > d, b1 = cand_dist(t1) > d, b2 = cand_dist(t2) > d,
               b3 = cand_dist(t3) > d;
    t3 = b2 ? t2 : (b3 ? e : t3);
    t2 = b1 ? t1 : (b2 ? e : t2);
    t1 = b0 ? t0 : (b1 ? e : t1);
    t0 = b0 ? e : t0;
  }
  __device__ __forceinline__ void store(uint32_t* dst) const {
    *reinterpret_cast<uint4*>(dst) = make_uint4(t0, t1, t2, t3);
  }
};

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

// ========================================== rotation consistency (shared)
// src/ORBmatcher.cc:1582-1588: bin = round(rot * (1/30)) with rot in [0,360)
// -> only bins 0..12 are ever used (upstream quirk, kept).
__device__ __forceinline__ int rot_bin(float rot) {
  const float factor = 1.0f / 30;
  if (rot < 0.0f) rot += 360.0f;
  int bin = (int)round_half_away(rot * factor);
  if (bin == 30) bin = 0;
  return bin;
}

// ComputeThreeMaxima (src/ORBmatcher.cc:1765-1809) over 30 bin counts.
__device__ __forceinline__ void three_maxima(const int* h, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  ind1 = ind2 = ind3 = -1;
  for (int i = 0; i < 30; ++i) {
    const int s = h[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s; ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
  else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

