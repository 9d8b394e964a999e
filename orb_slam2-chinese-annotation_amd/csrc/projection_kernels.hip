// projection_kernels.hip -- gfx950 kernels of the projection-window ORBmatcher
// variants widened from SURVEY §8(f):
//   SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)   relocalisation
//   SearchByProjection(KeyFrame*, Scw, points, matched, th)  loop closing
//   Fuse(KeyFrame*, points, th), Fuse(KeyFrame*, Scw, points, th, replace)
//   SearchBySim3(KF1, KF2, matches12, s12, R12, t12, th)
// and SearchForTriangulation (BoW nodes + epipolar test).
//
// Every variant projects a map point into a (key)frame, opens the
// GetFeaturesInArea window at the predicted scale and keeps the first
// minimum-distance keypoint.  k_pp_match does that per point (thread per
// point, no LDS).  The variants without keypoint claims (Fuse x2, each
// direction of SearchBySim3) are finished there; the two that lock
// keypoints first-come (relocalisation, Sim3 projection) keep the first
// TOPK candidates and are replayed in order by k_pp_resolve, one wave,
// speculatively 64 points at a time.
#include <algorithm>
#include <climits>

#include "matcher_common.h"

enum PPMode { PP_RELOC = 0, PP_SIM3_SBP = 1, PP_FUSE = 2, PP_FUSE_SIM3 = 3, PP_SIM3_DIR = 4 };

struct PPParams {
  float R[9], t[3], Ow[3];  // world -> camera of the searched frame (first stage)
  float R2[9], t2[3];       // SearchBySim3: camera A -> camera B (sR, t)
  float fx, fy, cx, cy, bf;
  float minX, maxX, minY, maxY, invW, invH;
  float th, logScale;
  int nLevels, thr, checkOri;
  float scale[ORB_MAX_LEVELS], invSigma2[ORB_MAX_LEVELS];
};

// projected point: position, predicted window and levels; valid = 0 when the
// reference skips the point before its window scan
struct PPRec {
  float u, v, ur, radius;
  int minL, maxL, valid, pad;
};

__device__ __forceinline__ void pp_xform(const float* R, const float* t, const float* P,
                                         float* o) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
    o[r] = ((R[3 * r] * P[0] + R[3 * r + 1] * P[1]) + R[3 * r + 2] * P[2]) + t[r];
}

__device__ __forceinline__ float pp_norm(const float* a) {
  const double ss = (((double)a[0] * a[0]) + (double)a[1] * a[1]) + (double)a[2] * a[2];
  return (float)__dsqrt_rn(ss);
}

__device__ __forceinline__ double pp_dot(const float* a, const float* b) {
  return (((double)a[0] * b[0]) + (double)a[1] * b[1]) + (double)a[2] * b[2];
}

// MapPoint::PredictScale (src/MapPoint.cc:417-450), logf pinned
__device__ __forceinline__ int pp_level(float maxDistance, float dist, const PPParams& P) {
  const float ratio = __fdiv_rn(maxDistance, dist);
  const float q = ceilf(__fdiv_rn((float)pinned_log((double)ratio), P.logScale));
  if (q < 0.f) return 0;
  if (q >= (float)P.nLevels) return P.nLevels - 1;
  return (int)q;
}

__device__ __forceinline__ bool pp_in_kf(const PPParams& P, float x, float y) {
  return x >= P.minX && x < P.maxX && y >= P.minY && y < P.maxY;  // KeyFrame::IsInImage
}

// The reference's per-point projection and gates for each mode.
template <int MODE>
__device__ __forceinline__ PPRec pp_project(const orb_map_point_t& mp, const PPParams& P) {
  PPRec r;
  r.u = r.v = r.ur = r.radius = 0.f;
  r.minL = r.maxL = 0;
  r.valid = 0;
  r.pad = 0;
  float Pc[3];
  pp_xform(P.R, P.t, mp.pos, Pc);
  if (MODE == PP_SIM3_DIR) {  // p3Dc2 = sR21 * (R1w P + t1w) + t21 (:1266-1268)
    float Pb[3];
    pp_xform(P.R2, P.t2, Pc, Pb);
    Pc[0] = Pb[0]; Pc[1] = Pb[1]; Pc[2] = Pb[2];
  }
  float u, v, invz;
  if (MODE == PP_RELOC) {  // no depth test (:1660-1664)
    invz = (float)(1.0 / (double)Pc[2]);
    u = P.fx * Pc[0] * invz + P.cx;
    v = P.fy * Pc[1] * invz + P.cy;
    if (u < P.minX || u > P.maxX || v < P.minY || v > P.maxY) return r;
  } else {
    if (Pc[2] < 0.0f) return r;
    if (MODE == PP_SIM3_SBP || MODE == PP_FUSE) invz = __fdiv_rn(1.0f, Pc[2]);
    else invz = (float)(1.0 / (double)Pc[2]);
    const float x = Pc[0] * invz, y = Pc[1] * invz;
    u = P.fx * x + P.cx;
    v = P.fy * y + P.cy;
    if (!pp_in_kf(P, u, v)) return r;
  }
  const float maxD = 1.2f * mp.max_distance, minD = 0.8f * mp.min_distance;
  float dist;
  if (MODE == PP_SIM3_DIR) {
    dist = pp_norm(Pc);  // cv::norm(p3Dc2) (:1288)
  } else {
    const float PO[3] = {mp.pos[0] - P.Ow[0], mp.pos[1] - P.Ow[1], mp.pos[2] - P.Ow[2]};
    dist = pp_norm(PO);
    if (dist < minD || dist > maxD) return r;
    if (MODE != PP_RELOC && pp_dot(PO, mp.normal) < 0.5 * (double)dist) return r;
  }
  if (MODE == PP_SIM3_DIR && (dist < minD || dist > maxD)) return r;
  const int lvl = pp_level(mp.max_distance, dist, P);
  r.u = u;
  r.v = v;
  r.ur = u - P.bf * invz;
  r.radius = P.th * P.scale[lvl];
  r.minL = lvl - 1;
  r.maxL = MODE == PP_RELOC ? lvl + 1 : lvl;  // GetFeaturesInArea levels / loop filter
  r.valid = 1;
  return r;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_pp_match(
    const orb_map_point_t* __restrict__ mps, const uint8_t* __restrict__ mpValid,
    const uint8_t* __restrict__ mpSkip, const uint8_t* __restrict__ mpDesc, int n,
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc,
    const float* __restrict__ uright, const int32_t* __restrict__ cellStart,
    const int32_t* __restrict__ cellIdx, PPParams P, PPRec* __restrict__ recs,
    int32_t* __restrict__ best, uint32_t* __restrict__ topk, int32_t* __restrict__ ncand) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const orb_map_point_t mp = mps[i];
  PPRec r;
  r.valid = 0;
  // `seen` = the per-variant "already found" set; SearchBySim3 uses mpSkip
  // (vbAlreadyMatched) and mpValid (pMP != NULL) instead
  if (!mp.bad && (MODE == PP_SIM3_DIR || !mp.seen) && (!mpValid || mpValid[i]) &&
      (!mpSkip || !mpSkip[i]))
    r = pp_project<MODE>(mp, P);
  const bool claims = MODE == PP_RELOC || MODE == PP_SIM3_SBP;
  if (claims) recs[i] = r;
  if (!r.valid) {
    if (claims) ncand[i] = 0;
    else best[i] = -1;
    return;
  }
  ProjParams G;
  G.minX = P.minX; G.minY = P.minY; G.invW = P.invW; G.invH = P.invH;
  const ulonglong4 q = load_desc(mpDesc + (size_t)i * 32);
  if (claims) {
    Top4 top;
    int count = 0;
    for_features_in_area(keys, cellStart, cellIdx, G, r.u, r.v, r.radius, r.minL, r.maxL,
                         [&](int idx, const orb_keypoint_t& kp) {
                           const int d = hamming256(q, load_desc(desc + (size_t)idx * 32));
                           ++count;
                           top.insert(pack_cand(idx, d, kp.octave), d);
                         });
    top.store(topk + (size_t)i * TOPK);
    ncand[i] = count;
  } else {
    int bd = 256, bi = -1;
    for_features_in_area(keys, cellStart, cellIdx, G, r.u, r.v, r.radius, r.minL, r.maxL,
                         [&](int idx, const orb_keypoint_t& kp) {
                           if (MODE == PP_FUSE) {  // reprojection gate (:997-1025)
                             const float ex = r.u - kp.x, ey = r.v - kp.y;
                             const float isg = P.invSigma2[kp.octave];
                             if (uright && uright[idx] >= 0) {
                               const float er = r.ur - uright[idx];
                               const float e2 = ex * ex + ey * ey + er * er;
                               if ((double)(e2 * isg) > 7.8) return;
                             } else {
                               const float e2 = ex * ex + ey * ey;
                               if ((double)(e2 * isg) > 5.99) return;
                             }
                           }
                           const int d = hamming256(q, load_desc(desc + (size_t)idx * 32));
                           if (d < bd) { bd = d; bi = idx; }
                         });
    best[i] = bd <= P.thr ? bi : -1;
  }
}

__device__ __forceinline__ void pp_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bool pp_locked(const uint32_t* bm, int idx) {
  return (bm[idx >> 5] >> (idx & 31)) & 1u;
}

// First-come replay of the claiming variants.  kpMatch holds the entry
// state (-1 free, >= 0 point index already there, which locks the keypoint)
// and receives this call's assignments; the relocalisation rotation filter
// marks the keypoints it resets with -2.
__global__ __launch_bounds__(64) void k_pp_resolve(
    const orb_keypoint_t* __restrict__ keys, const uint8_t* __restrict__ desc, int nkeys,
    const uint8_t* __restrict__ kpLocked, const uint8_t* __restrict__ mpDesc,
    const float* __restrict__ mpAngle, int n, const int32_t* __restrict__ cellStart,
    const int32_t* __restrict__ cellIdx, PPParams P, const PPRec* __restrict__ recs,
    const uint32_t* __restrict__ topk, const int32_t* __restrict__ ncand,
    int32_t* __restrict__ kpMatch, int32_t* __restrict__ nmatches) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ int hist[32];
  const int lane = threadIdx.x;
  const int words = (nkeys + 31) >> 5;
  const int wpad = (words + 3) & ~3;
  uint32_t* bm = dyn;                  // keypoint locks
  int* claimBy = (int*)(dyn + wpad);   // earliest claiming lane of the batch
  int* accIdx = claimBy + ((nkeys + 3) & ~3);  // keypoint accepted by each point
  for (int w = lane; w < words; w += 64) {
    uint32_t m = 0u;
    for (int b = 0; b < 32; ++b) {
      const int k = w * 32 + b;
      if (k < nkeys && ((kpLocked && kpLocked[k]) || kpMatch[k] >= 0)) m |= 1u << b;
    }
    bm[w] = m;
  }
  for (int k = lane; k < nkeys; k += 64) claimBy[k] = 64;
  if (lane < 32) hist[lane] = 0;
  __syncthreads();
  int start = 0;
  while (start < n) {
    const int m = start + lane;
    const bool active = m < n;
    const int nc = active ? ncand[m] : 0;
    uint32_t e0 = 0xFFFFFFFFu, e1 = 0xFFFFFFFFu, e2 = 0xFFFFFFFFu, e3 = 0xFFFFFFFFu;
    if (nc > 0) {
      const uint4 v = *reinterpret_cast<const uint4*>(topk + (size_t)m * TOPK);
      e0 = v.x; e1 = v.y; e2 = v.z; e3 = v.w;
    }
    const uint32_t e[TOPK] = {e0, e1, e2, e3};
    int bi = -1, bd = 256, consumed = 0;
#pragma unroll
    for (int j = 0; j < TOPK; ++j) {
      if (bi < 0 && j < nc) {
        ++consumed;
        if (!pp_locked(bm, cand_idx(e[j]))) { bi = cand_idx(e[j]); bd = cand_dist(e[j]); }
      }
    }
    const bool slow = nc > TOPK && bi < 0;
    const bool accept = !slow && bi >= 0 && bd <= P.thr;
    if (accept) atomicMin(&claimBy[bi], lane);
    pp_wave_sync();
    bool conflict = false;
#pragma unroll
    for (int j = 0; j < TOPK; ++j)
      if (j < consumed) conflict |= claimBy[cand_idx(e[j])] < lane;
    pp_wave_sync();
    if (accept) claimBy[bi] = 64;
    const unsigned long long bad = __ballot(active && (conflict || slow));
    const int commit = bad ? (int)__builtin_ctzll(bad) : 64;
    if (active && lane < commit) {
      accIdx[m] = accept ? bi : -1;
      if (accept) atomicOr(&bm[bi >> 5], 1u << (bi & 31));
    }
    int advance = commit;
    if (commit < 64 && ((__ballot(slow) >> commit) & 1ull)) {
      pp_wave_sync();
      if (lane == commit) {  // exact rescan of the window against the current locks
        const PPRec r = recs[m];
        ProjParams G;
        G.minX = P.minX; G.minY = P.minY; G.invW = P.invW; G.invH = P.invH;
        const ulonglong4 q = load_desc(mpDesc + (size_t)m * 32);
        int sd = 256, si = -1;
        for_features_in_area(keys, cellStart, cellIdx, G, r.u, r.v, r.radius, r.minL, r.maxL,
                             [&](int idx, const orb_keypoint_t&) {
                               if (pp_locked(bm, idx)) return;
                               const int d = hamming256(q, load_desc(desc + (size_t)idx * 32));
                               if (d < sd) { sd = d; si = idx; }
                             });
        accIdx[m] = -1;
        if (si >= 0 && sd <= P.thr) {
          accIdx[m] = si;
          bm[si >> 5] |= 1u << (si & 31);
        }
      }
      advance = commit + 1;
    }
    pp_wave_sync();
    start += advance;
  }
  // assignments, then the rotation histogram filter (relocalisation only)
  int accepted = 0;
  for (int m = lane; m < n; m += 64) {
    const int k = accIdx[m];
    if (k < 0) continue;
    kpMatch[k] = m;
    ++accepted;
    if (P.checkOri) atomicAdd(&hist[rot_bin(mpAngle[m] - keys[k].angle)], 1);
  }
  pp_wave_sync();
  int ind1 = -1, ind2 = -1, ind3 = -1;
  if (P.checkOri) three_maxima(hist, ind1, ind2, ind3);
  int removed = 0;
  if (P.checkOri)
    for (int m = lane; m < n; m += 64) {
      const int k = accIdx[m];
      if (k < 0) continue;
      const int b = rot_bin(mpAngle[m] - keys[k].angle);
      if (b != ind1 && b != ind2 && b != ind3) {
        kpMatch[k] = -2;
        ++removed;
      }
    }
  const int a = wave_sum(accepted), rm = wave_sum(removed);
  if (lane == 0) *nmatches = a - rm;
}

// SearchBySim3 mutual check (:1406-1423): match12[i1] = idx2 iff the two
// directions agree.
__global__ __launch_bounds__(256) void k_sim3_mutual(const int32_t* __restrict__ m1, int n1,
                                                     const int32_t* __restrict__ m2,
                                                     int32_t* __restrict__ match12,
                                                     int32_t* __restrict__ nfound) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool ok = false;
  if (i < n1) {
    const int j = m1[i];
    ok = j >= 0 && m2[j] == i;
    match12[i] = ok ? j : -1;
  }
  const int c = __popcll(__ballot(ok));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(nfound, c);
}

// ================================================= SearchForTriangulation
// src/ORBmatcher.cc:718-901.  vbMatched2 is never set in this fork (nor
// upstream), so every KF1 feature is independent: one wave per KF1 node,
// lanes over the KF2 features of the same node; the reference keeps the LAST
// passing candidate of minimum distance (dist <= bestDist), i.e. the minimum
// of (dist, -position).  k_tri_finish applies the rotation filter.
struct TriParams {
  float F[9];
  float ex, ey;
  int onlyStereo, checkOri;
  float scale[ORB_MAX_LEVELS], sigma2[ORB_MAX_LEVELS];
};

__global__ __launch_bounds__(256) void k_tri_match(
    const orb_keypoint_t* __restrict__ k1, const uint8_t* __restrict__ d1,
    const float* __restrict__ ur1, const uint8_t* __restrict__ hasMp1, int nodes1,
    const uint32_t* __restrict__ ids1, const int32_t* __restrict__ offs1,
    const uint32_t* __restrict__ feats1, const orb_keypoint_t* __restrict__ k2,
    const uint8_t* __restrict__ d2, const float* __restrict__ ur2,
    const uint8_t* __restrict__ hasMp2, int nodes2, const uint32_t* __restrict__ ids2,
    const int32_t* __restrict__ offs2, const uint32_t* __restrict__ feats2, TriParams T,
    int32_t* __restrict__ match12, int32_t* __restrict__ acc) {
  const int lane = threadIdx.x & 63;
  const int a = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (a >= nodes1) return;
  const uint32_t id = ids1[a];
  int lo = 0, hi = nodes2;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (ids2[mid] < id) lo = mid + 1; else hi = mid;
  }
  const bool found = lo < nodes2 && ids2[lo] == id;
  for (int p = offs1[a]; p < offs1[a + 1]; ++p) {
    const int idx1 = (int)feats1[p];
    acc[p] = -1;
    if (!found || hasMp1[idx1]) continue;
    const bool st1 = ur1 && ur1[idx1] >= 0;
    if (T.onlyStereo && !st1) continue;
    const orb_keypoint_t kp1 = k1[idx1];
    const float la = kp1.x * T.F[0] + kp1.y * T.F[3] + T.F[6];  // epipolar line (:147-149)
    const float lb = kp1.x * T.F[1] + kp1.y * T.F[4] + T.F[7];
    const float lc = kp1.x * T.F[2] + kp1.y * T.F[5] + T.F[8];
    const float den = la * la + lb * lb;
    const ulonglong4 q = load_desc(d1 + (size_t)idx1 * 32);
    const int fb = offs2[lo], fe = offs2[lo + 1];
    uint32_t key = 0xFFFFFFFFu;  // (dist << 20) | (0xFFFFF - position): min = last minimum
    for (int c = fb + lane; c < fe; c += 64) {
      const int idx2 = (int)feats2[c];
      if (hasMp2[idx2]) continue;
      const bool st2 = ur2 && ur2[idx2] >= 0;
      if (T.onlyStereo && !st2) continue;
      const int dist = hamming256(q, load_desc(d2 + (size_t)idx2 * 32));
      if (dist > 50) continue;
      const orb_keypoint_t kp2 = k2[idx2];
      if (!st1 && !st2) {
        const float dx = T.ex - kp2.x, dy = T.ey - kp2.y;
        if (dx * dx + dy * dy < 100 * T.scale[kp2.octave]) continue;
      }
      if (den == 0) continue;
      const float num = la * kp2.x + lb * kp2.y + lc;
      const float dsqr = __fdiv_rn(num * num, den);
      if (!((double)dsqr < 3.84 * (double)T.sigma2[kp2.octave])) continue;
      const uint32_t k = ((uint32_t)dist << 20) | (uint32_t)(0xFFFFF - (c - fb));
      key = min(key, k);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, o));
    if (lane == 0 && key != 0xFFFFFFFFu) {
      const int idx2 = (int)feats2[fb + (0xFFFFF - (int)(key & 0xFFFFFu))];
      match12[idx1] = idx2;
      acc[p] = idx2;
    }
  }
}

__global__ __launch_bounds__(256) void k_tri_finish(int nFeats1, const uint32_t* __restrict__ feats1,
                                                    const orb_keypoint_t* __restrict__ k1,
                                                    const orb_keypoint_t* __restrict__ k2,
                                                    int checkOri, const int32_t* __restrict__ acc,
                                                    int32_t* __restrict__ match12,
                                                    int32_t* __restrict__ nmatches) {
  __shared__ int hist[32];
  __shared__ int tmp[17];
  const int t = threadIdx.x;
  if (t < 32) hist[t] = 0;
  __syncthreads();
  int na = 0;
  for (int p = t; p < nFeats1; p += 256) {
    const int j = acc[p];
    if (j < 0) continue;
    ++na;
    if (checkOri) atomicAdd(&hist[rot_bin(k1[feats1[p]].angle - k2[j].angle)], 1);
  }
  __syncthreads();
  int ind1 = -1, ind2 = -1, ind3 = -1;
  if (checkOri) three_maxima(hist, ind1, ind2, ind3);
  int removed = 0;
  if (checkOri)
    for (int p = t; p < nFeats1; p += 256) {
      const int j = acc[p];
      if (j < 0) continue;
      const int b = rot_bin(k1[feats1[p]].angle - k2[j].angle);
      if (b != ind1 && b != ind2 && b != ind3) {
        match12[feats1[p]] = -1;
        ++removed;
      }
    }
  int totA, totR;
  block_excl_scan(na, tmp, &totA);
  block_excl_scan(removed, tmp, &totR);
  if (t == 0) *nmatches = totA - totR;
}

// ----------------------------------------------------------------- launchers
extern "C" size_t orb_k_pp_params_size(void) { return sizeof(PPParams); }
extern "C" size_t orb_k_pp_rec_size(void) { return sizeof(PPRec); }
extern "C" size_t orb_k_tri_params_size(void) { return sizeof(TriParams); }

extern "C" hipError_t orb_k_pp_match(int mode, const orb_map_point_t* mps, const uint8_t* mpValid,
                                     const uint8_t* mpSkip, const uint8_t* mpDesc, int n,
                                     const orb_keypoint_t* keys, const uint8_t* desc,
                                     const float* uright, const int32_t* cellStart,
                                     const int32_t* cellIdx, const void* params, void* recs,
                                     int32_t* best, uint32_t* topk, int32_t* ncand,
                                     hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const PPParams P = *(const PPParams*)params;
  PPRec* R = static_cast<PPRec*>(recs);
  const dim3 g((n + 255) / 256), b(256);
  switch (mode) {
    case PP_RELOC:
      hipLaunchKernelGGL(k_pp_match<PP_RELOC>, g, b, 0, s, mps, mpValid, mpSkip, mpDesc, n, keys,
                         desc, uright, cellStart, cellIdx, P, R, best, topk, ncand);
      break;
    case PP_SIM3_SBP:
      hipLaunchKernelGGL(k_pp_match<PP_SIM3_SBP>, g, b, 0, s, mps, mpValid, mpSkip, mpDesc, n,
                         keys, desc, uright, cellStart, cellIdx, P, R, best, topk, ncand);
      break;
    case PP_FUSE:
      hipLaunchKernelGGL(k_pp_match<PP_FUSE>, g, b, 0, s, mps, mpValid, mpSkip, mpDesc, n, keys,
                         desc, uright, cellStart, cellIdx, P, R, best, topk, ncand);
      break;
    case PP_FUSE_SIM3:
      hipLaunchKernelGGL(k_pp_match<PP_FUSE_SIM3>, g, b, 0, s, mps, mpValid, mpSkip, mpDesc, n,
                         keys, desc, uright, cellStart, cellIdx, P, R, best, topk, ncand);
      break;
    case PP_SIM3_DIR:
      hipLaunchKernelGGL(k_pp_match<PP_SIM3_DIR>, g, b, 0, s, mps, mpValid, mpSkip, mpDesc, n,
                         keys, desc, uright, cellStart, cellIdx, P, R, best, topk, ncand);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" size_t orb_k_pp_resolve_lds(int nkeys, int n) {
  const size_t words = (size_t)((nkeys + 31) / 32);
  return (((words + 3) & ~(size_t)3) + (((size_t)nkeys + 3) & ~(size_t)3) +
          (size_t)std::max(n, 1)) * 4;
}

extern "C" hipError_t orb_k_pp_resolve(const orb_keypoint_t* keys, const uint8_t* desc,
                                       int nkeys, const uint8_t* kpLocked, const uint8_t* mpDesc,
                                       const float* mpAngle, int n, const int32_t* cellStart,
                                       const int32_t* cellIdx, const void* params,
                                       const void* recs, const uint32_t* topk,
                                       const int32_t* ncand, int32_t* kpMatch,
                                       int32_t* nmatches, hipStream_t s) {
  const PPParams P = *(const PPParams*)params;
  const size_t lds = orb_k_pp_resolve_lds(nkeys, n);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_pp_resolve,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_pp_resolve, dim3(1), dim3(64), lds, s, keys, desc, nkeys, kpLocked, mpDesc,
                     mpAngle, n, cellStart, cellIdx, P, static_cast<const PPRec*>(recs), topk,
                     ncand, kpMatch, nmatches);
  return hipGetLastError();
}

extern "C" hipError_t orb_k_sim3_mutual(const int32_t* m1, int n1, const int32_t* m2,
                                        int32_t* match12, int32_t* nfound, hipStream_t s) {
  hipError_t e = hipMemsetAsync(nfound, 0, 4, s);
  if (e != hipSuccess || n1 <= 0) return e;
  hipLaunchKernelGGL(k_sim3_mutual, dim3((n1 + 255) / 256), dim3(256), 0, s, m1, n1, m2, match12,
                     nfound);
  return hipGetLastError();
}

extern "C" hipError_t orb_k_triangulation(
    const orb_keypoint_t* k1, const uint8_t* d1, const float* ur1, const uint8_t* hasMp1,
    int nodes1, const uint32_t* ids1, const int32_t* offs1, const uint32_t* feats1, int nFeats1,
    const orb_keypoint_t* k2, const uint8_t* d2, const float* ur2, const uint8_t* hasMp2,
    int nodes2, const uint32_t* ids2, const int32_t* offs2, const uint32_t* feats2,
    const void* params, int32_t* match12, int32_t* acc, int32_t* nmatches, hipStream_t s) {
  const TriParams T = *(const TriParams*)params;
  if (nodes1 > 0) {
    hipLaunchKernelGGL(k_tri_match, dim3((nodes1 + 3) / 4), dim3(256), 0, s, k1, d1, ur1, hasMp1,
                       nodes1, ids1, offs1, feats1, k2, d2, ur2, hasMp2, nodes2, ids2, offs2,
                       feats2, T, match12, acc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_tri_finish, dim3(1), dim3(256), 0, s, nFeats1, feats1, k1, k2,
                     T.checkOri, acc, match12, nmatches);
  return hipGetLastError();
}
