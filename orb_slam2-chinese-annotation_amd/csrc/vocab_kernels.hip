// vocab_kernels.hip -- gfx950 kernels of the DBoW2 vocabulary transform
// (Frame::ComputeBoW src/Frame.cc:439-449, KeyFrame::ComputeBoW
// src/KeyFrame.cc:60-71 -> TemplatedVocabulary::transform,
// Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1128-1283).
//
// Device tree layout (built by runtime.cpp from the loadFromTextFile node
// table): nodes renumbered breadth-first so that every node's children sit at
// consecutive device positions in the reference's child order.  Position p
// holds {first child position, child count}, the 32-byte descriptor, the word
// id / weight the reference reads at a leaf, and the reference node id (for
// the FeatureVector).  A descent step is then one 8-byte load of the current
// node, one contiguous read of its children's descriptors, and a reduction:
// no child-id indirection.
//
// k_voc_descend: a 16-lane group per feature, lane j scores child j (chunks of
// 16 for wider nodes) with 4 x v_bcnt; the group's min over (distance, child
// order) -- the reference's strict '<' keeps the first minimum -- is a 4-step
// xor-shuffle reduction.  Hamming bit-count work: VALU, no MFMA.
// k_voc_vectors: a workgroup per frame builds the BowVector (std::map
// WordId -> value: addWeight sums in feature order, or addIfNotExist keeps
// the first) and the FeatureVector (std::map NodeId -> ascending feature
// indices) by a bitonic sort of (key << 32 | feature) in LDS; the
// normalisation sum runs sequentially in word order so every double rounds
// exactly as BowVector::normalize's loop does.
#include "orb_device.h"

#define VOC_GROUP 16
#define VOC_STOP 0xFFFFFFFFu

struct VocNodeInfo {
  int32_t first;  // device position of the first child
  int32_t count;  // number of children (0 = Node::isLeaf)
};

__global__ __launch_bounds__(256) void k_voc_descend(
    const VocNodeInfo* __restrict__ info, const uint4* __restrict__ ndesc,
    const uint32_t* __restrict__ nword, const double* __restrict__ nweight,
    const uint32_t* __restrict__ norig, int nidLevel, const uint8_t* __restrict__ desc,
    const int32_t* __restrict__ counts, int nSingle, int stride, int nFrames,
    uint32_t* __restrict__ fword, double* __restrict__ fweight, uint32_t* __restrict__ fnode) {
  const int g = threadIdx.x & (VOC_GROUP - 1);
  const long long gid = (long long)blockIdx.x * (256 / VOC_GROUP) + (threadIdx.x / VOC_GROUP);
  const int frame = (int)(gid / stride);
  const int i = (int)(gid - (long long)frame * stride);
  if (frame >= nFrames) return;
  const int n = counts ? counts[frame] : nSingle;
  if (i >= n) return;  // group-uniform
  const size_t slot = (size_t)frame * stride + i;
  const uint4* fp = reinterpret_cast<const uint4*>(desc + slot * 32);
  const uint4 f0 = fp[0], f1 = fp[1];

  int node = 0, level = 0;
  int nidPos = 0;  // nid_level <= 0 -> root (:1246)
  VocNodeInfo cur = info[0];
  do {
    ++level;
    uint32_t best = 0xFFFFFFFFu;
    for (int base = 0; base < cur.count; base += VOC_GROUP) {
      const int c = base + g;
      uint32_t key = 0xFFFFFFFFu;
      if (c < cur.count) {
        const uint4* cp = ndesc + (size_t)(cur.first + c) * 2;
        const uint4 a = cp[0], b = cp[1];
        const int d = __popc(a.x ^ f0.x) + __popc(a.y ^ f0.y) + __popc(a.z ^ f0.z) +
                      __popc(a.w ^ f0.w) + __popc(b.x ^ f1.x) + __popc(b.y ^ f1.y) +
                      __popc(b.z ^ f1.z) + __popc(b.w ^ f1.w);
        key = ((uint32_t)d << 23) | (uint32_t)c;
      }
#pragma unroll
      for (int m = 1; m < VOC_GROUP; m <<= 1) key = min(key, (uint32_t)__shfl_xor((int)key, m, VOC_GROUP));
      best = min(best, key);
    }
    node = cur.first + (int)(best & 0x7FFFFFu);
    if (level == nidLevel) nidPos = node;
    cur = info[node];
  } while (cur.count > 0);
  if (nidLevel > level) nidPos = node;  // leaf above nid_level (reference: uninitialised)
  if (g == 0) {
    const double w = nweight[node];
    fword[slot] = w > 0 ? nword[node] : VOC_STOP;
    fweight[slot] = w;
    fnode[slot] = norig[nidPos];
  }
}

// Bitonic sort of P (power of two) 64-bit keys in LDS, ascending.
__device__ __forceinline__ void lds_bitonic(unsigned long long* keys, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = keys[i], b = keys[ixj];
          const bool asc = (i & k) == 0;
          if ((a > b) == asc) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Exclusive scan of per-thread counts over the workgroup (256 threads).
__device__ __forceinline__ int block_excl_scan(int v, int* red, int& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int inc = wave_incl_scan(v);
  if (lane == 63) red[wv] = inc;
  __syncthreads();
  int off = 0;
  total = 0;
  for (int w = 0; w < 4; ++w) {
    if (w < wv) off += red[w];
    total += red[w];
  }
  __syncthreads();
  return off + inc - v;
}

struct VocVecParams {
  int stride, tf, must, l2;
};

// One workgroup (256 threads) per frame; dynamic LDS = P * 16 bytes.
__global__ __launch_bounds__(256) void k_voc_vectors(
    const uint32_t* __restrict__ fword, const double* __restrict__ fweight,
    const uint32_t* __restrict__ fnode, const int32_t* __restrict__ counts, int nSingle,
    VocVecParams V, int P, uint32_t* __restrict__ bowWords, double* __restrict__ bowValues,
    int32_t* __restrict__ nWords, uint32_t* __restrict__ fvNodes, int32_t* __restrict__ fvOffs,
    uint32_t* __restrict__ fvFeats, int32_t* __restrict__ nFv) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long vsm[];
  unsigned long long* keys = vsm;
  double* vals = reinterpret_cast<double*>(vsm + P);
  __shared__ int red[4];
  __shared__ double normShared;
  const int f = blockIdx.x;
  const int n = counts ? counts[f] : nSingle;
  const size_t base = (size_t)f * V.stride;
  const uint32_t* W = fword + base;
  const double* WT = fweight + base;
  const uint32_t* ND = fnode + base;
  const int T = blockDim.x;
  const int per = P / T > 0 ? P / T : 1;  // contiguous elements per thread in the scans

  // ---------------- BowVector: sort (word, feature) of the non-stopped features
  for (int i = threadIdx.x; i < P; i += T)
    keys[i] = (i < n && W[i] != VOC_STOP) ? (((unsigned long long)W[i] << 32) | (uint32_t)i)
                                          : ~0ull;
  __syncthreads();
  lds_bitonic(keys, P);
  // heads of word runs; thread t owns [t*per, t*per+per)
  int cnt = 0;
  const int i0 = threadIdx.x * per;
  for (int i = i0; i < i0 + per && i < P; ++i) {
    const unsigned long long k = keys[i];
    cnt += (k != ~0ull) && (i == 0 || (keys[i - 1] >> 32) != (k >> 32));
  }
  int nw;
  int pos = block_excl_scan(cnt, red, nw);
  for (int i = i0; i < i0 + per && i < P; ++i) {
    const unsigned long long k = keys[i];
    if (k == ~0ull || (i > 0 && (keys[i - 1] >> 32) == (k >> 32))) continue;
    const uint32_t word = (uint32_t)(k >> 32);
    double v = WT[(uint32_t)k];
    if (V.tf) {  // addWeight: += in ascending feature order
      for (int j = i + 1; j < P && keys[j] != ~0ull && (uint32_t)(keys[j] >> 32) == word; ++j)
        v += WT[(uint32_t)keys[j]];
    }  // else addIfNotExist: the first feature's weight
    bowWords[base + pos] = word;
    vals[pos] = v;
    ++pos;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double norm = 0.0;
    if (V.must) {  // BowVector::normalize (BowVector.cpp:59-81), in word order
      if (!V.l2) {
        for (int j = 0; j < nw; ++j) norm += fabs(vals[j]);
      } else {
        for (int j = 0; j < nw; ++j) norm += vals[j] * vals[j];
        norm = sqrt(norm);
      }
    } else if (V.tf && nw > 0) {
      norm = (double)nw;  // :1176-1181, divide by v.size()
    }
    normShared = norm;
    nWords[f] = nw;
  }
  __syncthreads();
  const double norm = normShared;
  for (int j = threadIdx.x; j < nw; j += T)
    bowValues[base + j] = norm > 0.0 ? vals[j] / norm : vals[j];
  __syncthreads();

  // ---------------- FeatureVector: sort (node, feature)
  for (int i = threadIdx.x; i < P; i += T)
    keys[i] = (i < n && W[i] != VOC_STOP) ? (((unsigned long long)ND[i] << 32) | (uint32_t)i)
                                          : ~0ull;
  __syncthreads();
  lds_bitonic(keys, P);
  cnt = 0;
  int valid = 0;
  for (int i = i0; i < i0 + per && i < P; ++i) {
    const unsigned long long k = keys[i];
    if (k == ~0ull) continue;
    ++valid;
    cnt += (i == 0 || (keys[i - 1] >> 32) != (k >> 32));
  }
  int nnodes, nvalid;
  pos = block_excl_scan(cnt, red, nnodes);
  block_excl_scan(valid, red, nvalid);
  uint32_t* FN = fvNodes + base;
  int32_t* FO = fvOffs + (size_t)f * (V.stride + 1);
  uint32_t* FF = fvFeats + base;
  for (int i = i0; i < i0 + per && i < P; ++i) {
    const unsigned long long k = keys[i];
    if (k == ~0ull) continue;
    FF[i] = (uint32_t)k;
    if (i == 0 || (keys[i - 1] >> 32) != (k >> 32)) {
      FN[pos] = (uint32_t)(k >> 32);
      FO[pos] = i;
      ++pos;
    }
  }
  if (threadIdx.x == 0) {
    FO[nnodes] = nvalid;
    nFv[f] = nnodes;
  }
}

extern "C" hipError_t orb_k_voc_descend(const void* info, const void* ndesc, const uint32_t* nword,
                                        const double* nweight, const uint32_t* norig,
                                        int nidLevel, const uint8_t* desc, const int32_t* counts,
                                        int nSingle, int stride, int nFrames, uint32_t* fword,
                                        double* fweight, uint32_t* fnode, hipStream_t s) {
  const long long groups = (long long)stride * nFrames;
  if (groups <= 0) return hipSuccess;
  const long long blocks = (groups + (256 / VOC_GROUP) - 1) / (256 / VOC_GROUP);
  hipLaunchKernelGGL(k_voc_descend, dim3((unsigned)blocks), dim3(256), 0, s,
                     (const VocNodeInfo*)info, (const uint4*)ndesc, nword, nweight, norig,
                     nidLevel, desc, counts, nSingle, stride, nFrames, fword, fweight, fnode);
  return hipGetLastError();
}

extern "C" int orb_k_voc_max_features() { return 8192; }

extern "C" hipError_t orb_k_voc_vectors(const uint32_t* fword, const double* fweight,
                                        const uint32_t* fnode, const int32_t* counts, int nSingle,
                                        int stride, int tf, int must, int l2, int nFrames,
                                        uint32_t* bowWords, double* bowValues, int32_t* nWords,
                                        uint32_t* fvNodes, int32_t* fvOffs, uint32_t* fvFeats,
                                        int32_t* nFv, hipStream_t s) {
  if (nFrames <= 0) return hipSuccess;
  int P = 256;
  while (P < stride) P <<= 1;
  if (P > 8192) return hipErrorInvalidValue;
  VocVecParams V{stride, tf, must, l2};
  const size_t lds = (size_t)P * 16;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_voc_vectors,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_voc_vectors, dim3(nFrames), dim3(256), lds, s, fword, fweight,
                     fnode, counts, nSingle, V, P, bowWords, bowValues, nWords, fvNodes, fvOffs,
                     fvFeats, nFv);
  return hipGetLastError();
}
