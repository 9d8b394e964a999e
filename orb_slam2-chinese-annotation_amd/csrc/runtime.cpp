// runtime.cpp -- host runtime behind the C ABI (include/orb_abi.h).
//
// Owns devices, streams, extraction plans and device scratch; launches the
// gfx950 kernels of extractor_kernels.hip / matcher_kernels.hip.  There is no
// CPU compute path: every ORB result comes from the HIP kernels, and every
// entry point fails with ORB_ENODEV / ORB_EDEVICE if the GPU path cannot run.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <shared_mutex>
#include <cmath>
#include <vector>

#include "../../include/orb_abi.h"
#include "orb_plan.h"
#include "orb_synth.h"

// ------------------------------------------------------- kernel launchers
extern "C" {
hipError_t orb_k_upload_constants(hipStream_t s);
hipError_t orb_k_upload_umax(const int* umax16, hipStream_t s);
hipError_t orb_k_pyr_resize(const uint8_t* src, long long srcImgPitch, int srcStride, int sw,
                            int sh, uint8_t* dst, long long dstImgPitch, int dstStride, int dw,
                            int dh, const int* xofs, const void* alpha, const int* yofs,
                            const void* beta, int mode, int nimg, hipStream_t s);
size_t orb_k_fast_band_lds(int bandElems);
hipError_t orb_k_copy_pinned(void* dst, const void* src, size_t bytes, hipStream_t s);
hipError_t orb_k_copy_to_pinned(void* dst, const void* src, size_t bytes, hipStream_t s);
size_t orb_k_fast_cells_lds(int maxRows, int maxCols);
bool orb_k_fast_cells_fits(const OrbPlanDesc* plan);

hipError_t orb_k_pyr_resize2(const uint8_t* src, long long srcImgPitch, int srcStride, int w0,
                             int h0, uint8_t* mid, long long midImgPitch, int midStride, int w1,
                             int h1, const int* xo1, const void* al1, const int* yo1,
                             const void* be1, uint8_t* dst, long long dstImgPitch, int dstStride,
                             int w2, int h2, const int* xo2, const void* al2, const int* yo2,
                             const void* be2, int nimg, hipStream_t s);
int orb_k_pyr_resize2_fits(int w0, int h0, int w1, int h1, const int* xo1, const int* yo1, int w2,
                           int h2, const int* xo2, const int* yo2);
hipError_t orb_k_fast_cells(const uint8_t* img0, long long img0Pitch, int img0Stride,
                            const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                            const OrbCellDesc* cells, uint32_t* cellKeys, int32_t* cellCount,
                            int32_t* errFlag, int cellBeg, int cellEnd, int nimg, hipStream_t s);
hipError_t orb_k_fast_band(const uint8_t* img0, long long img0Pitch, int img0Stride,
                           const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                           const OrbBandDesc* bands, int nbands, const OrbCellDesc* cells,
                           uint32_t* cellKeys, int32_t* cellCount, int32_t* errFlag, int nimg,
                           hipStream_t s);
size_t orb_k_octree_lds(int nodeCapMax, int maxCellsPerLevel, int ldsKeyCap);
hipError_t orb_k_octree(const OrbPlanDesc* plan, const int32_t* cellCount,
                        const uint32_t* cellKeys, uint32_t* gKeys, uint16_t* gNid, int ldsKeyCap,
                        int nodeCapMax, int maxCellsPerLevel, uint32_t* outKeys,
                        int32_t* outCount, int32_t* errFlag, int levelBeg, int levelEnd, int nimg,
                        uint8_t* gNodes, long long nodeStride, hipStream_t s);
hipError_t orb_k_blur_levels(const uint8_t* img0, long long img0Pitch, int img0Stride,
                             const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                             const OrbTileDesc* tiles, uint8_t* blur, long long blurPitch,
                             int nimg, hipStream_t s);
hipError_t orb_k_orient_desc(const uint8_t* img0, long long img0Pitch, int img0Stride,
                             const uint8_t* arena, long long arenaPitch, const OrbPlanDesc* plan,
                             const uint32_t* outKeys, const int32_t* outCount,
                             const int32_t* errFlag, orb_keypoint_t* kps, uint8_t* desc,
                             int capacity, int32_t* counts, int nimg, int levelBeg,
                             int levelEnd, hipStream_t s);
hipError_t orb_k_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* out, hipStream_t s);
hipError_t orb_k_grid_build(const orb_keypoint_t* keys, const int32_t* nkeys, int kpStride,
                            float minX, float minY, float invW, float invH, int32_t* cellStart,
                            int32_t* cellIdx, int nproblems, hipStream_t s);
hipError_t orb_k_proj_candidates(const orb_keypoint_t* keys, const uint8_t* desc,
                                 const float* uright, const uint8_t* locked, int kpStride,
                                 const int32_t* nkeys, const orb_mp_track_t* mps,
                                 const uint8_t* mpDesc,
                                 const int32_t* nmps, int mpStride, int mpMax,
                                 const int32_t* cellStart, const int32_t* cellIdx,
                                 const void* stagedGrid, const void* params, uint32_t* topk,
                                 int32_t* ncand, int nproblems, hipStream_t s);
hipError_t orb_k_grid_build_staged(const orb_keypoint_t* keys, const int32_t* nkeys,
                                   const uint8_t* locked, const float* uright, int kpStride,
                                   float minX, float minY, float invW, float invH,
                                   int32_t* cellStart, int32_t* cellIdx, void* staged,
                                   int nproblems, hipStream_t s);
int orb_k_grid_stage_max(void);
hipError_t orb_k_proj_resolve(const orb_keypoint_t* keys, const uint8_t* desc,
                              const float* uright, const uint8_t* locked, const int32_t* nkeys,
                              int kpStride, const orb_mp_track_t* mps, const uint8_t* mpDesc,
                              const int32_t* nmps, int mpStride, const int32_t* cellStart,
                              const int32_t* cellIdx, const void* params, const uint32_t* topk,
                              const int32_t* ncand, int32_t* kpMatch, int32_t* nmatches,
                              int nproblems, int schedule, int jacobiRounds, int32_t* jacScratch,
                              hipStream_t s);
int orb_k_proj_resolve_kernel(int nproblems, int kpStride, int mpStride, int schedule);
size_t orb_k_proj_jacobi_bytes(int kpStride, int mpStride, int nproblems, int schedule);
size_t orb_k_proj_params_size(void);
size_t orb_k_proj_ovf_bytes(int nproblems);
size_t orb_k_stereo_params_size(void);
hipError_t orb_k_stereo(const orb_keypoint_t* lkeys, const uint8_t* ldesc, const int32_t* nleft,
                        const orb_keypoint_t* rkeys, const uint8_t* rdesc, const int32_t* nright,
                        int kpStride, int maxLeft, const void* pyr, const void* params,
                        float* uRight, float* depth, int32_t* sad, int npairs,
                        int32_t* rowStart, int32_t* rowIdx, hipStream_t s);
void orb_k_stereo_scratch(const void* params, int kpStride, size_t* startInts, size_t* idxInts);
size_t orb_k_frame_params_size(void);
size_t orb_k_frustum_params_size(void);
hipError_t orb_k_frustum(const orb_map_point_t* mps, const int32_t* nmps, int mpStride,
                         int mpMax, const orb_pose_t* poses, const void* params,
                         orb_mp_track_t* tracks, int32_t* nInView, int nproblems, hipStream_t s);
hipError_t orb_k_frame_proj(const orb_keypoint_t* keys, const uint8_t* desc, const float* uright,
                            const uint8_t* locked, int nkeys, const orb_last_mp_t* last,
                            const uint8_t* lastDesc, int nlast, const int32_t* cellStart,
                            const int32_t* cellIdx, const void* params, uint32_t* topk,
                            int32_t* ncand, int32_t* kpMatch, int32_t* nmatches, hipStream_t s);
hipError_t orb_k_bow(const uint8_t* kfDesc, const float* kfAngle, const int32_t* kfMp,
                     const uint8_t* kfBad, int kfNodes, const uint32_t* kfNodeIds,
                     const int32_t* kfOffs, const uint32_t* kfFeats, int nKfFeats,
                     const uint8_t* fDesc, const float* fAngle, int fNodes,
                     const uint32_t* fNodeIds, const int32_t* fOffs, const uint32_t* fFeats,
                     int nF, const int32_t* fMp, const uint8_t* fBad, int thLow,
                     float nnratio, int checkOri, int32_t* fMatch, int32_t* accF,
                     int32_t* nmatches, hipStream_t s);
size_t orb_k_pp_params_size(void);
size_t orb_k_pp_rec_size(void);
size_t orb_k_tri_params_size(void);
size_t orb_k_pp_resolve_lds(int nkeys, int n);
hipError_t orb_k_pp_match(int mode, const orb_map_point_t* mps, const uint8_t* mpValid,
                          const uint8_t* mpSkip, const uint8_t* mpDesc, int n,
                          const orb_keypoint_t* keys, const uint8_t* desc, const float* uright,
                          const int32_t* cellStart, const int32_t* cellIdx, const void* params,
                          void* recs, int32_t* best, uint32_t* topk, int32_t* ncand,
                          hipStream_t s);
hipError_t orb_k_pp_resolve(const orb_keypoint_t* keys, const uint8_t* desc, int nkeys,
                            const uint8_t* kpLocked, const uint8_t* mpDesc, const float* mpAngle,
                            int n, const int32_t* cellStart, const int32_t* cellIdx,
                            const void* params, const void* recs, const uint32_t* topk,
                            const int32_t* ncand, int32_t* kpMatch, int32_t* nmatches,
                            hipStream_t s);
hipError_t orb_k_sim3_mutual(const int32_t* m1, int n1, const int32_t* m2, int32_t* match12,
                             int32_t* nfound, hipStream_t s);
hipError_t orb_k_triangulation(const orb_keypoint_t* k1, const uint8_t* d1, const float* ur1,
                               const uint8_t* hasMp1, int nodes1, const uint32_t* ids1,
                               const int32_t* offs1, const uint32_t* feats1, int nFeats1,
                               const orb_keypoint_t* k2, const uint8_t* d2, const float* ur2,
                               const uint8_t* hasMp2, int nodes2, const uint32_t* ids2,
                               const int32_t* offs2, const uint32_t* feats2, const void* params,
                               int32_t* match12, int32_t* acc, int32_t* nmatches, hipStream_t s);
size_t orb_k_init_params_size(void);
size_t orb_k_init_list_len(void);
size_t orb_k_init_topk(void);
size_t orb_k_init_lds(int kpStride);
hipError_t orb_k_search_init(const orb_keypoint_t* keys1, const uint8_t* desc1, const int32_t* n1,
                             const orb_keypoint_t* keys2, const uint8_t* desc2, const int32_t* n2,
                             int kpStride, float* prev, const int32_t* cellStart,
                             const int32_t* cellIdx, const void* params, int32_t* qList,
                             int32_t* qOrder, int32_t* nQ, void* stage, int32_t* nStage, uint32_t* topk,
                             uint32_t* list, int32_t* ncand, int32_t* m12, int32_t* nmatches,
                             int nproblems, hipStream_t s);
size_t orb_k_init_key_size(void);
hipError_t orb_k_distinctive(const int32_t* offs, const uint8_t* desc, int nmp, int32_t* best,
                             uint8_t* out, hipStream_t s);
hipError_t orb_k_voc_descend(const void* info, const void* ndesc, const uint32_t* nword,
                             const double* nweight, const uint32_t* norig, int nidLevel,
                             const uint8_t* desc, const int32_t* counts, int nSingle, int stride,
                             int nFrames, uint32_t* fword, double* fweight, uint32_t* fnode,
                             hipStream_t s);
int orb_k_voc_max_features(void);
hipError_t orb_k_undistort_points(const void* params, int n, const float* in, float* out,
                                  hipStream_t s);
hipError_t orb_k_undistort_keys(const void* params, int nFrames, const int32_t* counts,
                                int nSingle, int stride, const void* in, void* out, int copyOnly,
                                hipStream_t s);
size_t orb_k_undistort_params_size(void);
hipError_t orb_k_voc_vectors(const uint32_t* fword, const double* fweight, const uint32_t* fnode,
                             const int32_t* counts, int nSingle, int stride, int tf, int must,
                             int l2, int nFrames, uint32_t* bowWords, double* bowValues,
                             int32_t* nWords, uint32_t* fvNodes, int32_t* fvOffs,
                             uint32_t* fvFeats, int32_t* nFv, hipStream_t s);
}

namespace {

#define HIP_TRY(expr)                                   \
  do {                                                  \
    hipError_t _e = (expr);                             \
    if (_e != hipSuccess) {                             \
      if (getenv("ORB_AMD_DEBUG"))                      \
        fprintf(stderr, "[orb_amd] %s:%d %s -> %s\n", __FILE__, __LINE__, #expr, \
                hipGetErrorString(_e));                 \
      return _e == hipErrorOutOfMemory ? ORB_ENOMEM : ORB_EDEVICE; \
    }                                                   \
  } while (0)

static inline int cvRoundF(float v) { return (int)lrintf(v); }
static inline short satShort(int v) { return (short)std::min(std::max(v, -32768), 32767); }

static bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cst) == hipSuccess && cst != hipStreamCaptureStatusNone;
}

// Call order on one handle.  Every call reuses the handle's device scratch
// (the extractor's arena, cell keys and octree tables; the matcher's grid,
// candidate lists and claim buffers), and a batch call runs asynchronously on
// whatever stream its caller passes, so a call on a stream other than the
// previous call's makes its stream wait for that call first (on the device, no
// host synchronisation), and every call records where it ended.  The reference
// has the same rule in host form: an ORBextractor is not reentrant
// (include/ORBextractor.h:85), a Frame drives two instances concurrently
// (src/Frame.cc:81-84).  A stream being captured into a graph is left to the
// caller's ordering of the graph's launches.  (Growing a scratch buffer is
// safe on its own: hipFree synchronises the device.)
#ifndef ORB_CALL_ORDER
#define ORB_CALL_ORDER 1  // 0: no cross-stream waits (the ordering test's negative control only)
#endif
static inline bool must_wait(hipStream_t last, hipStream_t s) {
  return ORB_CALL_ORDER && last && last != s;
}
struct CallOrder {
  hipEvent_t ev;
  hipStream_t* last;
  hipStream_t s;
  bool capture;
  orb_status_t status = ORB_OK;
  CallOrder(hipEvent_t e, hipStream_t* l, hipStream_t st)
      : ev(e), last(l), s(st), capture(stream_capturing(st)) {
    if (!capture && must_wait(*last, s) && hipStreamWaitEvent(s, ev, 0) != hipSuccess)
      status = ORB_EDEVICE;
  }
  // the call synchronised its stream: nothing of it is pending any more
  void settled() {
    if (!capture) *last = nullptr;
    capture = true;
  }
  ~CallOrder() {
    if (!capture && hipEventRecord(ev, s) == hipSuccess) *last = s;
  }
};

// Wait for a stream whose results the caller reads next.  The synchronous
// entry points (one frame, one SearchByProjection) sit on the tracking
// thread's critical path, where hipStreamSynchronize returned 5-13 us after
// the stream's last operation (profiles/r06_dropin_timeline.txt); polling the
// stream returns within a query (~1 us) of it.  Bounded: past 2 ms of polling
// the wait blocks as hipStreamSynchronize does.
#ifndef ORB_POLL_WAIT
#define ORB_POLL_WAIT 1  // A/B knob (0: hipStreamSynchronize)
#endif
static hipError_t stream_wait(hipStream_t s) {
  if (!ORB_POLL_WAIT) return hipStreamSynchronize(s);
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 1;; ++i) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    if ((i & 63) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2))
      return hipStreamSynchronize(s);
  }
}

// Growable device buffer.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  orb_status_t ensure(size_t n) {
    if (n <= bytes) return ORB_OK;
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, n) != hipSuccess) return ORB_ENOMEM;
    bytes = n;
    return ORB_OK;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T>
  T* as() const { return (T*)p; }
};

// Pinned host staging for the host-buffer API: one contiguous DMA each way
// (a 2-D copy from pageable memory goes row by row, ~7 us per row).
struct HostBuf {
  void* p = nullptr;
  size_t bytes = 0;
  orb_status_t ensure(size_t n) {
    if (n <= bytes) return ORB_OK;
    if (p) hipHostFree(p);
    p = nullptr;
    bytes = 0;
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return ORB_ENOMEM;
    bytes = n;
    return ORB_OK;
  }
  void release() {
    if (p) hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T>
  T* as() const { return (T*)p; }
};

// HIP-event timing of kernel stages on the stream they are launched on.  Each
// profiled call takes a fresh set of events from a pool (no synchronisation in
// the launch path); read() drains every recorded set and accumulates per-stage
// milliseconds, so a timed region of K calls is measured without perturbing it.
struct StageProfiler {
  // Per call: (begin, end) event pairs per stage -- up to maxSeg[stage]
  // segments, e.g. one per level for a stage launched level by level, whose
  // durations are summed -- recorded on whichever stream runs that stage
  // (stages may overlap), plus a (begin, end) pair for the whole call on the
  // caller's stream.
  static constexpr int kMaxStages = 8;
  bool enabled = false;
  bool serial = false;  // isolated timing: every stage on the caller's stream, one after another
  int nStages = 0;
  const char* names[kMaxStages] = {};
  int maxSeg[kMaxStages] = {1, 1, 1, 1, 1, 1, 1, 1};
  std::vector<std::vector<hipEvent_t>> pool;  // each: 2 * sum(maxSeg) + 2 events
  std::vector<std::vector<uint8_t>> segs;     // per call: segments recorded per stage
  size_t used = 0;
  double ms[kMaxStages + 1] = {};
  long launches[kMaxStages + 1] = {};
  int launchesPerCall[kMaxStages] = {};

  int base(int stage) const {
    int o = 0;
    for (int i = 0; i < stage; ++i) o += maxSeg[i];
    return o;
  }
  int total() const { return base(nStages); }
  void reset() {
    used = 0;
    for (int i = 0; i <= kMaxStages; ++i) { ms[i] = 0; launches[i] = 0; }
  }
  std::vector<hipEvent_t>* begin_call() {
    if (!enabled) return nullptr;
    if (used == pool.size()) {
      pool.emplace_back(2 * total() + 2);
      for (hipEvent_t& e : pool.back()) hipEventCreate(&e);
      segs.emplace_back(kMaxStages, 0);
    }
    std::fill(segs[used].begin(), segs[used].end(), (uint8_t)1);
    return &pool[used++];
  }
  // of the current call: stage not run / run as n segments
  void not_run(int stage) { segs[used - 1][stage] = 0; }
  void segments(int stage, int n) { segs[used - 1][stage] = (uint8_t)n; }
  hipEvent_t b(std::vector<hipEvent_t>* ev, int stage, int seg = 0) const {
    return (*ev)[2 * (base(stage) + seg)];
  }
  hipEvent_t e(std::vector<hipEvent_t>* ev, int stage, int seg = 0) const {
    return (*ev)[2 * (base(stage) + seg) + 1];
  }
  hipEvent_t t0(std::vector<hipEvent_t>* ev) const { return (*ev)[2 * total()]; }
  hipEvent_t t1(std::vector<hipEvent_t>* ev) const { return (*ev)[2 * total() + 1]; }
  void drain() {
    for (size_t c = 0; c < used; ++c) {
      std::vector<hipEvent_t>& ev = pool[c];
      if (hipEventSynchronize(t1(&ev)) != hipSuccess) continue;
      for (int i = 0; i < nStages; ++i) {
        if (launchesPerCall[i] == 0 || segs[c][i] == 0) continue;  // stage not run
        bool ok = true;
        double sum = 0;
        for (int g = 0; g < segs[c][i] && ok; ++g) {
          float t = 0.f;
          ok = hipEventElapsedTime(&t, b(&ev, i, g), e(&ev, i, g)) == hipSuccess;
          sum += t;
        }
        if (ok) {
          ms[i] += sum;
          launches[i] += launchesPerCall[i];
        } else {
          (void)hipGetLastError();  // clear it: torch checks the last error after its launches
        }
      }
      float t = 0.f;
      if (hipEventElapsedTime(&t, t0(&ev), t1(&ev)) == hipSuccess) {
        ms[nStages] += t;
        launches[nStages] += 1;
      }
    }
    used = 0;
  }
  void destroy() {
    for (auto& v : pool)
      for (hipEvent_t ev : v) hipEventDestroy(ev);
    pool.clear();
    segs.clear();
    used = 0;
  }
};

#define PROF_REC(ev, evt, strm) \
  do {                                            \
    if (ev) HIP_TRY(hipEventRecord((evt), (strm))); \
  } while (0)

orb_status_t check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ORB_ENODEV;
  if (device < 0 || device >= n) return ORB_EINVAL;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ORB_EDEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    if (getenv("ORB_AMD_DEBUG")) fprintf(stderr, "[orb_amd] device %d is %s, need gfx950\n", device, prop.gcnArchName);
    return ORB_ENODEV;
  }
  return ORB_OK;
}

}  // namespace

// ================================================================ extractor
struct orb_extractor {
  int device = 0;
  int nfeatures = 0, nlevels = 0, iniTh = 0, minTh = 0;
  float scaleFactorF = 1.2f;
  double scaleFactor = 1.2;
  std::vector<float> scale, invScale, sigma2, invSigma2;
  std::vector<int> quota;
  int umax[16];
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // the device's shared side stream: FAST beside the resize chain
  hipStream_t privSide = nullptr; // this handle's side stream while its caller's stream is captured
  hipEvent_t evL0Fork = nullptr, evL0Join = nullptr;  // level-0 FAST beside the resize chain
  hipEvent_t evLvl = nullptr;  // the resize chain has written level FAST_SIDE_LEVELS
  hipEvent_t evBatch = nullptr;  // recorded at the end of every run_batch on its stream
  hipStream_t lastStream = nullptr;  // the stream evBatch was last recorded on (null: none pending)
  bool ownStream = false;
  std::mutex mu;

  // plan for the current image size
  int planW = -1, planH = -1;
  OrbPlanDesc plan;
  std::vector<OrbCellDesc> cells;
  long long arenaBytes = 0, blurBytes = 0;
  int maxCellsPerLevel = 0, nodeCapMax = 0, ldsKeyCap = 0;
  int nResizePairs = 0;  // resize launches per call with the level pairs (PYR_PAIR_MAX_IMAGES)
  DevBuf dCells, dRtab, dTiles, dBands;

  // batch scratch
  int batchCap = 0;
  DevBuf dBlur;  // one image's blurred levels (orb_extractor_blurred_level, on demand)
  DevBuf dArena, dCellKeys, dCellCount, dGKeys, dGNid, dOutKeys, dOutCount, dErr;
  DevBuf dOctNodes;            // octree node tables in global memory (large nfeatures)
  long long octNodeBytes = 0;  // per (image, level) slice; 0: node tables in LDS
  // single-image API scratch
  // single-image API: dImg (the image at a 64-B row pitch) and dOne = [count,
  // pad x3 | cap keypoints | cap x 32 descriptors], mirrored by the pinned
  // hImg / hOut so each call is one DMA in and one DMA out
  DevBuf dImg, dOne;
  HostBuf hImg, hOut, hLvl;  // hLvl: staging of orb_extractor_pyramid_level / _blurred_level
  // host mirror of the single-frame call's levels 1.. (orb_extractor_host_pyramid):
  // once asked for, the arena's D2H joins every later call's graph
  HostBuf hPyr;
  bool pyrReadback = false, hPyrValid = false;
  int oneCap = 0;            // capacity of the dOne layout
  bool lastSingle = false;   // the last call was orb_extractor_extract (dOne is current)
  // the whole single-image call (H2D, every kernel, D2H) as one hipGraph per
  // plan; keyed by the buffers it captured (any reallocation re-captures)
  hipGraphExec_t oneExec = nullptr;
  std::vector<const void*> oneKey;
  int lastW = 0, lastH = 0;
  size_t lastImgStride = 0;
  const uint8_t* lastImg0 = nullptr;  // level 0 of the last batch (device)
  size_t lastImg0Pitch = 0;
  int lastImg0Stride = 0;

  // profiling: stages k_pyr_resize (x nlevels-1), k_blur_levels, k_fast_band, k_octree,
  // k_orient_desc
  StageProfiler prof;
};

static void compute_tables(orb_extractor* h) {
  const int L = h->nlevels;
  h->scale.assign(L, 0.f);
  h->sigma2.assign(L, 0.f);
  h->scale[0] = 1.0f;
  h->sigma2[0] = 1.0f;
  for (int i = 1; i < L; ++i) {  // src/ORBextractor.cc:437-441 (scaleFactor is a double member)
    h->scale[i] = (float)((double)h->scale[i - 1] * h->scaleFactor);
    h->sigma2[i] = h->scale[i] * h->scale[i];
  }
  h->invScale.resize(L);
  h->invSigma2.resize(L);
  for (int i = 0; i < L; ++i) {
    h->invScale[i] = 1.0f / h->scale[i];
    h->invSigma2[i] = 1.0f / h->sigma2[i];
  }
  h->quota.assign(L, 0);  // :453-464
  const float factor = (float)(1.0f / h->scaleFactor);
  float nDesired = (float)h->nfeatures * (1 - factor) /
                   (1 - (float)pow((double)factor, (double)L));
  int sum = 0;
  for (int l = 0; l < L - 1; ++l) {
    h->quota[l] = cvRoundF(nDesired);
    sum += h->quota[l];
    nDesired *= factor;
  }
  h->quota[L - 1] = std::max(h->nfeatures - sum, 0);
  const int HP = 15;  // :473-488
  const int vmax = (int)floorf(HP * sqrtf(2.f) / 2 + 1);
  const int vmin = (int)ceilf(HP * sqrtf(2.f) / 2);
  const double hp2 = HP * HP;
  for (int v = 0; v <= vmax; ++v) h->umax[v] = (int)lrint(sqrt(hp2 - v * v));
  for (int v = HP, v0 = 0; v >= vmin; --v) {
    while (h->umax[v0] == h->umax[v0 + 1]) ++v0;
    h->umax[v] = v0;
    ++v0;
  }
}

// Build the plan for a W x H input (level sizes, resize tables, FAST cells,
// octree roots, output slots) and upload its tables.
#ifndef PYR_FUSE2
#define PYR_FUSE2 1  // level pairs in one k_pyr_resize2 launch where they fit (0: one launch per level)
#endif
#ifndef PYR_PAIR_MAX_IMAGES
// calls of at most this many images take the level pairs; larger batches one
// launch per level: the pairs save a frame 4 us of latency but cost batches
// 0.3-1 % (C4), 1.5 % (C3) and 2 % (C5) (profiles/r06_resize2_fast_runs.txt)
#define PYR_PAIR_MAX_IMAGES 8
#endif
static orb_status_t build_plan(orb_extractor* h, int W, int H) {
  if (h->planW == W && h->planH == H) return ORB_OK;
  const int L = h->nlevels;
  OrbPlanDesc P;
  memset(&P, 0, sizeof(P));
  P.nlevels = L;
  P.iniTh = h->iniTh;
  P.minTh = h->minTh;
  P.srcW = W;
  P.srcH = H;
  std::vector<OrbCellDesc> cells;
  std::vector<int32_t> rtab;
  std::vector<OrbTileDesc> tiles;
  std::vector<OrbBandDesc> bands;
  int maxBandBytes = 0;
  const int bandBudget = ORB_BAND_BYTES;  // k_fast_band stages <= 8192 elements per pass
  long long arena = 0, blurArena = 0;
  int keyCap = 1, maxRows = 7, maxCols = 7, maxCellsPerLevel = 1, nodeCapMax = 1, slots = 0;
  for (int l = 0; l < L; ++l) {
    OrbLevelDesc& d = P.lv[l];
    d.w = l ? cvRoundF((float)W * h->invScale[l]) : W;  // src/ORBextractor.cc:1180
    d.h = l ? cvRoundF((float)H * h->invScale[l]) : H;
    // a level needs more than the 2 x 16 px FAST border in each direction
    // (src/ORBextractor.cc:797-800); at 32 px or less the reference's
    // DistributeOctTree divides by zero or sizes a vector negatively (:562-569)
    if (d.w < 33 || d.h < 33 || d.w > 4095 || d.h > 4095) return ORB_EINVAL;
    d.pitch = ((d.w + 127) & ~127) | 128;  // odd multiple of 128 B: whole-line rows, channel spread
    d.arenaOff = l ? arena : 0;
    if (l) arena += (long long)d.pitch * d.h;
    d.blurPitch = ((d.w + 127) & ~127) | 128;
    d.blurOff = blurArena;
    blurArena += (long long)d.blurPitch * d.h;
    d.tileBeg = (int)tiles.size();
    for (int y0 = 0; y0 < d.h; y0 += ORB_BLUR_TH)
      for (int x0 = 0; x0 < d.w; x0 += ORB_BLUR_TW) {
        OrbTileDesc t;
        t.level = (int16_t)l;
        t.x0 = (int16_t)x0;
        t.y0 = (int16_t)y0;
        t._pad = 0;
        tiles.push_back(t);
      }
    d.scale = h->scale[l];
    d.sizeF = (float)(int)(31 * h->scale[l]);
    d.quota = h->quota[l];
    // FAST cell grid, src/ORBextractor.cc:797-839
    const int minBX = 16, minBY = 16, maxBX = d.w - 16, maxBY = d.h - 16;
    const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
    const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
    // a level under 30 px of border-free width or height has no cells (the
    // reference's cell loops run zero times: no keypoints on that level)
    const int wCell = nCols > 0 ? (int)ceilf(width / nCols) : 0;
    const int hCell = nRows > 0 ? (int)ceilf(height / nRows) : 0;
    d.cellBeg = (int)cells.size();
    for (int i = 0; i < nRows && nCols > 0; ++i) {
      const float iniY = (float)(minBY + i * hCell);
      float maxY = iniY + hCell + 6;
      if (iniY >= maxBY - 3) continue;
      if (maxY > maxBY) maxY = (float)maxBY;
      for (int j = 0; j < nCols; ++j) {
        const float iniX = (float)(minBX + j * wCell);
        float maxX = iniX + wCell + 6;
        if (iniX >= maxBX - 6) continue;
        if (maxX > maxBX) maxX = (float)maxBX;
        OrbCellDesc c;
        c.level = (int16_t)l;
        c.y0 = (int16_t)(int)iniY;
        c.y1 = (int16_t)(int)maxY;
        c.x0 = (int16_t)(int)iniX;
        c.x1 = (int16_t)(int)maxX;
        c._pad = 0;
        cells.push_back(c);
        const int rows = c.y1 - c.y0, cols = c.x1 - c.x0;
        maxRows = std::max(maxRows, rows);
        maxCols = std::max(maxCols, cols);
        d.cellMaxRows = std::max(d.cellMaxRows, rows);
        d.cellMaxCols = std::max(d.cellMaxCols, cols);
        if (rows >= 7 && cols >= 7)
          keyCap = std::max(keyCap, ((rows - 6 + 1) / 2) * ((cols - 6 + 1) / 2));
      }
    }
    d.cellEnd = (int)cells.size();
    // FAST bands: runs of consecutive cells of one cell row whose union ROI
    // fits the band LDS budget (k_fast_band; ORB_BAND_BYTES)
    for (int c = d.cellBeg; c < d.cellEnd;) {
      OrbBandDesc b;
      b.level = (int16_t)l;
      b.y0 = cells[c].y0;
      b.y1 = cells[c].y1;
      b.x0 = cells[c].x0;
      b.x1 = cells[c].x1;
      b.cellBeg = c;
      int e = c + 1;
      while (e < d.cellEnd && cells[e].y0 == b.y0 && e - c < 64) {  // k_fast_band: <= 64 cells
        const int x1 = std::max<int>(b.x1, cells[e].x1);
        if ((b.y1 - b.y0) * ((x1 - b.x0 + 20) & ~7) > bandBudget) break;
        b.x1 = (int16_t)x1;
        ++e;
      }
      b.nCells = (int16_t)(e - c);
      // k_fast_band compacts a cell window with one lane per row and one
      // 64-bit word per row segment
      if (b.y1 - b.y0 - 6 > 64) return ORB_EINVAL;
      for (int k = c; k < e; ++k)
        if (cells[k].x1 - cells[k].x0 - 6 > 64) return ORB_EINVAL;
      // k_fast_band's LDS row pitch in elements ((C + 20) & ~7, see the kernel)
      maxBandBytes = std::max(maxBandBytes, (b.y1 - b.y0) * ((b.x1 - b.x0 + 20) & ~7));
      bands.push_back(b);
      c = e;
    }
    maxCellsPerLevel = std::max(maxCellsPerLevel, d.cellEnd - d.cellBeg);
    // octree roots, src/ORBextractor.cc:562-564
    d.Wr = maxBX - minBX;
    d.Hr = maxBY - minBY;
    d.nIni = (int)roundf((float)d.Wr / d.Hr);
    // no root at all (width under half the height): the reference indexes an
    // empty root vector for every key (:569,588); a level without cells has no
    // keys, so one root stands in for none
    if (d.nIni <= 0 && d.cellEnd > d.cellBeg) return ORB_EINVAL;
    d.nIni = std::max(d.nIni, 1);
    d.hX = (float)d.Wr / d.nIni;
    d.nodeCap = (std::max(d.quota + 4, 4 * d.nIni + 4) + 1) & ~1;  // even: k_orient_desc slot pairs
    // k_octree labels a level's keys with 16-bit node indices (its final-phase
    // sort key packs size 24 | creation order 24 | node 16 bits): a level's
    // quota may reach 65,530 (nfeatures ~300,000 at 1.2 / 8 levels)
    if (d.nodeCap > 65534) return ORB_EINVAL;
    nodeCapMax = std::max(nodeCapMax, d.nodeCap);
    d.outOff = slots;
    slots += d.nodeCap;
    // resize tables (level l from level l-1), SURVEY.md Appendix A.2
    if (l) {
      const int sw = P.lv[l - 1].w, sh = P.lv[l - 1].h;
      const double scale_x = 1. / ((double)d.w / sw), scale_y = 1. / ((double)d.h / sh);
      d.rtabX = (int)rtab.size();
      rtab.resize(rtab.size() + 2 * (size_t)d.w);
      int xmax = d.w;
      for (int dx = 0; dx < d.w; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
          xmax = std::min(xmax, dx);
          if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        const short a0 = satShort(cvRoundF((1.f - fx) * 2048)), a1 = satShort(cvRoundF(fx * 2048));
        rtab[d.rtabX + dx] = sx;
        rtab[d.rtabX + d.w + dx] = (int32_t)(((uint32_t)(uint16_t)a1 << 16) | (uint16_t)a0);
      }
      d.xmax = xmax;
      d.rtabY = (int)rtab.size();
      rtab.resize(rtab.size() + 2 * (size_t)d.h);
      for (int dy = 0; dy < d.h; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)floorf(fy);
        fy -= sy;
        const short b0 = satShort(cvRoundF((1.f - fy) * 2048)), b1 = satShort(cvRoundF(fy * 2048));
        rtab[d.rtabY + dy] = sy;
        rtab[d.rtabY + d.h + dy] = (int32_t)(((uint32_t)(uint16_t)b1 << 16) | (uint16_t)b0);
      }
      // k_pyr_resize stages each 128 x 32 output tile's source window in LDS
      // (narrow 44 x 44 dwords up to a 1.25 downscale, wide 64 x 64 beyond),
      // and each thread's 4 columns read 8 staged source bytes: the level takes
      // the first variant every tile fits, else the untiled generic kernel
      // (per-level downscales beyond ~1.9: scaleFactor > 1.9, which no
      // ORB-SLAM2 configuration uses)
      const int32_t* xo = &rtab[d.rtabX];
      const int32_t* yo = &rtab[d.rtabY];
      auto tiles_fit = [&](int SR, int SWd) {
        for (int x = 0; x < d.w; x += 4)
          if (xo[std::min(x + 3, d.w - 1)] - xo[x] > 6) return false;
        for (int x0 = 0; x0 < d.w; x0 += 128) {
          const int xl = std::min(x0 + 127, d.w - 1), xt = std::min(x0 + 124, d.w - 1);
          const int colBase = xo[x0] & ~3, sxB = std::min(xo[xl] + 1, sw - 1);
          const int nW = ((sxB - colBase) >> 2) + 1, lastRead = ((xo[xt] - colBase) >> 2) + 2;
          if (nW > 64 || nW > SWd || lastRead >= SWd) return false;
        }
        for (int y0 = 0; y0 < d.h; y0 += 32) {
          const int yl = std::min(y0 + 31, d.h - 1);
          const int syA = std::min(std::max(yo[y0], 0), sh - 1);
          const int syB = std::min(std::max(yo[yl] + 1, 0), sh - 1);
          if (syB - syA + 1 > SR) return false;
        }
        return true;
      };
      const bool narrowOk = (double)sw / d.w <= 1.25 && (double)sh / d.h <= 1.25;
      d.resizeMode = narrowOk && tiles_fit(44, 44) ? ORB_RESIZE_NARROW
                     : tiles_fit(64, 64)          ? ORB_RESIZE_WIDE
                                                  : ORB_RESIZE_GENERIC;
    }
  }
  // Pairs of levels built by one launch (k_pyr_resize2: level l + 1 from a
  // level-l region the workgroup computes in LDS from level l - 1): greedily
  // from level 1, where both levels take the narrow tiles and every tile of
  // the pair fits the kernel's windows (every ORB-SLAM2 configuration: 1+2,
  // 3+4, 5+6, then 7 alone); other levels keep one launch each
  int nResize = 0;
  for (int l = 1; l < L;) {
    OrbLevelDesc& d = P.lv[l];
    d.resize2 = 0;
    if (PYR_FUSE2 && l + 1 < L && d.resizeMode == ORB_RESIZE_NARROW &&
        P.lv[l + 1].resizeMode == ORB_RESIZE_NARROW) {
      const OrbLevelDesc& e = P.lv[l + 1];
      d.resize2 = orb_k_pyr_resize2_fits(P.lv[l - 1].w, P.lv[l - 1].h, d.w, d.h, &rtab[d.rtabX],
                                         &rtab[d.rtabY], e.w, e.h, &rtab[e.rtabX], &rtab[e.rtabY]);
    }
    l += d.resize2 ? 2 : 1;
    ++nResize;
  }
  // k_fast_band: one band = at least one cell; its pixels and scores + the
  // candidate queue must fit the 64 KiB a workgroup may allocate
  if (orb_k_fast_band_lds(maxBandBytes) > 64 * 1024) return ORB_EINVAL;
  P.ncells = (int)cells.size();
  P.nBlurTiles = (int)tiles.size();
  P.nBands = (int)bands.size();
  P.maxBandBytes = maxBandBytes;
  P.keyCap = keyCap;
  P.slotsPerImage = slots;
  P.maxCellRows = maxRows;
  P.maxCellCols = maxCols;
  // octree LDS: node tables + keys within ~52 KiB (three workgroups per CU
  // overlap their latency-bound passes; budgets of 24-64 KiB measured 52 +- 1 %);
  // a level with more candidate keys keeps them in global scratch instead
  const size_t nodeBytes = orb_k_octree_lds(nodeCapMax, maxCellsPerLevel, 0);
  const size_t budget = (size_t)ORB_OCTREE_LDS_KB * 1024;
  // node tables beyond 128 KiB (nfeatures above ~7,500 at 1.2 / 8 levels) go
  // to a global scratch slice per (image, level); the LDS then holds keys only
  const bool octGlobal = nodeBytes > 128 * 1024;
  const size_t ldsNodes = octGlobal ? 0 : nodeBytes;
  int ldsKeyCap = ldsNodes < budget ? (int)((budget - ldsNodes) / 6) : 0;
  ldsKeyCap &= ~7;
  if (ldsNodes + (size_t)ldsKeyCap * 6 > 160 * 1024) return ORB_EINVAL;

  hipSetDevice(h->device);
  // the tables below are read by the previous call's kernels, which may still
  // run on another stream (CallOrder): the uploads wait for that call
  if (must_wait(h->lastStream, h->stream)) HIP_TRY(hipStreamWaitEvent(h->stream, h->evBatch, 0));
  orb_status_t st = h->dCells.ensure(cells.size() * sizeof(OrbCellDesc));
  if (st) return st;
  st = h->dRtab.ensure(std::max<size_t>(rtab.size(), 1) * 4);
  if (st) return st;
  st = h->dTiles.ensure(tiles.size() * sizeof(OrbTileDesc));
  if (st) return st;
  st = h->dBands.ensure(bands.size() * sizeof(OrbBandDesc));
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(h->dBands.p, bands.data(), bands.size() * sizeof(OrbBandDesc),
                         hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(h->dTiles.p, tiles.data(), tiles.size() * sizeof(OrbTileDesc),
                         hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(h->dCells.p, cells.data(), cells.size() * sizeof(OrbCellDesc),
                         hipMemcpyHostToDevice, h->stream));
  if (!rtab.empty())
    HIP_TRY(hipMemcpyAsync(h->dRtab.p, rtab.data(), rtab.size() * 4, hipMemcpyHostToDevice,
                           h->stream));
  HIP_TRY(stream_wait(h->stream));
  h->lastStream = nullptr;  // the previous call has finished (waited for above)
  h->plan = P;
  h->cells.swap(cells);
  h->arenaBytes = (arena + 255) & ~255LL;
  h->blurBytes = (blurArena + 255) & ~255LL;
  h->maxCellsPerLevel = maxCellsPerLevel;
  h->nodeCapMax = nodeCapMax;
  h->ldsKeyCap = ldsKeyCap;
  h->octNodeBytes = octGlobal ? (long long)((nodeBytes + 255) & ~(size_t)255) : 0;
  h->planW = W;
  h->planH = H;
  h->nResizePairs = nResize;
  h->prof.launchesPerCall[0] = nResize;
  h->batchCap = 0;  // scratch layout depends on the plan
  return ORB_OK;
}

static orb_status_t ensure_batch(orb_extractor* h, int B) {
  if (B <= h->batchCap) return ORB_OK;
  const OrbPlanDesc& P = h->plan;
  const size_t cellSlots = (size_t)B * P.ncells * P.keyCap;
  orb_status_t st;
  if ((st = h->dArena.ensure((size_t)B * h->arenaBytes))) return st;
  if ((st = h->dCellKeys.ensure(cellSlots * 4))) return st;
  if ((st = h->dGKeys.ensure(cellSlots * 4))) return st;
  if ((st = h->dGNid.ensure(cellSlots * 2))) return st;
  if ((st = h->dCellCount.ensure((size_t)B * P.ncells * 4))) return st;
  if ((st = h->dOutKeys.ensure((size_t)B * P.slotsPerImage * 4))) return st;
  if ((st = h->dOutCount.ensure((size_t)B * P.nlevels * 4))) return st;
  if ((st = h->dErr.ensure((size_t)B * 4))) return st;
  if (h->octNodeBytes &&
      (st = h->dOctNodes.ensure((size_t)B * P.nlevels * (size_t)h->octNodeBytes)))
    return st;
  h->batchCap = B;
  return ORB_OK;
}

static int stream_prio(bool least);
// The shared side streams (shared_side_stream below) are destroyed by an exit
// handler; run_batch holds g_sideUse shared while it enqueues, and a call that
// starts after the release fails with ORB_EDEVICE instead of launching on a
// destroyed stream (e.g. from a thread still running at exit).
static std::shared_mutex g_sideUse;
static bool g_sideReleased = false;

// Schedule constants of run_batch (compile-time A/B: tools/build_variant.sh)
#ifndef FAST_CELLS_MIN_BATCH
#define FAST_CELLS_MIN_BATCH 4  // smaller calls take k_fast_band on one stream
#endif
#ifndef FAST_SIDE_LEVELS
// levels 1..FAST_SIDE_LEVELS follow level 0 on the side stream: extraction
// alone 1.770 / 1.723 / 1.708 / 1.709 ms per 512 frames for 0 / 1 / 2 / 3,
// bench 259.7k / 262.3k / 263.6k / 263.4k frames/s (profiles/r03_schedule_xcd.txt)
#define FAST_SIDE_LEVELS 2
#endif
#ifndef FAST_L0_INLINE
#define FAST_L0_INLINE 0  // 1: level 0's FAST on the caller's stream (one dispatch; PMC passes)
#endif

static orb_status_t run_batch(orb_extractor* h, const uint8_t* d_images, int B, size_t stride,
                              size_t imgPitch, orb_keypoint_t* d_kps, uint8_t* d_desc,
                              int capacity, int32_t* d_counts, hipStream_t s,
                              bool capturing = false) {
  // Stage chain: pyramid -> FAST -> octree -> orient + blur + descriptors
  // (k_orient_desc blurs each keypoint's window in LDS).
  const OrbPlanDesc& P = h->plan;
  const int32_t* rt = h->dRtab.as<int32_t>();
  uint8_t* arena = h->dArena.as<uint8_t>();
  const long long ap = h->arenaBytes;
  // the side stream: the device's shared one, or -- while the caller's stream
  // is being captured into a graph -- a stream of this handle's own, so a
  // capture never pulls another handle's side work into its graph
  std::shared_lock<std::shared_mutex> sideUse(g_sideUse);
  if (g_sideReleased) return ORB_EDEVICE;  // process exit has begun
  hipStream_t side = h->stream2;
  capturing = capturing || stream_capturing(s);
  {
    if (capturing) {
      if (!h->privSide &&
          hipStreamCreateWithPriority(&h->privSide, hipStreamNonBlocking, stream_prio(true)) != hipSuccess) {
        h->privSide = nullptr;
        return ORB_EDEVICE;
      }
      side = h->privSide;
    }
  }
  StageProfiler& pf = h->prof;
  std::vector<hipEvent_t>* ev = pf.begin_call();
  PROF_REC(ev, pf.t0(ev), s);
  // the FAST kernels clear each image's status flag (one launch fewer per call);
  // a plan without cells launches no FAST kernel
  if (P.ncells == 0) HIP_TRY(hipMemsetAsync(h->dErr.p, 0, (size_t)B * 4, s));
  // k_fast_cells (one wave per cell) unless a tiny level's cells outgrow its
  // staging; k_fast_band (one workgroup per run of cells) otherwise and for a
  // frame or two per call (the band kernel's fewer, larger workgroups and a
  // single stream give the lower latency)
  const bool useBands = B < FAST_CELLS_MIN_BATCH || !orb_k_fast_cells_fits(&P);
  pf.names[2] = useBands ? "k_fast_band" : "k_fast_cells";
  // k_fast_cells over the cells [cb, ce) (whole levels) on stream st
  auto fast = [&](int cb, int ce, hipStream_t st) -> hipError_t {
    return orb_k_fast_cells(d_images, (long long)imgPitch, (int)stride, arena, ap, &P,
                            h->dCells.as<OrbCellDesc>(), h->dCellKeys.as<uint32_t>(),
                            h->dCellCount.as<int32_t>(), h->dErr.as<int32_t>(), cb, ce, B, st);
  };
  // Level 0 is the caller's image: its FAST cells need no pyramid, so they run
  // on the side stream beside the latency-bound resize chain (fork / join by
  // events, graph-capturable).  Levels 1..sideLevels follow on the side stream
  // in one launch once the chain has written level sideLevels; the rest follow
  // the chain on the main stream.  (Measured and not kept: every level on the
  // side stream as the chain writes it, 255k vs 260k frames/s, the chain losing
  // its CUs to FAST, profiles/r03_fast_schedule.txt; the octree and descriptors
  // of the side levels on the side stream too, round 4.)
  const int l0End = P.lv[0].cellEnd;
  // (profile mode 2 times each stage alone: no side stream)
  const bool l0Side = !useBands && !FAST_L0_INLINE && !(ev && pf.serial) && l0End > 0 && P.nlevels > 1;
  const int sideLevels = l0Side ? std::min(FAST_SIDE_LEVELS, P.nlevels - 1) : 0;
  const int sideEnd = sideLevels > 0 ? P.lv[sideLevels].cellEnd : l0End;
  if (l0Side) {
    HIP_TRY(hipEventRecord(h->evL0Fork, s));
    HIP_TRY(hipStreamWaitEvent(side, h->evL0Fork, 0));
    PROF_REC(ev, pf.b(ev, 5), side);
    HIP_TRY(fast(0, l0End, side));
    PROF_REC(ev, pf.e(ev, 5), side);
    if (sideLevels == 0) HIP_TRY(hipEventRecord(h->evL0Join, side));
  } else if (ev) {
    pf.not_run(5);
  }
  // the resize chain on the caller's stream (one launch per level: the
  // one-launch chain k_pyr_chain measured slower, 0.0386 vs 0.0269 ms per
  // frame, profiles/r04_step11.txt)
  PROF_REC(ev, pf.b(ev, 0), s);
  const bool pairs = B <= PYR_PAIR_MAX_IMAGES;
  h->prof.launchesPerCall[0] = pairs ? h->nResizePairs : P.nlevels - 1;
  for (int l = 1; l < P.nlevels; ++l) {
    const OrbLevelDesc& d = P.lv[l];
    const OrbLevelDesc& sd = P.lv[l - 1];
    const uint8_t* src = l == 1 ? d_images : arena + sd.arenaOff;
    const long long srcPitch = l == 1 ? (long long)imgPitch : ap;
    const int srcStride = l == 1 ? (int)stride : sd.pitch;
    const bool pair = pairs && d.resize2;
    const int top = pair ? l + 1 : l;  // last level this launch writes
    if (pair) {
      const OrbLevelDesc& e = P.lv[l + 1];
      HIP_TRY(orb_k_pyr_resize2(src, srcPitch, srcStride, sd.w, sd.h, arena + d.arenaOff, ap, d.pitch,
                                d.w, d.h, rt + d.rtabX, rt + d.rtabX + d.w, rt + d.rtabY,
                                rt + d.rtabY + d.h, arena + e.arenaOff, ap, e.pitch, e.w, e.h,
                                rt + e.rtabX, rt + e.rtabX + e.w, rt + e.rtabY, rt + e.rtabY + e.h,
                                B, s));
    } else {
      HIP_TRY(orb_k_pyr_resize(src, srcPitch, srcStride, sd.w, sd.h, arena + d.arenaOff, ap, d.pitch,
                               d.w, d.h, rt + d.rtabX, rt + d.rtabX + d.w, rt + d.rtabY,
                               rt + d.rtabY + d.h, d.resizeMode, B, s));
    }
    l = top;
    if (l >= sideLevels && l - (pair ? 1 : 0) <= sideLevels) {  // this launch wrote level sideLevels
      if (sideEnd > l0End) {
        HIP_TRY(hipEventRecord(h->evLvl, s));
        HIP_TRY(hipStreamWaitEvent(side, h->evLvl, 0));
        PROF_REC(ev, pf.b(ev, 5, 1), side);
        HIP_TRY(fast(l0End, sideEnd, side));
        PROF_REC(ev, pf.e(ev, 5, 1), side);
        if (ev) pf.segments(5, 2);
      }
      HIP_TRY(hipEventRecord(h->evL0Join, side));
    }
  }
  PROF_REC(ev, pf.e(ev, 0), s);
  PROF_REC(ev, pf.b(ev, 2), s);
  if (useBands)
    HIP_TRY(orb_k_fast_band(d_images, (long long)imgPitch, (int)stride, arena, ap, &P,
                            h->dBands.as<OrbBandDesc>(), P.nBands, h->dCells.as<OrbCellDesc>(),
                            h->dCellKeys.as<uint32_t>(), h->dCellCount.as<int32_t>(),
                            h->dErr.as<int32_t>(), B, s));
  else
    HIP_TRY(fast(l0Side ? sideEnd : 0, P.ncells, s));
  PROF_REC(ev, pf.e(ev, 2), s);
  // (level 0's octree on the side stream as well measured no gain: the octree's
  // time is its per-workgroup pass latency, not level 0's size)
  if (l0Side) HIP_TRY(hipStreamWaitEvent(s, h->evL0Join, 0));
  PROF_REC(ev, pf.b(ev, 3), s);
  HIP_TRY(orb_k_octree(&P, h->dCellCount.as<int32_t>(), h->dCellKeys.as<uint32_t>(),
                       h->dGKeys.as<uint32_t>(), h->dGNid.as<uint16_t>(), h->ldsKeyCap,
                       h->nodeCapMax, h->maxCellsPerLevel, h->dOutKeys.as<uint32_t>(),
                       h->dOutCount.as<int32_t>(), h->dErr.as<int32_t>(), 0, P.nlevels, B,
                       h->octNodeBytes ? h->dOctNodes.as<uint8_t>() : nullptr, h->octNodeBytes, s));
  PROF_REC(ev, pf.e(ev, 3), s);
  PROF_REC(ev, pf.b(ev, 4), s);
  HIP_TRY(orb_k_orient_desc(d_images, (long long)imgPitch, (int)stride, arena, ap, &P,
                            h->dOutKeys.as<uint32_t>(), h->dOutCount.as<int32_t>(),
                            h->dErr.as<int32_t>(), d_kps, d_desc, capacity, d_counts, B, 0,
                            P.nlevels, s));
  PROF_REC(ev, pf.e(ev, 4), s);
  PROF_REC(ev, pf.t1(ev), s);
  if (!capturing) {  // readbacks and the next call on another stream wait for it (CallOrder)
    HIP_TRY(hipEventRecord(h->evBatch, s));
    h->lastStream = s;
  }
  h->lastImg0 = d_images;
  h->lastImg0Pitch = imgPitch;
  h->lastImg0Stride = (int)stride;
  return ORB_OK;
}

extern "C" {

int orb_abi_version(void) { return ORB_ABI_VERSION; }

const char* orb_status_string(orb_status_t s) {
  switch (s) {
    case ORB_OK: return "ok";
    case ORB_EEMPTY: return "empty input";
    case ORB_EINVAL: return "invalid argument";
    case ORB_ENOMEM: return "device out of memory";
    case ORB_EDEVICE: return "HIP device error";
    case ORB_ECAPACITY: return "buffer too small";
    case ORB_ENODEV: return "no gfx950 device";
  }
  return "unknown";
}

orb_status_t orb_device_count(int* n) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  if (n) *n = c;
  return c > 0 ? ORB_OK : ORB_ENODEV;
}

// Stream priorities: the least (least == true) or the normal stream priority of
// the device; SIDE_PRIO (compile-time A/B: 0 least, 1 normal, 2 greatest) picks
// the "least" one for the pooled side stream of a SIDE_CUMASK=0 build and for
// the handles' own streams.
#ifndef SIDE_PRIO
#define SIDE_PRIO 0
#endif
static int stream_prio(bool least) {
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (!least) return 0;
  return SIDE_PRIO == 0 ? lo : SIDE_PRIO == 1 ? 0 : hi;
}
// One side stream per device, shared by every extractor handle of the process.
// Each stream holds an HSA queue, and a process with more queues than the
// hardware maps at once (the bench with its C3 / C5 handles: 11, with one
// side stream per handle) saw the side stream's cross-queue fork / join slow
// its extraction by 30-50 % whenever a matcher ran beside it
// (profiles/r03_streams.txt).  Handles on one device share it safely: fork /
// join are per-handle events.
#ifndef SIDE_CUMASK
#define SIDE_CUMASK 1  // the side stream on an HSA queue of its own (a full-CU-mask stream)
#endif
static std::mutex g_sideMu;
static hipStream_t g_side[64] = {};
// The side streams are released by the process's exit handlers before the HIP
// runtime's own teardown: a CU-masked stream left to that teardown crashed the
// process at exit under rocprofv3 --kernel-trace (SIGSEGV in __cxa_finalize,
// after the profiler's finalisation; profiles/r05_exit_crash.txt).
static void release_side_streams() {
  std::unique_lock<std::shared_mutex> u(g_sideUse);  // no run_batch is enqueueing
  std::lock_guard<std::mutex> g(g_sideMu);
  g_sideReleased = true;
  for (hipStream_t& st : g_side)
    if (st) {
      hipStreamDestroy(st);  // waits for the stream's work
      st = nullptr;
    }
}
static hipStream_t shared_side_stream(int device, int prio) {
  hipStream_t* s = g_side;
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> g(g_sideMu);
  static bool registered = false;
#ifndef SIDE_RELEASE_AT_EXIT
#define SIDE_RELEASE_AT_EXIT 1  // 0: leave the side streams to the runtime's teardown (the test's negative control)
#endif
  if (SIDE_RELEASE_AT_EXIT && !registered) registered = std::atexit(release_side_streams) == 0;
  if (!s[device]) {
    hipError_t e;
    if (SIDE_CUMASK) {
      // HIP gives a CU-masked stream an HSA queue of its own instead of a
      // pooled one: a mask of every CU of the device
      hipDeviceProp_t prop;
      e = hipGetDeviceProperties(&prop, device);
      if (e == hipSuccess) {
        std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0u);
        for (int c = 0; c < prop.multiProcessorCount; ++c) mask[c >> 5] |= 1u << (c & 31);
        e = hipExtStreamCreateWithCUMask(&s[device], (uint32_t)mask.size(), mask.data());
      }
    } else {
      e = hipStreamCreateWithPriority(&s[device], hipStreamNonBlocking, prio);
    }
    if (e != hipSuccess) s[device] = nullptr;
  }
  return s[device];  // until exit
}

// A handle's own stream (single-frame calls, host-buffer matchers, readbacks,
// graph capture) at the device's least priority.  HIP backs the streams of a
// process by a few HSA queues per priority level and maps a new stream onto
// the least-used queue of its level; normal-priority streams a library
// creates early (ORB-SLAM2 builds its extractors and matchers at start-up)
// take normal queues the caller's own streams then share: a caller's
// high-priority stream ran 2x slower beside busy normal-priority streams
// after three idle normal streams had been created first, with or without
// this library (tools/probe/contention_probe.py, profiles/r05_contention.txt).
// The least priority keeps the library out of the pools the caller's streams
// use (the side stream has a queue of its own, SIDE_CUMASK).
#ifndef OWN_PRIO
#define OWN_PRIO 0  // handles' own streams: 0 least priority, 1 normal (compile-time A/B)
#endif
static hipError_t create_own_stream(hipStream_t* s) {
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, OWN_PRIO ? 0 : stream_prio(true));
}

static bool create_side_streams(orb_extractor* h) {
  // The side stream must not share an HSA queue with the caller's stream: two
  // streams on one queue run in submission order, which would serialise level
  // 0's FAST with the resize chain.  It is a full-CU-mask stream (a queue of
  // its own, round 5); a SIDE_CUMASK=0 build takes a least-priority pooled
  // stream instead (round 3: the chain on the caller's stream then wins the
  // CUs the side FAST also wants, extraction 1.703 vs 1.727 ms per 512
  // frames; profiles/r03_streams.txt)
  h->stream2 = shared_side_stream(h->device, stream_prio(true));
  return h->stream2 != nullptr;
}

orb_status_t orb_extractor_create(int nfeatures, float scale_factor, int nlevels, int ini_th_fast,
                                  int min_th_fast, int device, orb_extractor_t** out) {
  if (!out) return ORB_EINVAL;
  *out = nullptr;
  // (a scale factor of 1 makes the reference's quota series 0 / 0,
  // src/ORBextractor.cc:453-455; the per-level node bound is the planner's)
  if (nfeatures < 0 || nlevels < 1 || nlevels > ORB_MAX_LEVELS || !(scale_factor > 1.0f) ||
      !std::isfinite(scale_factor))
    return ORB_EINVAL;
  orb_status_t st = check_device(device);
  if (st) return st;
  orb_extractor* h = new orb_extractor();
  h->device = device;
  h->nfeatures = nfeatures;
  h->scaleFactorF = scale_factor;
  h->scaleFactor = (double)scale_factor;
  h->nlevels = nlevels;
  h->iniTh = ini_th_fast;
  h->minTh = min_th_fast;
  compute_tables(h);
  hipSetDevice(device);
  if (create_own_stream(&h->stream) != hipSuccess ||
      !create_side_streams(h) ||
      hipEventCreateWithFlags(&h->evL0Fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->evL0Join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->evLvl, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->evBatch, hipEventDisableTiming) != hipSuccess) {
    if (h->stream) hipStreamDestroy(h->stream);
    if (h->evL0Fork) hipEventDestroy(h->evL0Fork);
    if (h->evL0Join) hipEventDestroy(h->evL0Join);
    if (h->evLvl) hipEventDestroy(h->evLvl);
    if (h->evBatch) hipEventDestroy(h->evBatch);
    delete h;
    return ORB_EDEVICE;
  }
  h->ownStream = true;
  h->prof.nStages = 6;
  h->prof.maxSeg[5] = 2;  // side-stream FAST: level 0, then levels 1..FAST_SIDE_LEVELS
  const char* names[6] = {"k_pyr_resize", "k_blur_levels", "k_fast_band", "k_octree",
                          "k_orient_desc", "k_fast_cells_side"};
  for (int i = 0; i < 6; ++i) {
    h->prof.names[i] = names[i];
    h->prof.launchesPerCall[i] = 1;
  }
  h->prof.launchesPerCall[0] = std::max(nlevels - 1, 0);
  h->prof.launchesPerCall[1] = 0;  // k_blur_levels: orb_extractor_blurred_level only
  if (orb_k_upload_constants(h->stream) != hipSuccess ||
      orb_k_upload_umax(h->umax, h->stream) != hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess) {
    orb_extractor_destroy(h);
    return ORB_EDEVICE;
  }
  *out = h;
  return ORB_OK;
}

void orb_extractor_destroy(orb_extractor_t* h) {
  if (!h) return;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->lastStream) hipEventSynchronize(h->evBatch);  // a batch call on a caller's stream
  DevBuf* bufs[] = {&h->dCells, &h->dRtab, &h->dTiles, &h->dBlur, &h->dArena, &h->dCellKeys, &h->dCellCount, &h->dOctNodes,
                    &h->dGKeys, &h->dGNid, &h->dOutKeys, &h->dOutCount, &h->dErr,
                    &h->dImg, &h->dOne};
  for (DevBuf* b : bufs) b->release();
  h->hImg.release();
  h->hOut.release();
  h->hLvl.release();
  h->hPyr.release();
  if (h->oneExec) hipGraphExecDestroy(h->oneExec);
  h->prof.destroy();
  if (h->ownStream && h->stream) hipStreamDestroy(h->stream);
  if (h->privSide) hipStreamDestroy(h->privSide);
  if (h->evL0Fork) hipEventDestroy(h->evL0Fork);
  if (h->evL0Join) hipEventDestroy(h->evL0Join);
  if (h->evLvl) hipEventDestroy(h->evLvl);
  if (h->evBatch) hipEventDestroy(h->evBatch);
  delete h;
}

int orb_extractor_get_levels(const orb_extractor_t* h) { return h ? h->nlevels : 0; }
float orb_extractor_get_scale_factor(const orb_extractor_t* h) { return h ? (float)h->scaleFactor : 0.f; }
void orb_extractor_get_scale_factors(const orb_extractor_t* h, float* o) {
  if (h && o) std::copy(h->scale.begin(), h->scale.end(), o);
}
void orb_extractor_get_inverse_scale_factors(const orb_extractor_t* h, float* o) {
  if (h && o) std::copy(h->invScale.begin(), h->invScale.end(), o);
}
void orb_extractor_get_scale_sigma_squares(const orb_extractor_t* h, float* o) {
  if (h && o) std::copy(h->sigma2.begin(), h->sigma2.end(), o);
}
void orb_extractor_get_inverse_scale_sigma_squares(const orb_extractor_t* h, float* o) {
  if (h && o) std::copy(h->invSigma2.begin(), h->invSigma2.end(), o);
}
void orb_extractor_get_features_per_level(const orb_extractor_t* h, int32_t* o) {
  if (h && o) std::copy(h->quota.begin(), h->quota.end(), o);
}

int orb_extractor_capacity(const orb_extractor_t* hc, int width, int height) {
  orb_extractor* h = const_cast<orb_extractor*>(hc);
  if (!h) return -1;
  std::lock_guard<std::mutex> g(h->mu);
  if (build_plan(h, width, height) != ORB_OK) return -1;
  return h->plan.slotsPerImage;
}

void* orb_extractor_stream(orb_extractor_t* h) { return h ? (void*)h->stream : nullptr; }

orb_status_t orb_extractor_extract_batch(orb_extractor_t* h, const uint8_t* d_images,
                                         int n_images, int width, int height, size_t stride,
                                         size_t image_pitch, orb_keypoint_t* d_keypoints,
                                         uint8_t* d_descriptors, int capacity,
                                         int32_t* d_counts, void* stream) {
  if (!h || !d_images || !d_keypoints || !d_descriptors || !d_counts) return ORB_EINVAL;
  if (n_images <= 0 || width <= 0 || height <= 0) return ORB_EEMPTY;
  if (stride < (size_t)width || image_pitch < stride * (size_t)height) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  hipSetDevice(h->device);
  orb_status_t st = build_plan(h, width, height);
  if (st) return st;
  if (capacity < h->plan.slotsPerImage) return ORB_ECAPACITY;
  if ((st = ensure_batch(h, n_images))) return st;
  hipStream_t s = stream ? (hipStream_t)stream : h->stream;
  // the previous call may still run on another stream: its scratch is this
  // call's scratch (CallOrder)
  if (must_wait(h->lastStream, s) && !stream_capturing(s))
    HIP_TRY(hipStreamWaitEvent(s, h->evBatch, 0));
  st = run_batch(h, d_images, n_images, stride, image_pitch, d_keypoints, d_descriptors, capacity,
                 d_counts, s);
  if (st) return st;
  h->lastSingle = false;
  h->lastW = width;
  h->lastH = height;
  return ORB_OK;
}

// Row pitch of the one-frame path's staged image (pinned and device): the
// width itself (the kernels take any stride), so a contiguous caller image is
// staged with one memcpy instead of one per row
#ifndef ONE_PITCH_ALIGN
#define ONE_PITCH_ALIGN 1  // (A/B knob: 64 = rows padded to 64 bytes)
#endif
static size_t one_stride(int width) {
  return ((size_t)width + ONE_PITCH_ALIGN - 1) / ONE_PITCH_ALIGN * ONE_PITCH_ALIGN;
}

orb_status_t orb_extractor_extract(orb_extractor_t* h, const uint8_t* image, int width,
                                   int height, size_t stride, orb_keypoint_t* keypoints,
                                   uint8_t* descriptors, int capacity, int* n_keypoints) {
  if (!h) return ORB_EINVAL;
  if (!image || width <= 0 || height <= 0) return ORB_EEMPTY;  // src/ORBextractor.cc:1095-1096
  if (stride < (size_t)width || !n_keypoints) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  hipSetDevice(h->device);
  orb_status_t st = build_plan(h, width, height);
  if (st) return st;
  const int cap = h->plan.slotsPerImage;
  const size_t dstride = one_stride(width);
  const size_t pitch = dstride * height;
  const size_t pitch16 = (pitch + 15) & ~(size_t)15;  // k_copy_pinned moves 16-byte words
  const size_t kOff = 16, dOff = kOff + (size_t)cap * sizeof(orb_keypoint_t);
  const size_t outBytes = dOff + (size_t)cap * 32;
  if ((st = ensure_batch(h, 1))) return st;
  if ((st = h->dImg.ensure(pitch16))) return st;
  if ((st = h->dOne.ensure(outBytes))) return st;
  if ((st = h->hImg.ensure(pitch16))) return st;
  if ((st = h->hOut.ensure(outBytes))) return st;
  if (h->pyrReadback && (st = h->hPyr.ensure((size_t)std::max<long long>(h->arenaBytes, 1)))) return st;
  h->hPyrValid = false;
  // a batch call may still run on a caller's stream (CallOrder)
  if (must_wait(h->lastStream, h->stream)) HIP_TRY(hipStreamWaitEvent(h->stream, h->evBatch, 0));
  // image -> pinned staging at the device row pitch
  if (stride == dstride)
    memcpy(h->hImg.p, image, pitch);
  else
    for (int y = 0; y < height; ++y)
      memcpy(h->hImg.as<uint8_t>() + (size_t)y * dstride, image + (size_t)y * stride, (size_t)width);
  uint8_t* d1 = h->dOne.as<uint8_t>();
  // one DMA in, the extraction, one DMA out of the count and every record slot
  auto upload = [&]() -> orb_status_t {
    HIP_TRY(orb_k_copy_pinned(h->dImg.p, h->hImg.p, pitch16, h->stream));
    return ORB_OK;
  };
  auto enqueue = [&](bool capturing) -> orb_status_t {
    orb_status_t r = run_batch(h, h->dImg.as<uint8_t>(), 1, dstride, pitch,
                               reinterpret_cast<orb_keypoint_t*>(d1 + kOff), d1 + dOff, cap,
                               reinterpret_cast<int32_t*>(d1), h->stream, capturing);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(h->hOut.p, d1, outBytes, hipMemcpyDeviceToHost, h->stream));
    if (h->pyrReadback && h->arenaBytes > 0)  // levels 1.. for the host mirror, one DMA
      HIP_TRY(hipMemcpyAsync(h->hPyr.p, h->dArena.p, (size_t)h->arenaBytes, hipMemcpyDeviceToHost,
                             h->stream));
    return ORB_OK;
  };
  if (h->prof.enabled) {  // (the stage events need the launches issued one by one)
    if ((st = upload()) || (st = enqueue(false))) return st;
  } else {
    // the DMA in goes out before the graph, not as its first node: it runs
    // while hipGraphLaunch is still being processed on the host (~20 us of
    // host time before a graph's first node starts on the GPU,
    // profiles/r06_dropin_timeline.txt)
    if ((st = upload())) return st;
    const std::vector<const void*> key = {
        h->dImg.p, h->dOne.p, h->hImg.p, h->hOut.p, h->dArena.p, h->dCellKeys.p, h->dGKeys.p,
        h->dGNid.p, h->dCellCount.p, h->dOutKeys.p, h->dOutCount.p, h->dErr.p, h->dRtab.p,
        h->dBands.p, h->dCells.p, h->dBlur.p, h->dTiles.p, h->dOctNodes.p,
        h->pyrReadback ? h->hPyr.p : nullptr, (const void*)(intptr_t)width,
        (const void*)(intptr_t)height, (const void*)(intptr_t)cap};
    if (!h->oneExec || key != h->oneKey) {
      if (h->oneExec) hipGraphExecDestroy(h->oneExec);
      h->oneExec = nullptr;
      hipGraph_t graph = nullptr;
      HIP_TRY(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
      st = enqueue(true);
      hipError_t ce = hipStreamEndCapture(h->stream, &graph);
      if (st) {
        if (graph) hipGraphDestroy(graph);
        return st;
      }
      if (ce != hipSuccess) return ORB_EDEVICE;
      hipError_t ie = hipGraphInstantiate(&h->oneExec, graph, nullptr, nullptr, 0);
      hipGraphDestroy(graph);
      if (ie != hipSuccess) {
        h->oneExec = nullptr;
        return ORB_EDEVICE;
      }
      h->oneKey = key;
    }
    HIP_TRY(hipGraphLaunch(h->oneExec, h->stream));
    HIP_TRY(hipEventRecord(h->evBatch, h->stream));
    // a replayed graph skips run_batch's bookkeeping: level 0 of this call is
    // the staged image again, not whatever an intervening batch call pointed at
    h->lastImg0 = h->dImg.as<uint8_t>();
    h->lastImg0Pitch = pitch;
    h->lastImg0Stride = (int)dstride;
  }
  HIP_TRY(stream_wait(h->stream));
  h->lastStream = nullptr;  // nothing of this handle is pending
  h->oneCap = cap;
  h->lastSingle = true;
  h->hPyrValid = h->pyrReadback;
  const uint8_t* ho = h->hOut.as<uint8_t>();
  int32_t n = 0;
  memcpy(&n, ho, 4);
  h->lastW = width;
  h->lastH = height;
  // a negative count: the octree hit an internal limit (never at ORB-SLAM2 settings)
  if (n < 0) return ORB_EDEVICE;
  *n_keypoints = n;
  if (n > capacity) return ORB_ECAPACITY;
  if (n > 0) {
    memcpy(keypoints, ho + kOff, (size_t)n * sizeof(orb_keypoint_t));
    if (descriptors) memcpy(descriptors, ho + dOff, (size_t)n * 32);
  }
  return ORB_OK;
}

orb_status_t orb_extractor_batch_level(orb_extractor_t* h, int image, int level,
                                       const uint8_t** d_level, int* width, int* height,
                                       size_t* stride) {
  if (!h || level < 0 || level >= h->nlevels || h->planW < 0 || !h->lastImg0) return ORB_EINVAL;
  if (image < 0 || image >= h->batchCap) return ORB_EINVAL;
  const OrbLevelDesc& d = h->plan.lv[level];
  if (width) *width = d.w;
  if (height) *height = d.h;
  if (level == 0) {
    if (d_level) *d_level = h->lastImg0 + (size_t)image * h->lastImg0Pitch;
    if (stride) *stride = (size_t)h->lastImg0Stride;
  } else {
    if (d_level) *d_level = h->dArena.as<uint8_t>() + (size_t)image * h->arenaBytes + d.arenaOff;
    if (stride) *stride = (size_t)d.pitch;
  }
  return ORB_OK;
}

// Device level -> caller's host rows through the pinned staging block: a 2-D
// copy straight into pageable memory goes row by row.
static orb_status_t copy_level_to_host(orb_extractor_t* h, uint8_t* dst, size_t dst_stride,
                                       const uint8_t* src, size_t src_stride, int w, int hh) {
  orb_status_t st = h->hLvl.ensure((size_t)w * hh);
  if (st) return st;
  uint8_t* ho = h->hLvl.as<uint8_t>();
  HIP_TRY(hipMemcpy2DAsync(ho, (size_t)w, src, src_stride, (size_t)w, hh, hipMemcpyDeviceToHost,
                           h->stream));
  HIP_TRY(stream_wait(h->stream));
  for (int y = 0; y < hh; ++y) memcpy(dst + (size_t)y * dst_stride, ho + (size_t)y * w, (size_t)w);
  return ORB_OK;
}

orb_status_t orb_extractor_pyramid_level(orb_extractor_t* h, int level, uint8_t* dst,
                                         size_t dst_stride, int* width, int* height) {
  if (!h) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  const uint8_t* src = nullptr;
  int w = 0, hh = 0;
  size_t sstride = 0;
  orb_status_t st = orb_extractor_batch_level(h, 0, level, &src, &w, &hh, &sstride);
  if (st) return st;
  if (width) *width = w;
  if (height) *height = hh;
  if (!dst) return ORB_OK;
  if (dst_stride < (size_t)w) return ORB_EINVAL;
  hipSetDevice(h->device);
  HIP_TRY(hipStreamWaitEvent(h->stream, h->evBatch, 0));  // the batch may have run on a caller stream
  return copy_level_to_host(h, dst, dst_stride, src, sstride, w, hh);
}

orb_status_t orb_extractor_host_pyramid(orb_extractor_t* h, int level, const uint8_t** data,
                                        int* width, int* height, size_t* stride) {
  if (!h || !data) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  if (!h->lastSingle || level < 0 || level >= h->nlevels || h->planW < 0) return ORB_EINVAL;
  const OrbLevelDesc& d = h->plan.lv[level];
  if (width) *width = d.w;
  if (height) *height = d.h;
  if (level == 0) {  // the call's own pinned staging of the image
    *data = h->hImg.as<uint8_t>();
    if (stride) *stride = one_stride(d.w);
    return ORB_OK;
  }
  if (!h->hPyrValid) {
    // first request: this call's levels now (one DMA), every later call's in
    // its graph
    hipSetDevice(h->device);
    orb_status_t st = h->hPyr.ensure((size_t)std::max<long long>(h->arenaBytes, 1));
    if (st) return st;
    HIP_TRY(hipStreamWaitEvent(h->stream, h->evBatch, 0));
    HIP_TRY(hipMemcpyAsync(h->hPyr.p, h->dArena.p, (size_t)h->arenaBytes, hipMemcpyDeviceToHost,
                           h->stream));
    HIP_TRY(stream_wait(h->stream));
    h->pyrReadback = true;
    h->hPyrValid = true;
  }
  *data = h->hPyr.as<uint8_t>() + d.arenaOff;
  if (stride) *stride = (size_t)d.pitch;
  return ORB_OK;
}

orb_status_t orb_extractor_host_pyramid_off(orb_extractor_t* h) {
  if (!h) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  // the next single-frame call re-keys its graph without the pyramid DMA
  // (pyrReadback is part of the graph key); the mirror buffer is kept
  h->pyrReadback = false;
  h->hPyrValid = false;
  return ORB_OK;
}

orb_status_t orb_extractor_blurred_level(orb_extractor_t* h, int level, uint8_t* dst,
                                         size_t dst_stride, int* width, int* height) {
  if (!h) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  if (h->planW < 0 || h->batchCap <= 0 || level < 0 || level >= h->plan.nlevels) return ORB_EINVAL;
  const OrbLevelDesc& L = h->plan.lv[level];
  if (width) *width = L.w;
  if (height) *height = L.h;
  if (!dst) return ORB_OK;
  if (dst_stride < (size_t)L.w) return ORB_EINVAL;
  hipSetDevice(h->device);
  // The extraction never materialises blurred levels (k_orient_desc blurs
  // each keypoint's window in LDS): blur image 0 of the last call on demand
  // with k_blur_levels.
  HIP_TRY(hipStreamWaitEvent(h->stream, h->evBatch, 0));
  if (!h->lastImg0) return ORB_EINVAL;
  orb_status_t st = h->dBlur.ensure((size_t)h->blurBytes);
  if (st) return st;
  HIP_TRY(orb_k_blur_levels(h->lastImg0, (long long)h->lastImg0Pitch, h->lastImg0Stride,
                            h->dArena.as<uint8_t>(), h->arenaBytes, &h->plan,
                            h->dTiles.as<OrbTileDesc>(), h->dBlur.as<uint8_t>(), h->blurBytes, 1,
                            h->stream));
  return copy_level_to_host(h, dst, dst_stride, h->dBlur.as<uint8_t>() + L.blurOff, L.blurPitch,
                            L.w, L.h);
}

orb_status_t orb_extractor_profile(orb_extractor_t* h, int enable) {
  if (!h) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  hipSetDevice(h->device);
  h->prof.drain();
  h->prof.reset();
  h->prof.enabled = enable != 0;
  h->prof.serial = enable == 2;
  return ORB_OK;
}

// stage 0..5 = kernels, stage 6 = whole extraction call
orb_status_t orb_extractor_profile_read(orb_extractor_t* h, int stage, double* total_ms,
                                        int* launches, const char** name) {
  if (!h || stage < 0 || stage > h->prof.nStages) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  hipSetDevice(h->device);
  h->prof.drain();
  if (total_ms) *total_ms = h->prof.ms[stage];
  if (launches) *launches = (int)h->prof.launches[stage];
  if (name) *name = stage < h->prof.nStages ? h->prof.names[stage] : "extract_total";
  return ORB_OK;
}

}  // extern "C"

// ================================================================== matcher
struct FrustumParamsHost {  // mirrors FrustumParams in matcher_kernels.hip
  float fx, fy, cx, cy, bf;
  float minX, maxX, minY, maxY;
  float cosLimit, logScale;
  int nLevels;
};

static FrustumParamsHost frustum_params(const orb_camera_t* cam, float min_x, float max_x,
                                        float min_y, float max_y, float cos_limit,
                                        float log_scale, int n_levels) {
  FrustumParamsHost f;
  f.fx = cam->fx;
  f.fy = cam->fy;
  f.cx = cam->cx;
  f.cy = cam->cy;
  f.bf = cam->bf;
  f.minX = min_x;
  f.maxX = max_x;
  f.minY = min_y;
  f.maxY = max_y;
  f.cosLimit = cos_limit;
  f.logScale = log_scale;
  f.nLevels = n_levels;
  return f;
}

struct ProjParamsHost {  // mirrors ProjParams in matcher_common.h
  float minX, minY, invW, invH;
  float th, nnratio;
  int nLevels;
  float scale[ORB_MAX_LEVELS];
  uint32_t* ovf;
  uint32_t* ovfCtr;
  uint32_t gen;
};

struct StereoParamsHost {  // mirrors StereoParams in matcher_kernels.hip
  int nLevels;
  float bf, fx;
  int w[ORB_MAX_LEVELS], h[ORB_MAX_LEVELS];
  int strideL[ORB_MAX_LEVELS], strideR[ORB_MAX_LEVELS];
  float scale[ORB_MAX_LEVELS], invScale[ORB_MAX_LEVELS];
};
struct StereoPairLevelsHost {
  const uint8_t* L[ORB_MAX_LEVELS];
  const uint8_t* R[ORB_MAX_LEVELS];
};
struct FrameProjParamsHost {  // mirrors FrameProjParams
  float minX, maxX, minY, maxY, invW, invH;
  float fx, fy, cx, cy, bf;
  float th;
  int fwd, bwd, checkOri;
  float scale[ORB_MAX_LEVELS];
};

struct PPParamsHost {  // mirrors PPParams in projection_kernels.hip
  float R[9], t[3], Ow[3];
  float R2[9], t2[3];
  float fx, fy, cx, cy, bf;
  float minX, maxX, minY, maxY, invW, invH;
  float th, logScale;
  int nLevels, thr, checkOri;
  float scale[ORB_MAX_LEVELS], invSigma2[ORB_MAX_LEVELS];
};

struct TriParamsHost {  // mirrors TriParams
  float F[9];
  float ex, ey;
  int onlyStereo, checkOri;
  float scale[ORB_MAX_LEVELS], sigma2[ORB_MAX_LEVELS];
};

struct InitParamsHost {  // mirrors InitParams in mapping_kernels.hip
  float minX, minY, invW, invH;
  float r, nnratio;
  int checkOri;
};

struct orb_matcher {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t evLast = nullptr;        // recorded where the last call ended (CallOrder)
  hipStream_t lastStream = nullptr;   // its stream (null: nothing pending)
  std::mutex mu;
  // profiling: stages k_grid_build, k_proj_candidates + k_proj_resolve
  StageProfiler prof;
  DevBuf dKeys, dDesc, dUr, dLocked, dNKeys, dMps, dMpDesc, dNMps, dCellStart, dCellIdx, dTopk,
      dNcand, dKpMatch, dNMatch, dA, dB, dOut;
  DevBuf dJac;  // Jacobi-resolve scratch (ORB_RESOLVE_JACOBI)
  DevBuf dOvf, dOvfCtr;  // candidate lists of SearchByProjection(F, localMap) (ProjParams.ovf)
  uint32_t ovfGen = 0;
  int stagedN = -1, stagedM = -1;  // orb_match_projection_local_stage's layout
  bool begun = false, begunStereo = false, begunLocked = false;  // _begin sent the frame's part
  int resolveSchedule = ORB_RESOLVE_AUTO;  // orb_matcher_set_resolve
  int jacobiRounds = 6;
  // stereo / frame / BoW scratch
  DevBuf dStRowStart, dStRowIdx;  // stereo vRowIndices (CSR per pair)
  DevBuf dProjStage;              // cell-ordered keypoints for k_proj_candidates (16 B per slot)
  DevBuf dRKeys, dRDesc, dNR, dPyr, dPairLv, dDepth, dSad, dBowA, dBowB, dBowC, dBowD, dBowE,
      dBowF, dBowG, dBowH, dBowI, dBowJ, dBowK;
  HostBuf hPyr;  // pinned staging of the host stereo pyramids (one DMA)
  // orb_match_projection_local: every input in one pinned block / one DMA, and
  // the matches + count back in one
  HostBuf hIn, hOutM;
  DevBuf dIn;
  // frustum scratch
  DevBuf dMapPts, dPose, dTracks, dNInView;
  // SearchForInitialization / ComputeDistinctiveDescriptors scratch
  DevBuf dK1, dD1, dK2, dD2, dN1, dN2, dPrev, dList, dM12, dOffs, dObsDesc, dBest, dBestDesc,
      dInitQ, dInitStage, dInitCounts;
  DevBuf sx[24];  // projection / triangulation / KF-KF BoW scratch
  std::vector<uint8_t> hostScratch;
};

extern "C" {

int orb_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  // host-side convenience (static ORBmatcher::DescriptorDistance); the device
  // path is orb_hamming_batch.
  int d = 0;
  for (int i = 0; i < 4; ++i) {
    uint64_t x, y;
    memcpy(&x, a + 8 * i, 8);
    memcpy(&y, b + 8 * i, 8);
    d += __builtin_popcountll(x ^ y);
  }
  return d;
}

orb_status_t orb_matcher_create(int device, orb_matcher_t** out) {
  if (!out) return ORB_EINVAL;
  *out = nullptr;
  orb_status_t st = check_device(device);
  if (st) return st;
  if (orb_k_proj_params_size() != sizeof(ProjParamsHost) ||
      orb_k_stereo_params_size() != sizeof(StereoParamsHost) ||
      orb_k_frame_params_size() != sizeof(FrameProjParamsHost) ||
      orb_k_frustum_params_size() != sizeof(FrustumParamsHost) ||
      orb_k_init_params_size() != sizeof(InitParamsHost) ||
      orb_k_pp_params_size() != sizeof(PPParamsHost) ||
      orb_k_tri_params_size() != sizeof(TriParamsHost))
    return ORB_EINVAL;
  orb_matcher* m = new orb_matcher();
  m->device = device;
  m->prof.nStages = 3;
  m->prof.names[0] = "k_grid_build";
  m->prof.names[1] = "k_proj_candidates";
  m->prof.names[2] = "k_proj_resolve";
  for (int i = 0; i < 3; ++i) m->prof.launchesPerCall[i] = 1;
  hipSetDevice(device);
  if (create_own_stream(&m->stream) != hipSuccess) {
    delete m;
    return ORB_EDEVICE;
  }
  if (hipEventCreateWithFlags(&m->evLast, hipEventDisableTiming) != hipSuccess) {
    hipStreamDestroy(m->stream);
    delete m;
    return ORB_EDEVICE;
  }
  *out = m;
  return ORB_OK;
}

void orb_matcher_destroy(orb_matcher_t* m) {
  if (!m) return;
  hipSetDevice(m->device);
  hipStreamSynchronize(m->stream);
  if (m->lastStream) hipEventSynchronize(m->evLast);  // a batch call on a caller's stream
  DevBuf* bufs[] = {&m->dKeys, &m->dDesc, &m->dUr, &m->dLocked, &m->dNKeys, &m->dMps,
                    &m->dMpDesc, &m->dNMps, &m->dCellStart, &m->dCellIdx, &m->dTopk,
                    &m->dNcand, &m->dKpMatch, &m->dNMatch, &m->dA, &m->dB, &m->dOut, &m->dJac,
                    &m->dRKeys, &m->dRDesc, &m->dNR, &m->dPyr, &m->dPairLv, &m->dDepth,
                    &m->dSad, &m->dStRowStart, &m->dStRowIdx, &m->dProjStage, &m->dBowA, &m->dBowB, &m->dBowC, &m->dBowD, &m->dBowE,
                    &m->dBowF, &m->dBowG, &m->dBowH, &m->dBowI, &m->dBowJ, &m->dBowK,
                    &m->dMapPts, &m->dPose, &m->dTracks, &m->dNInView, &m->dK1, &m->dD1,
                    &m->dK2, &m->dD2, &m->dN1, &m->dN2, &m->dPrev, &m->dList, &m->dM12,
                    &m->dOffs, &m->dObsDesc, &m->dBest, &m->dBestDesc, &m->dInitQ,
                    &m->dInitStage, &m->dInitCounts, &m->dOvf, &m->dOvfCtr};
  for (DevBuf* b : bufs) b->release();
  m->hPyr.release();
  m->hIn.release();
  m->hOutM.release();
  m->dIn.release();
  for (DevBuf& b : m->sx) b.release();
  m->prof.destroy();
  hipStreamDestroy(m->stream);
  hipEventDestroy(m->evLast);
  delete m;
}

void* orb_matcher_stream(orb_matcher_t* m) { return m ? (void*)m->stream : nullptr; }

orb_status_t orb_hamming_batch(orb_matcher_t* m, const uint8_t* d_a, const uint8_t* d_b, int n,
                               int32_t* d_dist, void* stream) {
  if (!m || n < 0 || (n > 0 && (!d_a || !d_b || !d_dist))) return ORB_EINVAL;
  hipSetDevice(m->device);
  HIP_TRY(orb_k_hamming(d_a, d_b, n, d_dist, stream ? (hipStream_t)stream : m->stream));
  return ORB_OK;
}

static ProjParamsHost proj_params(float min_x, float max_x, float min_y, float max_y,
                                  int n_levels, const float* scale, float th, float nnratio) {
  ProjParamsHost P;
  memset(&P, 0, sizeof(P));
  P.minX = min_x;
  P.minY = min_y;
  // mfGridElementWidthInv / HeightInv, src/Frame.cc:240-241
  P.invW = (float)ORB_GRID_COLS / (max_x - min_x);
  P.invH = (float)ORB_GRID_ROWS / (max_y - min_y);
  P.th = th;
  P.nnratio = nnratio;
  P.nLevels = n_levels;
  for (int i = 0; i < n_levels && i < ORB_MAX_LEVELS; ++i) P.scale[i] = scale[i];
  return P;
}

// The candidate-list pool of n problems for this call (ProjParams.ovf): the
// per-problem slot counters are tagged with the call's gen, so they need no
// reset between calls -- only a zero fill when (re)allocated.
static orb_status_t ovf_pool(orb_matcher_t* m, int nproblems, ProjParamsHost& P, hipStream_t s) {
  orb_status_t st;
  if ((st = m->dOvf.ensure(orb_k_proj_ovf_bytes(nproblems)))) return st;
  const size_t oldBytes = m->dOvfCtr.bytes;  // (a reallocation may return the old address)
  if ((st = m->dOvfCtr.ensure((size_t)std::max(nproblems, 1) * 4))) return st;
  if (m->dOvfCtr.bytes != oldBytes) HIP_TRY(hipMemsetAsync(m->dOvfCtr.p, 0, m->dOvfCtr.bytes, s));
  m->ovfGen = m->ovfGen % 4095u + 1u;
  P.ovf = m->dOvf.as<uint32_t>();
  P.ovfCtr = m->dOvfCtr.as<uint32_t>();
  P.gen = m->ovfGen;
  return ORB_OK;
}

orb_status_t orb_match_projection_local_batch(
    orb_matcher_t* m, int n_problems, const orb_keypoint_t* d_keys, const uint8_t* d_desc,
    const int32_t* d_nkeys, const uint8_t* d_locked, int kp_stride,
    const orb_mp_track_t* d_mps, const uint8_t* d_mp_desc, const int32_t* d_nmps,
    int mp_stride, float min_x, float max_x, float min_y, float max_y, int n_levels,
    const float* scale_factors, float th, float nnratio, int32_t* d_kp_match,
    int32_t* d_nmatches, void* stream) {
  if (!m || n_problems < 0 || kp_stride <= 0 || mp_stride < 0 || !scale_factors ||
      n_levels <= 0 || n_levels > ORB_MAX_LEVELS || kp_stride >= (1 << 19) || !(max_x > min_x) ||
      !(max_y > min_y))
    return ORB_EINVAL;
  if (n_problems == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  ProjParamsHost P =
      proj_params(min_x, max_x, min_y, max_y, n_levels, scale_factors, th, nnratio);
  orb_status_t st;
  if ((st = ovf_pool(m, n_problems, P, s))) return st;
  if ((st = m->dCellStart.ensure((size_t)n_problems * (ORB_GRID_COLS * ORB_GRID_ROWS + 1) * 4)))
    return st;
  if ((st = m->dCellIdx.ensure((size_t)n_problems * kp_stride * 4))) return st;
  if ((st = m->dTopk.ensure((size_t)n_problems * std::max(mp_stride, 1) * 16))) return st;
  if ((st = m->dNcand.ensure((size_t)n_problems * std::max(mp_stride, 1) * 4))) return st;
  const bool stage = kp_stride <= orb_k_grid_stage_max();
  if (stage && (st = m->dProjStage.ensure((size_t)n_problems * kp_stride * 16))) return st;
  const size_t jb = orb_k_proj_jacobi_bytes(kp_stride, mp_stride, n_problems, m->resolveSchedule);
  if (jb && (st = m->dJac.ensure(jb))) return st;
  StageProfiler& pf = m->prof;
  std::vector<hipEvent_t>* ev = pf.begin_call();
  PROF_REC(ev, pf.t0(ev), s);
  PROF_REC(ev, pf.b(ev, 0), s);
  if (stage)
    HIP_TRY(orb_k_grid_build_staged(d_keys, d_nkeys, d_locked, nullptr, kp_stride, P.minX, P.minY,
                                    P.invW, P.invH, m->dCellStart.as<int32_t>(),
                                    m->dCellIdx.as<int32_t>(), m->dProjStage.p, n_problems, s));
  else
    HIP_TRY(orb_k_grid_build(d_keys, d_nkeys, kp_stride, P.minX, P.minY, P.invW, P.invH,
                             m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(), n_problems,
                             s));
  PROF_REC(ev, pf.e(ev, 0), s);
  PROF_REC(ev, pf.b(ev, 1), s);
  HIP_TRY(orb_k_proj_candidates(d_keys, d_desc, nullptr, d_locked, kp_stride, d_nkeys, d_mps, d_mp_desc,
                                d_nmps, mp_stride, mp_stride, m->dCellStart.as<int32_t>(),
                                m->dCellIdx.as<int32_t>(), stage ? m->dProjStage.p : nullptr,
                                &P, m->dTopk.as<uint32_t>(),
                                m->dNcand.as<int32_t>(), n_problems, s));
  PROF_REC(ev, pf.e(ev, 1), s);
  PROF_REC(ev, pf.b(ev, 2), s);
  HIP_TRY(orb_k_proj_resolve(d_keys, d_desc, nullptr, d_locked, d_nkeys, kp_stride, d_mps,
                             d_mp_desc, d_nmps, mp_stride, m->dCellStart.as<int32_t>(),
                             m->dCellIdx.as<int32_t>(), &P, m->dTopk.as<uint32_t>(),
                             m->dNcand.as<int32_t>(), d_kp_match, d_nmatches, n_problems,
                             m->resolveSchedule, m->jacobiRounds, m->dJac.as<int32_t>(), s));
  PROF_REC(ev, pf.e(ev, 2), s);
  PROF_REC(ev, pf.t1(ev), s);
  return ORB_OK;
}

orb_status_t orb_matcher_set_resolve(orb_matcher_t* m, int schedule, int jacobi_rounds) {
  if (!m || schedule < ORB_RESOLVE_AUTO || schedule > ORB_RESOLVE_JACOBI ||
      (schedule == ORB_RESOLVE_JACOBI && (jacobi_rounds < 1 || jacobi_rounds > 48)))
    return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  m->resolveSchedule = schedule;
  if (schedule == ORB_RESOLVE_JACOBI) m->jacobiRounds = jacobi_rounds;
  return ORB_OK;
}

orb_status_t orb_matcher_resolve_kernel(orb_matcher_t* m, int n_problems, int kp_stride,
                                        int mp_stride, int* kernel) {
  if (!m || !kernel || n_problems <= 0 || kp_stride <= 0 || mp_stride < 0) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  *kernel = orb_k_proj_resolve_kernel(n_problems, kp_stride, std::max(mp_stride, 1),
                                      m->resolveSchedule);
  return ORB_OK;
}

orb_status_t orb_matcher_profile(orb_matcher_t* m, int enable) {
  if (!m) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  m->prof.drain();
  m->prof.reset();
  m->prof.enabled = enable != 0;
  return ORB_OK;
}

orb_status_t orb_matcher_profile_read(orb_matcher_t* m, int stage, double* total_ms,
                                      int* launches, const char** name) {
  if (!m || stage < 0 || stage > m->prof.nStages) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  m->prof.drain();
  if (total_ms) *total_ms = m->prof.ms[stage];
  if (launches) *launches = (int)m->prof.launches[stage];
  if (name) *name = stage < m->prof.nStages ? m->prof.names[stage] : "match_total";
  return ORB_OK;
}

}  // extern "C"

// orb_match_projection_local's inputs, one pinned block and one DMA in (six
// pageable copies each staged by the runtime cost more than the kernels):
// [nk, nm | keys | descriptors | uR | locked | tracks | map-point descriptors],
// 16-B aligned
struct LocalLayout {
  size_t oKeys, oDesc, oUr, oLk, oMps, oMpd, inBytes;
};
static LocalLayout local_layout(int N, int M) {
  auto al16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
  LocalLayout L;
  L.oKeys = 16;
  L.oDesc = al16(L.oKeys + (size_t)N * sizeof(orb_keypoint_t));
  L.oUr = al16(L.oDesc + (size_t)N * 32);
  L.oLk = al16(L.oUr + (size_t)N * 4);
  L.oMps = al16(L.oLk + (size_t)N);
  L.oMpd = al16(L.oMps + (size_t)M * sizeof(orb_mp_track_t));
  L.inBytes = al16(L.oMpd + (size_t)M * 32);
  return L;
}

// The pinned input block for N keypoints and M map points (header written);
// caller holds m->mu
// A _begin whose _staged never came (or failed): its DMA may still read the
// pinned block, so wait for it before the block is rewritten; caller holds m->mu
static orb_status_t local_abandon(orb_matcher_t* m) {
  if (!m->begun) return ORB_OK;
  m->begun = false;
  hipSetDevice(m->device);
  HIP_TRY(stream_wait(m->stream));
  return ORB_OK;
}

static orb_status_t local_stage(orb_matcher_t* m, int N, int M, LocalLayout* out) {
  const LocalLayout L = local_layout(N, M);
  orb_status_t st;
  if ((st = local_abandon(m))) return st;
  if ((st = m->hIn.ensure(L.inBytes))) return st;
  const int32_t nk = N, nm = M;
  memcpy(m->hIn.as<uint8_t>(), &nk, 4);
  memcpy(m->hIn.as<uint8_t>() + 4, &nm, 4);
  *out = L;
  return ORB_OK;
}

// SearchByProjection(F, vpMapPoints) on the inputs staged in the pinned block:
// one DMA in, grid + candidates + resolve, one DMA out; caller holds m->mu.
// In two parts when the frame's part of the block was sent ahead
// (local_begin: its DMA and the keypoint grid run while the caller flattens
// the map into the rest of the block).
static orb_status_t local_ensure(orb_matcher_t* m, int N, int M, const LocalLayout& L) {
  orb_status_t st;
  // (inputs live in dIn below; only the outputs and the matcher scratch here)
  if ((st = m->dKpMatch.ensure((size_t)N * 4 + 16))) return st;  // + the count (one D2H)
  if ((st = m->dCellStart.ensure((size_t)(ORB_GRID_COLS * ORB_GRID_ROWS + 1) * 4))) return st;
  if ((st = m->dCellIdx.ensure((size_t)N * 4))) return st;
  if ((st = m->dTopk.ensure((size_t)std::max(M, 1) * 16))) return st;
  if ((st = m->dNcand.ensure((size_t)std::max(M, 1) * 4))) return st;
  if ((st = m->dIn.ensure(L.inBytes))) return st;
  if ((st = m->hOutM.ensure((size_t)N * 4 + 16))) return st;
  if (N <= orb_k_grid_stage_max() && (st = m->dProjStage.ensure((size_t)N * 16))) return st;
  const size_t jb = orb_k_proj_jacobi_bytes(N, std::max(M, 1), 1, m->resolveSchedule);
  if (jb && (st = m->dJac.ensure(jb))) return st;
  return ORB_OK;
}

// DMA of bytes [b0, b1) of the block, then (b0 == 0) the keypoint grid
static orb_status_t local_front(orb_matcher_t* m, int N, const LocalLayout& L, const ProjParamsHost& P,
                                bool urOn, bool lkOn, size_t b1, hipStream_t s) {
  HIP_TRY(orb_k_copy_pinned(m->dIn.p, m->hIn.p, b1, s));
  uint8_t* din = m->dIn.as<uint8_t>();
  const orb_keypoint_t* dKeys = reinterpret_cast<const orb_keypoint_t*>(din + L.oKeys);
  const int32_t* dNK = reinterpret_cast<const int32_t*>(din);
  const float* ur = urOn ? reinterpret_cast<const float*>(din + L.oUr) : nullptr;
  const uint8_t* lk = lkOn ? din + L.oLk : nullptr;
  if (N <= orb_k_grid_stage_max())
    HIP_TRY(orb_k_grid_build_staged(dKeys, dNK, lk, ur, N, P.minX, P.minY, P.invW, P.invH,
                                    m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(),
                                    m->dProjStage.p, 1, s));
  else
    HIP_TRY(orb_k_grid_build(dKeys, dNK, N, P.minX, P.minY, P.invW, P.invH,
                             m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(), 1, s));
  return ORB_OK;
}

static orb_status_t local_run(orb_matcher_t* m, int N, int M, const orb_frame_t* F, bool urOn,
                              bool lkOn, float th, float nnratio, int32_t* kp_match,
                              int32_t* nmatches, bool begun = false) {
  hipSetDevice(m->device);
  const LocalLayout L = local_layout(N, M);
  orb_status_t st;
  if (!begun && (st = local_ensure(m, N, M, L))) return st;
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  ProjParamsHost P = proj_params(F->min_x, F->max_x, F->min_y, F->max_y, F->n_levels,
                                 F->scale_factors, th, nnratio);
  if ((st = ovf_pool(m, 1, P, s))) return st;
  if (!begun) {
    if ((st = local_front(m, N, L, P, urOn, lkOn, L.inBytes, s))) return st;
  } else if (L.inBytes > L.oMps) {  // the map's part of the block
    HIP_TRY(orb_k_copy_pinned(m->dIn.as<uint8_t>() + L.oMps, m->hIn.as<uint8_t>() + L.oMps,
                              L.inBytes - L.oMps, s));
  }
  uint8_t* din = m->dIn.as<uint8_t>();
  const orb_keypoint_t* dKeys = reinterpret_cast<const orb_keypoint_t*>(din + L.oKeys);
  const uint8_t* dDesc = din + L.oDesc;
  const int32_t* dNK = reinterpret_cast<const int32_t*>(din);
  const int32_t* dNM = reinterpret_cast<const int32_t*>(din + 4);
  const orb_mp_track_t* dMps = reinterpret_cast<const orb_mp_track_t*>(din + L.oMps);
  const uint8_t* dMpd = din + L.oMpd;
  const float* ur = urOn ? reinterpret_cast<const float*>(din + L.oUr) : nullptr;
  const uint8_t* lk = lkOn ? din + L.oLk : nullptr;
  const bool stage = N <= orb_k_grid_stage_max();
  HIP_TRY(orb_k_proj_candidates(dKeys, dDesc, ur, lk, N, dNK, dMps, dMpd, dNM, std::max(M, 1), M,
                                m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(),
                                stage ? m->dProjStage.p : nullptr, &P, m->dTopk.as<uint32_t>(),
                                m->dNcand.as<int32_t>(), 1, s));
  HIP_TRY(orb_k_proj_resolve(dKeys, dDesc, ur, lk, dNK, N, dMps, dMpd, dNM, std::max(M, 1),
                             m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(), &P,
                             m->dTopk.as<uint32_t>(), m->dNcand.as<int32_t>(),
                             m->dKpMatch.as<int32_t>(), m->dKpMatch.as<int32_t>() + N, 1,
                             m->resolveSchedule, m->jacobiRounds, m->dJac.as<int32_t>(), s));
  // one DMA out (count, then the matches) into pinned memory
  HIP_TRY(orb_k_copy_to_pinned(m->hOutM.p, m->dKpMatch.p, (size_t)N * 4 + 4, s));
  HIP_TRY(stream_wait(s));
  order.settled();
  memcpy(kp_match, m->hOutM.p, (size_t)N * 4);
  memcpy(nmatches, m->hOutM.as<uint8_t>() + (size_t)N * 4, 4);
  return ORB_OK;
}

static bool local_frame_ok(const orb_frame_t* F) {
  return F && F->n >= 0 && F->scale_factors && F->n_levels > 0 && F->n_levels <= ORB_MAX_LEVELS &&
         F->n < (1 << 19);
}

extern "C" {

orb_status_t orb_match_projection_local(orb_matcher_t* m, const orb_frame_t* F,
                                        const uint8_t* kp_locked, int n_mp,
                                        const orb_mp_track_t* mps, const uint8_t* mp_desc,
                                        float th, float nnratio, int32_t* kp_match,
                                        int32_t* nmatches) {
  if (!m || !F || n_mp < 0 || (n_mp > 0 && (!mps || !mp_desc)) || !kp_match || !nmatches)
    return ORB_EINVAL;
  if (!local_frame_ok(F) || (F->n > 0 && (!F->keys || !F->descriptors))) return ORB_EINVAL;
  *nmatches = 0;
  if (F->n == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  const int N = F->n, M = n_mp;
  LocalLayout L;
  orb_status_t st = local_stage(m, N, M, &L);
  if (st) return st;
  uint8_t* hin = m->hIn.as<uint8_t>();
  memcpy(hin + L.oKeys, F->keys, (size_t)N * sizeof(orb_keypoint_t));
  memcpy(hin + L.oDesc, F->descriptors, (size_t)N * 32);
  if (F->u_right) memcpy(hin + L.oUr, F->u_right, (size_t)N * 4);
  if (kp_locked) memcpy(hin + L.oLk, kp_locked, (size_t)N);
  if (M > 0) {
    memcpy(hin + L.oMps, mps, (size_t)M * sizeof(orb_mp_track_t));
    memcpy(hin + L.oMpd, mp_desc, (size_t)M * 32);
  }
  return local_run(m, N, M, F, F->u_right != nullptr, kp_locked != nullptr, th, nnratio, kp_match,
                   nmatches);
}

orb_status_t orb_match_projection_local_stage(orb_matcher_t* m, int n_keys, int n_mp,
                                              orb_local_stage_t* out) {
  if (!m || !out || n_keys <= 0 || n_keys >= (1 << 19) || n_mp < 0) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  LocalLayout L;
  orb_status_t st = local_stage(m, n_keys, n_mp, &L);
  if (st) return st;
  uint8_t* hin = m->hIn.as<uint8_t>();
  out->keys = reinterpret_cast<orb_keypoint_t*>(hin + L.oKeys);
  out->descriptors = hin + L.oDesc;
  out->u_right = reinterpret_cast<float*>(hin + L.oUr);
  out->kp_locked = hin + L.oLk;
  out->mps = reinterpret_cast<orb_mp_track_t*>(hin + L.oMps);
  out->mp_desc = hin + L.oMpd;
  m->stagedN = n_keys;
  m->stagedM = n_mp;
  return ORB_OK;
}

orb_status_t orb_match_projection_local_begin(orb_matcher_t* m, const orb_frame_t* frame,
                                              int stereo, int locked) {
  if (!m || !local_frame_ok(frame)) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  if (frame->n <= 0 || frame->n != m->stagedN || m->begun) return ORB_EINVAL;
  hipSetDevice(m->device);
  const int N = frame->n, M = m->stagedM;
  const LocalLayout L = local_layout(N, M);
  orb_status_t st = local_ensure(m, N, M, L);
  if (st) return st;
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  // (th and nnratio do not enter the grid)
  const ProjParamsHost P = proj_params(frame->min_x, frame->max_x, frame->min_y, frame->max_y,
                                       frame->n_levels, frame->scale_factors, 1.f, 0.f);
  if ((st = local_front(m, N, L, P, stereo != 0, locked != 0, L.oMps, s))) return st;
  m->begun = true;
  m->begunStereo = stereo != 0;
  m->begunLocked = locked != 0;
  return ORB_OK;
}

orb_status_t orb_match_projection_local_staged(orb_matcher_t* m, const orb_frame_t* frame,
                                               int n_mp, int stereo, int locked, float th,
                                               float nnratio, int32_t* kp_match,
                                               int32_t* nmatches) {
  if (!m || !local_frame_ok(frame) || !kp_match || !nmatches) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  // the block must hold what _stage laid out for exactly these counts
  const bool begun = m->begun;
  const int sn = m->stagedN, sm = m->stagedM;
  m->stagedN = m->stagedM = -1;
  if (frame->n <= 0 || frame->n != sn || n_mp != sm ||
      (begun && (m->begunStereo != (stereo != 0) || m->begunLocked != (locked != 0)))) {
    const orb_status_t st = local_abandon(m);  // (the block must be staged again)
    return st ? st : ORB_EINVAL;
  }
  m->begun = false;
  *nmatches = 0;
  return local_run(m, frame->n, n_mp, frame, stereo != 0, locked != 0, th, nnratio, kp_match,
                   nmatches, begun);
}

// ----------------------------------------------------------------- frustum
orb_status_t orb_frustum(orb_matcher_t* m, int n_mp, const orb_map_point_t* mps,
                         const orb_pose_t* pose, const orb_camera_t* cam, float min_x,
                         float max_x, float min_y, float max_y, float viewing_cos_limit,
                         float log_scale_factor, int n_levels, orb_mp_track_t* tracks,
                         int32_t* n_in_view) {
  if (!m || n_mp < 0 || (n_mp > 0 && (!mps || !tracks)) || !pose || !cam || !n_in_view ||
      n_levels <= 0 || n_levels > ORB_MAX_LEVELS)
    return ORB_EINVAL;
  *n_in_view = 0;
  if (n_mp == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  orb_status_t st;
  if ((st = m->dMapPts.ensure((size_t)n_mp * sizeof(orb_map_point_t)))) return st;
  if ((st = m->dPose.ensure(sizeof(orb_pose_t)))) return st;
  if ((st = m->dTracks.ensure((size_t)n_mp * sizeof(orb_mp_track_t)))) return st;
  if ((st = m->dNInView.ensure(16))) return st;
  if ((st = m->dNMps.ensure(16))) return st;
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  HIP_TRY(hipMemcpyAsync(m->dMapPts.p, mps, (size_t)n_mp * sizeof(orb_map_point_t),
                         hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(m->dPose.p, pose, sizeof(orb_pose_t), hipMemcpyHostToDevice, s));
  const int32_t nm = n_mp;
  HIP_TRY(hipMemcpyAsync(m->dNMps.p, &nm, 4, hipMemcpyHostToDevice, s));
  const FrustumParamsHost fp = frustum_params(cam, min_x, max_x, min_y, max_y, viewing_cos_limit,
                                              log_scale_factor, n_levels);
  HIP_TRY(orb_k_frustum(m->dMapPts.as<orb_map_point_t>(), m->dNMps.as<int32_t>(), n_mp, n_mp,
                        m->dPose.as<orb_pose_t>(), &fp, m->dTracks.as<orb_mp_track_t>(),
                        m->dNInView.as<int32_t>(), 1, s));
  HIP_TRY(hipMemcpyAsync(tracks, m->dTracks.p, (size_t)n_mp * sizeof(orb_mp_track_t),
                         hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(n_in_view, m->dNInView.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_frustum_batch(orb_matcher_t* m, int n_problems, const orb_map_point_t* d_mps,
                               const int32_t* d_nmps, int mp_stride, const orb_pose_t* d_poses,
                               const orb_camera_t* cam, float min_x, float max_x, float min_y,
                               float max_y, float viewing_cos_limit, float log_scale_factor,
                               int n_levels, orb_mp_track_t* d_tracks, int32_t* d_n_in_view,
                               void* stream) {
  if (!m || n_problems < 0 || mp_stride < 0 || !cam || n_levels <= 0 ||
      n_levels > ORB_MAX_LEVELS)
    return ORB_EINVAL;
  if (n_problems == 0) return ORB_OK;
  if (!d_mps || !d_nmps || !d_poses || !d_tracks || !d_n_in_view || n_problems > 65535)
    return ORB_EINVAL;
  hipSetDevice(m->device);
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  const FrustumParamsHost fp = frustum_params(cam, min_x, max_x, min_y, max_y, viewing_cos_limit,
                                              log_scale_factor, n_levels);
  HIP_TRY(orb_k_frustum(d_mps, d_nmps, mp_stride, mp_stride, d_poses, &fp, d_tracks, d_n_in_view,
                        n_problems, s));
  return ORB_OK;
}

// ------------------------------------------------------------------ stereo
static orb_status_t upload(DevBuf& b, const void* src, size_t n, hipStream_t s) {
  orb_status_t st = b.ensure(std::max<size_t>(n, 16));
  if (st) return st;
  if (n) HIP_TRY(hipMemcpyAsync(b.p, src, n, hipMemcpyHostToDevice, s));
  return ORB_OK;
}

// the row-index scratch of orb_k_stereo for n_pairs pairs
static orb_status_t stereo_scratch(orb_matcher* m, const void* params, int kpStride, int npairs) {
  size_t a = 0, b = 0;
  orb_k_stereo_scratch(params, kpStride, &a, &b);
  orb_status_t st = m->dStRowStart.ensure(std::max<size_t>(a * npairs, 1) * 4);
  if (st) return st;
  return m->dStRowIdx.ensure(std::max<size_t>(b * npairs, 1) * 4);
}

orb_status_t orb_stereo_match(orb_matcher_t* m, const orb_stereo_input_t* in, float* u_right,
                              float* depth) {
  if (!m || !in || !in->left || !u_right || !depth) return ORB_EINVAL;
  const orb_frame_t* F = in->left;
  const int NL = F->n, NR = in->n_right, L = in->n_levels;
  if (NL < 0 || NR < 0 || L <= 0 || L > ORB_MAX_LEVELS || !F->scale_factors ||
      !in->inv_scale_factors || !in->left_levels || !in->right_levels || !in->level_width ||
      !in->level_height || !in->level_stride || !(in->fx > 0))
    return ORB_EINVAL;
  // every level must be a real image: rows at least as long as the level
  // (the staging copy reads w bytes of each row at y * stride)
  for (int l = 0; l < L; ++l)
    if (in->level_width[l] <= 0 || in->level_height[l] <= 0 ||
        in->level_stride[l] < (int64_t)in->level_width[l] || !in->left_levels[l] ||
        !in->right_levels[l])
      return ORB_EINVAL;
  for (int i = 0; i < NL; ++i) { u_right[i] = -1.0f; depth[i] = -1.0f; }
  if (NL == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  const int stride = std::max(NL, std::max(NR, 1));
  orb_status_t st;
  if ((st = upload(m->dKeys, F->keys, (size_t)NL * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(m->dDesc, F->descriptors, (size_t)NL * 32, s))) return st;
  if ((st = upload(m->dRKeys, in->right_keys, (size_t)NR * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(m->dRDesc, in->right_desc, (size_t)NR * 32, s))) return st;
  const int32_t nl = NL, nr = NR;
  if ((st = upload(m->dNKeys, &nl, 4, s))) return st;
  if ((st = upload(m->dNR, &nr, 4, s))) return st;
  // both pyramids, packed with 64-byte pitches
  StereoParamsHost P;
  memset(&P, 0, sizeof(P));
  P.nLevels = L;
  P.bf = in->bf;
  P.fx = in->fx;
  size_t total = 0;
  std::vector<size_t> off(L);
  for (int l = 0; l < L; ++l) {
    P.w[l] = in->level_width[l];
    P.h[l] = in->level_height[l];
    P.strideL[l] = P.strideR[l] = (P.w[l] + 63) & ~63;
    P.scale[l] = F->scale_factors[l];
    P.invScale[l] = in->inv_scale_factors[l];
    off[l] = total;
    total += 2 * (size_t)P.strideL[l] * P.h[l];
  }
  if ((st = m->dPyr.ensure(total))) return st;
  StereoPairLevelsHost lv;
  memset(&lv, 0, sizeof(lv));
  uint8_t* base = m->dPyr.as<uint8_t>();
  // both pyramids -> pinned staging in the device layout -> one DMA (2-D copies
  // from pageable memory go row by row)
  if ((st = m->hPyr.ensure(total))) return st;
  uint8_t* hb = m->hPyr.as<uint8_t>();
  for (int l = 0; l < L; ++l) {
    const size_t rowsL = (size_t)P.strideL[l] * P.h[l];
    for (int y = 0; y < P.h[l]; ++y) {
      memcpy(hb + off[l] + (size_t)y * P.strideL[l],
             in->left_levels[l] + (size_t)y * in->level_stride[l], (size_t)P.w[l]);
      memcpy(hb + off[l] + rowsL + (size_t)y * P.strideR[l],
             in->right_levels[l] + (size_t)y * in->level_stride[l], (size_t)P.w[l]);
    }
    lv.L[l] = base + off[l];
    lv.R[l] = base + off[l] + rowsL;
  }
  HIP_TRY(hipMemcpyAsync(base, hb, total, hipMemcpyHostToDevice, s));
  if ((st = upload(m->dPairLv, &lv, sizeof(lv), s))) return st;
  if ((st = m->dUr.ensure((size_t)stride * 4))) return st;
  if ((st = m->dDepth.ensure((size_t)stride * 4))) return st;
  if ((st = m->dSad.ensure((size_t)stride * 4))) return st;
  if ((st = stereo_scratch(m, &P, stride, 1))) return st;
  HIP_TRY(orb_k_stereo(m->dKeys.as<orb_keypoint_t>(), m->dDesc.as<uint8_t>(),
                       m->dNKeys.as<int32_t>(), m->dRKeys.as<orb_keypoint_t>(),
                       m->dRDesc.as<uint8_t>(), m->dNR.as<int32_t>(), stride, NL, m->dPairLv.p, &P,
                       m->dUr.as<float>(), m->dDepth.as<float>(), m->dSad.as<int32_t>(), 1,
                       m->dStRowStart.as<int32_t>(), m->dStRowIdx.as<int32_t>(), s));
  HIP_TRY(hipMemcpyAsync(u_right, m->dUr.p, (size_t)NL * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(depth, m->dDepth.p, (size_t)NL * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_stereo_match_batch(orb_matcher_t* m, int n_pairs, orb_extractor_t* left_ext,
                                    orb_extractor_t* right_ext, const orb_keypoint_t* d_left_keys,
                                    const uint8_t* d_left_desc, const int32_t* d_left_n,
                                    const orb_keypoint_t* d_right_keys,
                                    const uint8_t* d_right_desc, const int32_t* d_right_n,
                                    int kp_stride, float bf, float fx, float* d_u_right,
                                    float* d_depth, int32_t* d_sad, void* stream) {
  if (!m || !left_ext || !right_ext || n_pairs < 0 || kp_stride <= 0 || !(fx > 0) ||
      !d_u_right || !d_depth || !d_sad)
    return ORB_EINVAL;
  if (n_pairs == 0) return ORB_OK;
  const int L = orb_extractor_get_levels(left_ext);
  if (L != orb_extractor_get_levels(right_ext)) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  StereoParamsHost P;
  memset(&P, 0, sizeof(P));
  P.nLevels = L;
  P.bf = bf;
  P.fx = fx;
  orb_extractor_get_scale_factors(left_ext, P.scale);
  orb_extractor_get_inverse_scale_factors(left_ext, P.invScale);
  std::vector<StereoPairLevelsHost> lv(n_pairs);
  for (int i = 0; i < n_pairs; ++i) {
    memset(&lv[i], 0, sizeof(StereoPairLevelsHost));
    for (int l = 0; l < L; ++l) {
      int wl, hl, wr, hr;
      size_t sl, sr;
      orb_status_t st = orb_extractor_batch_level(left_ext, i, l, &lv[i].L[l], &wl, &hl, &sl);
      if (st) return st;
      st = orb_extractor_batch_level(right_ext, i, l, &lv[i].R[l], &wr, &hr, &sr);
      if (st) return st;
      if (wl != wr || hl != hr) return ORB_EINVAL;
      P.w[l] = wl;
      P.h[l] = hl;
      P.strideL[l] = (int)sl;
      P.strideR[l] = (int)sr;
    }
  }
  orb_status_t st = m->dPairLv.ensure(lv.size() * sizeof(StereoPairLevelsHost));
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(m->dPairLv.p, lv.data(), lv.size() * sizeof(StereoPairLevelsHost),
                         hipMemcpyHostToDevice, s));
  if ((st = stereo_scratch(m, &P, kp_stride, n_pairs))) return st;
  HIP_TRY(orb_k_stereo(d_left_keys, d_left_desc, d_left_n, d_right_keys, d_right_desc, d_right_n,
                       kp_stride, kp_stride, m->dPairLv.p, &P, d_u_right, d_depth, d_sad,
                       n_pairs, m->dStRowStart.as<int32_t>(), m->dStRowIdx.as<int32_t>(), s));
  // the pair-level pointer table must outlive the asynchronous launch
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

// Frame::ComputeStereoMatches for the pair the two handles extracted last with
// orb_extractor_extract (src/Frame.cc:81-93 runs the two ExtractORB threads,
// then ComputeStereoMatches): keypoints, descriptors and both pyramids are
// read where the extractions left them in HBM; only mvuRight / mvDepth travel.
orb_status_t orb_stereo_match_extracted(orb_matcher_t* m, orb_extractor_t* left_ext,
                                        orb_extractor_t* right_ext, float bf, float fx,
                                        float* u_right, float* depth, int capacity,
                                        int* n_left) {
  if (!m || !left_ext || !right_ext || left_ext == right_ext || !(fx > 0) || !n_left)
    return ORB_EINVAL;
  // both handles stay locked while their last-call state is read and used
  orb_extractor* a = left_ext < right_ext ? left_ext : right_ext;
  orb_extractor* b = left_ext < right_ext ? right_ext : left_ext;
  std::lock_guard<std::mutex> ga(a->mu), gb(b->mu);
  if (!left_ext->lastSingle || !right_ext->lastSingle) return ORB_EINVAL;
  // the kernels read both handles' device buffers on the matcher's device
  if (m->device != left_ext->device || m->device != right_ext->device) return ORB_EINVAL;
  const int L = left_ext->nlevels;
  if (L != right_ext->nlevels || left_ext->planW != right_ext->planW ||
      left_ext->planH != right_ext->planH)
    return ORB_EINVAL;
  int32_t nL = 0, nR = 0;
  memcpy(&nL, left_ext->hOut.p, 4);
  memcpy(&nR, right_ext->hOut.p, 4);
  if (nL < 0 || nR < 0) return ORB_EDEVICE;
  *n_left = nL;
  if (!u_right && !depth) return ORB_OK;  // size query
  if (nL > capacity) return ORB_ECAPACITY;
  if (nL == 0) return ORB_OK;
  if (!u_right || !depth) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  HIP_TRY(hipStreamWaitEvent(s, left_ext->evBatch, 0));
  HIP_TRY(hipStreamWaitEvent(s, right_ext->evBatch, 0));
  StereoParamsHost P;
  memset(&P, 0, sizeof(P));
  P.nLevels = L;
  P.bf = bf;
  P.fx = fx;
  std::copy(left_ext->scale.begin(), left_ext->scale.end(), P.scale);
  std::copy(left_ext->invScale.begin(), left_ext->invScale.end(), P.invScale);
  StereoPairLevelsHost lv;
  memset(&lv, 0, sizeof(lv));
  for (int l = 0; l < L; ++l) {
    const OrbLevelDesc& dl = left_ext->plan.lv[l];
    const OrbLevelDesc& dr = right_ext->plan.lv[l];
    P.w[l] = dl.w;
    P.h[l] = dl.h;
    if (l == 0) {  // level 0 = the image staged by orb_extractor_extract
      lv.L[0] = left_ext->dImg.as<uint8_t>();
      lv.R[0] = right_ext->dImg.as<uint8_t>();
      P.strideL[0] = (int)one_stride(dl.w);
      P.strideR[0] = (int)one_stride(dr.w);
    } else {
      lv.L[l] = left_ext->dArena.as<uint8_t>() + dl.arenaOff;
      lv.R[l] = right_ext->dArena.as<uint8_t>() + dr.arenaOff;
      P.strideL[l] = dl.pitch;
      P.strideR[l] = dr.pitch;
    }
  }
  orb_status_t st;
  if ((st = m->dPairLv.ensure(sizeof(lv)))) return st;
  if ((st = m->dUr.ensure((size_t)nL * 4))) return st;
  if ((st = m->dDepth.ensure((size_t)nL * 4))) return st;
  if ((st = m->dSad.ensure((size_t)nL * 4))) return st;
  if ((st = m->hPyr.ensure((size_t)nL * 8 + sizeof(lv)))) return st;
  memcpy(m->hPyr.as<uint8_t>() + (size_t)nL * 8, &lv, sizeof(lv));
  HIP_TRY(hipMemcpyAsync(m->dPairLv.p, m->hPyr.as<uint8_t>() + (size_t)nL * 8, sizeof(lv),
                         hipMemcpyHostToDevice, s));
  const uint8_t* l1 = left_ext->dOne.as<uint8_t>();
  const uint8_t* r1 = right_ext->dOne.as<uint8_t>();
  const int stride = std::max(left_ext->oneCap, right_ext->oneCap);
  // the two records blocks have their own capacities: pair 0 only, so the
  // shared kpStride of the kernel is never applied
  if ((st = stereo_scratch(m, &P, stride, 1))) return st;
  HIP_TRY(orb_k_stereo(reinterpret_cast<const orb_keypoint_t*>(l1 + 16),
                       l1 + 16 + (size_t)left_ext->oneCap * sizeof(orb_keypoint_t),
                       reinterpret_cast<const int32_t*>(l1),
                       reinterpret_cast<const orb_keypoint_t*>(r1 + 16),
                       r1 + 16 + (size_t)right_ext->oneCap * sizeof(orb_keypoint_t),
                       reinterpret_cast<const int32_t*>(r1), stride, nL, m->dPairLv.p, &P,
                       m->dUr.as<float>(), m->dDepth.as<float>(), m->dSad.as<int32_t>(), 1,
                       m->dStRowStart.as<int32_t>(), m->dStRowIdx.as<int32_t>(), s));
  HIP_TRY(hipMemcpyAsync(m->hPyr.p, m->dUr.p, (size_t)nL * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(m->hPyr.as<uint8_t>() + (size_t)nL * 4, m->dDepth.p, (size_t)nL * 4,
                         hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  memcpy(u_right, m->hPyr.p, (size_t)nL * 4);
  memcpy(depth, m->hPyr.as<uint8_t>() + (size_t)nL * 4, (size_t)nL * 4);
  return ORB_OK;
}

// -------------------------------------------------- SearchByProjection(F, LastF)
orb_status_t orb_match_projection_frame(orb_matcher_t* m, const orb_frame_t* C,
                                        const uint8_t* kp_locked, int n_last,
                                        const orb_last_mp_t* last, const uint8_t* last_desc,
                                        const orb_camera_t* cam, float tlc_z, float th,
                                        int mono, int check_orientation, int32_t* kp_match,
                                        int32_t* nmatches) {
  if (!m || !C || !cam || n_last < 0 || (n_last > 0 && (!last || !last_desc)) || !kp_match ||
      !nmatches || C->n < 0 || (C->n > 0 && (!C->keys || !C->descriptors)) ||
      !C->scale_factors || C->n_levels <= 0 || C->n_levels > ORB_MAX_LEVELS ||
      C->n >= (1 << 19))
    return ORB_EINVAL;
  *nmatches = 0;
  for (int i = 0; i < C->n; ++i) kp_match[i] = -1;
  if (C->n == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  const int N = C->n, M = n_last;
  orb_status_t st;
  if ((st = upload(m->dKeys, C->keys, (size_t)N * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(m->dDesc, C->descriptors, (size_t)N * 32, s))) return st;
  if (C->u_right && (st = upload(m->dUr, C->u_right, (size_t)N * 4, s))) return st;
  if (kp_locked && (st = upload(m->dLocked, kp_locked, (size_t)N, s))) return st;
  const int32_t nk = N;
  if ((st = upload(m->dNKeys, &nk, 4, s))) return st;
  if ((st = upload(m->dA, last, (size_t)M * sizeof(orb_last_mp_t), s))) return st;
  if ((st = upload(m->dB, last_desc, (size_t)M * 32, s))) return st;
  if ((st = m->dCellStart.ensure((size_t)(ORB_GRID_COLS * ORB_GRID_ROWS + 1) * 4))) return st;
  if ((st = m->dCellIdx.ensure((size_t)N * 4))) return st;
  if ((st = m->dTopk.ensure((size_t)std::max(M, 1) * 16))) return st;
  if ((st = m->dNcand.ensure((size_t)std::max(M, 1) * 4))) return st;
  if ((st = m->dKpMatch.ensure((size_t)N * 4))) return st;
  if ((st = m->dNMatch.ensure(16))) return st;
  FrameProjParamsHost P;
  memset(&P, 0, sizeof(P));
  P.minX = C->min_x; P.maxX = C->max_x; P.minY = C->min_y; P.maxY = C->max_y;
  P.invW = (float)ORB_GRID_COLS / (C->max_x - C->min_x);
  P.invH = (float)ORB_GRID_ROWS / (C->max_y - C->min_y);
  P.fx = cam->fx; P.fy = cam->fy; P.cx = cam->cx; P.cy = cam->cy; P.bf = cam->bf;
  P.th = th;
  P.fwd = (tlc_z > cam->mb && !mono) ? 1 : 0;   // src/ORBmatcher.cc:1482-1484
  P.bwd = (-tlc_z > cam->mb && !mono) ? 1 : 0;
  P.checkOri = check_orientation ? 1 : 0;
  for (int i = 0; i < C->n_levels; ++i) P.scale[i] = C->scale_factors[i];
  HIP_TRY(orb_k_grid_build(m->dKeys.as<orb_keypoint_t>(), m->dNKeys.as<int32_t>(), N, P.minX,
                           P.minY, P.invW, P.invH, m->dCellStart.as<int32_t>(),
                           m->dCellIdx.as<int32_t>(), 1, s));
  HIP_TRY(orb_k_frame_proj(m->dKeys.as<orb_keypoint_t>(), m->dDesc.as<uint8_t>(),
                           C->u_right ? m->dUr.as<float>() : nullptr,
                           kp_locked ? m->dLocked.as<uint8_t>() : nullptr, N,
                           m->dA.as<orb_last_mp_t>(), m->dB.as<uint8_t>(), M,
                           m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(), &P,
                           m->dTopk.as<uint32_t>(), m->dNcand.as<int32_t>(),
                           m->dKpMatch.as<int32_t>(), m->dNMatch.as<int32_t>(), s));
  HIP_TRY(hipMemcpyAsync(kp_match, m->dKpMatch.p, (size_t)N * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nmatches, m->dNMatch.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

// ------------------------------------------------------------- SearchByBoW
orb_status_t orb_match_bow(orb_matcher_t* m, int n_kf, const uint8_t* kf_desc,
                           const float* kf_angle, const int32_t* kf_mp,
                           const uint8_t* kf_mp_bad, int kf_nodes, const uint32_t* kf_node_ids,
                           const int32_t* kf_offs, const uint32_t* kf_feats, int n_f,
                           const uint8_t* f_desc, const float* f_angle, int f_nodes,
                           const uint32_t* f_node_ids, const int32_t* f_offs,
                           const uint32_t* f_feats, float nnratio, int check_orientation,
                           int32_t* f_match, int32_t* nmatches) {
  if (!m || n_kf < 0 || n_f < 0 || kf_nodes < 0 || f_nodes < 0 || !f_match || !nmatches ||
      (kf_nodes > 0 && (!kf_node_ids || !kf_offs)) || (f_nodes > 0 && (!f_node_ids || !f_offs)))
    return ORB_EINVAL;
  *nmatches = 0;
  for (int j = 0; j < n_f; ++j) f_match[j] = -1;
  if (n_kf == 0 || n_f == 0 || kf_nodes == 0 || f_nodes == 0) return ORB_OK;
  const int nKfFeats = kf_offs[kf_nodes], nFFeats = f_offs[f_nodes];
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  orb_status_t st;
  if ((st = upload(m->dBowA, kf_desc, (size_t)n_kf * 32, s))) return st;
  if ((st = upload(m->dBowB, kf_angle, (size_t)n_kf * 4, s))) return st;
  if ((st = upload(m->dBowC, kf_mp, (size_t)n_kf * 4, s))) return st;
  if (kf_mp_bad && (st = upload(m->dBowD, kf_mp_bad, (size_t)n_kf, s))) return st;
  if ((st = upload(m->dBowE, kf_node_ids, (size_t)kf_nodes * 4, s))) return st;
  if ((st = upload(m->dBowF, kf_offs, (size_t)(kf_nodes + 1) * 4, s))) return st;
  if ((st = upload(m->dBowG, kf_feats, (size_t)nKfFeats * 4, s))) return st;
  if ((st = upload(m->dDesc, f_desc, (size_t)n_f * 32, s))) return st;
  if ((st = upload(m->dBowH, f_angle, (size_t)n_f * 4, s))) return st;
  if ((st = upload(m->dBowI, f_node_ids, (size_t)f_nodes * 4, s))) return st;
  if ((st = upload(m->dBowJ, f_offs, (size_t)(f_nodes + 1) * 4, s))) return st;
  if ((st = upload(m->dBowK, f_feats, (size_t)nFFeats * 4, s))) return st;
  if ((st = m->dKpMatch.ensure((size_t)n_f * 4))) return st;
  if ((st = m->dTopk.ensure((size_t)std::max(nKfFeats, 1) * 4))) return st;
  if ((st = m->dNMatch.ensure(16))) return st;
  HIP_TRY(hipMemsetAsync(m->dKpMatch.p, 0xFF, (size_t)n_f * 4, s));
  HIP_TRY(orb_k_bow(m->dBowA.as<uint8_t>(), m->dBowB.as<float>(), m->dBowC.as<int32_t>(),
                    kf_mp_bad ? m->dBowD.as<uint8_t>() : nullptr, kf_nodes,
                    m->dBowE.as<uint32_t>(), m->dBowF.as<int32_t>(), m->dBowG.as<uint32_t>(),
                    nKfFeats, m->dDesc.as<uint8_t>(), m->dBowH.as<float>(), f_nodes,
                    m->dBowI.as<uint32_t>(), m->dBowJ.as<int32_t>(), m->dBowK.as<uint32_t>(), n_f,
                    nullptr, nullptr, 50, nnratio, check_orientation, m->dKpMatch.as<int32_t>(),
                    m->dTopk.as<int32_t>(), m->dNMatch.as<int32_t>(), s));
  HIP_TRY(hipMemcpyAsync(f_match, m->dKpMatch.p, (size_t)n_f * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nmatches, m->dNMatch.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

// ------------------------------------------------- SearchForInitialization
static orb_status_t search_init_device(orb_matcher_t* m, int P, const orb_keypoint_t* d_keys1,
                                       const uint8_t* d_desc1, const int32_t* d_n1,
                                       const orb_keypoint_t* d_keys2, const uint8_t* d_desc2,
                                       const int32_t* d_n2, int kp_stride, float min_x,
                                       float max_x, float min_y, float max_y, int window_size,
                                       float nnratio, int check_orientation, float* d_prev,
                                       int32_t* d_m12, int32_t* d_nmatches, hipStream_t s) {
  InitParamsHost ip;
  memset(&ip, 0, sizeof(ip));
  ip.minX = min_x;
  ip.minY = min_y;
  ip.invW = (float)ORB_GRID_COLS / (max_x - min_x);  // src/Frame.cc:240-241
  ip.invH = (float)ORB_GRID_ROWS / (max_y - min_y);
  ip.r = (float)window_size;
  ip.nnratio = nnratio;
  ip.checkOri = check_orientation ? 1 : 0;
  const size_t slots = (size_t)P * kp_stride;
  orb_status_t st;
  if ((st = m->dCellStart.ensure((size_t)P * (ORB_GRID_COLS * ORB_GRID_ROWS + 1) * 4))) return st;
  if ((st = m->dCellIdx.ensure(slots * 4))) return st;
  if ((st = m->dTopk.ensure(slots * orb_k_init_topk() * 4))) return st;
  if ((st = m->dList.ensure(slots * orb_k_init_list_len() * 4))) return st;
  if ((st = m->dNcand.ensure(slots * 4))) return st;
  if ((st = m->dInitQ.ensure(slots * 8))) return st;
  if ((st = m->dInitStage.ensure(slots * orb_k_init_key_size()))) return st;
  if ((st = m->dInitCounts.ensure((size_t)P * 8))) return st;
  HIP_TRY(orb_k_grid_build(d_keys2, d_n2, kp_stride, ip.minX, ip.minY, ip.invW, ip.invH,
                           m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(), P, s));
  HIP_TRY(orb_k_search_init(d_keys1, d_desc1, d_n1, d_keys2, d_desc2, d_n2, kp_stride, d_prev,
                            m->dCellStart.as<int32_t>(), m->dCellIdx.as<int32_t>(), &ip,
                            m->dInitQ.as<int32_t>(), m->dInitQ.as<int32_t>() + slots,
                            m->dInitCounts.as<int32_t>(),
                            m->dInitStage.p, m->dInitCounts.as<int32_t>() + P,
                            m->dTopk.as<uint32_t>(), m->dList.as<uint32_t>(),
                            m->dNcand.as<int32_t>(), d_m12, d_nmatches, P, s));
  return ORB_OK;
}

static bool init_stride_ok(int kp_stride) {
  return kp_stride > 0 && kp_stride < (1 << 19) && orb_k_init_lds(kp_stride) <= 160 * 1024;
}

orb_status_t orb_search_for_initialization(orb_matcher_t* m, const orb_frame_t* f1,
                                           const orb_frame_t* f2, float* prev_matched,
                                           int window_size, float nnratio,
                                           int check_orientation, int32_t* matches12,
                                           int32_t* nmatches) {
  if (!m || !f1 || !f2 || !nmatches || f1->n < 0 || f2->n < 0 ||
      (f1->n > 0 && (!f1->keys || !f1->descriptors || !prev_matched || !matches12)) ||
      (f2->n > 0 && (!f2->keys || !f2->descriptors)) || !(f2->max_x > f2->min_x) ||
      !(f2->max_y > f2->min_y))
    return ORB_EINVAL;
  *nmatches = 0;
  const int N1 = f1->n, N2 = f2->n;
  for (int i = 0; i < N1; ++i) matches12[i] = -1;
  if (N1 == 0 || N2 == 0) return ORB_OK;
  const int stride = std::max(N1, N2);
  if (!init_stride_ok(stride)) return ORB_ECAPACITY;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  orb_status_t st;
  if ((st = upload(m->dK1, f1->keys, (size_t)N1 * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(m->dD1, f1->descriptors, (size_t)N1 * 32, s))) return st;
  if ((st = upload(m->dK2, f2->keys, (size_t)N2 * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(m->dD2, f2->descriptors, (size_t)N2 * 32, s))) return st;
  if ((st = upload(m->dPrev, prev_matched, (size_t)N1 * 8, s))) return st;
  const int32_t ns[2] = {N1, N2};
  if ((st = upload(m->dN1, ns, 8, s))) return st;
  if ((st = m->dM12.ensure((size_t)stride * 4))) return st;
  if ((st = m->dNMatch.ensure(16))) return st;
  if ((st = search_init_device(m, 1, m->dK1.as<orb_keypoint_t>(), m->dD1.as<uint8_t>(),
                               m->dN1.as<int32_t>(), m->dK2.as<orb_keypoint_t>(),
                               m->dD2.as<uint8_t>(), m->dN1.as<int32_t>() + 1, stride, f2->min_x,
                               f2->max_x, f2->min_y, f2->max_y, window_size, nnratio,
                               check_orientation, m->dPrev.as<float>(), m->dM12.as<int32_t>(),
                               m->dNMatch.as<int32_t>(), s)))
    return st;
  HIP_TRY(hipMemcpyAsync(matches12, m->dM12.p, (size_t)N1 * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(prev_matched, m->dPrev.p, (size_t)N1 * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nmatches, m->dNMatch.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_search_for_initialization_batch(
    orb_matcher_t* m, int n_problems, const orb_keypoint_t* d_keys1, const uint8_t* d_desc1,
    const int32_t* d_n1, const orb_keypoint_t* d_keys2, const uint8_t* d_desc2,
    const int32_t* d_n2, int kp_stride, float min_x, float max_x, float min_y, float max_y,
    int window_size, float nnratio, int check_orientation, float* d_prev_matched,
    int32_t* d_matches12, int32_t* d_nmatches, void* stream) {
  if (!m || n_problems < 0 || !(max_x > min_x) || !(max_y > min_y)) return ORB_EINVAL;
  if (n_problems == 0) return ORB_OK;
  if (!d_keys1 || !d_desc1 || !d_n1 || !d_keys2 || !d_desc2 || !d_n2 || !d_prev_matched ||
      !d_matches12 || !d_nmatches || n_problems > 65535)
    return ORB_EINVAL;
  if (!init_stride_ok(kp_stride)) return kp_stride <= 0 ? ORB_EINVAL : ORB_ECAPACITY;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  return search_init_device(m, n_problems, d_keys1, d_desc1, d_n1, d_keys2, d_desc2, d_n2,
                            kp_stride, min_x, max_x, min_y, max_y, window_size, nnratio,
                            check_orientation, d_prev_matched, d_matches12, d_nmatches, s);
}

// ------------------------------------------ ComputeDistinctiveDescriptors
orb_status_t orb_distinctive_descriptors(orb_matcher_t* m, int n_mp, const int32_t* obs_offs,
                                         const uint8_t* obs_desc, int32_t* best_idx,
                                         uint8_t* descriptors) {
  if (!m || n_mp < 0 || (n_mp > 0 && (!obs_offs || !best_idx))) return ORB_EINVAL;
  if (n_mp == 0) return ORB_OK;
  if (obs_offs[0] != 0) return ORB_EINVAL;
  for (int i = 0; i < n_mp; ++i)
    if (obs_offs[i + 1] < obs_offs[i]) return ORB_EINVAL;
  const size_t nobs = (size_t)obs_offs[n_mp];
  if (nobs > 0 && !obs_desc) return ORB_EINVAL;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  orb_status_t st;
  if ((st = upload(m->dOffs, obs_offs, (size_t)(n_mp + 1) * 4, s))) return st;
  if ((st = upload(m->dObsDesc, obs_desc, nobs * 32, s))) return st;
  if ((st = m->dBest.ensure((size_t)n_mp * 4))) return st;
  if (descriptors && (st = upload(m->dBestDesc, descriptors, (size_t)n_mp * 32, s))) return st;
  HIP_TRY(orb_k_distinctive(m->dOffs.as<int32_t>(), m->dObsDesc.as<uint8_t>(), n_mp,
                            m->dBest.as<int32_t>(),
                            descriptors ? m->dBestDesc.as<uint8_t>() : nullptr, s));
  HIP_TRY(hipMemcpyAsync(best_idx, m->dBest.p, (size_t)n_mp * 4, hipMemcpyDeviceToHost, s));
  if (descriptors)
    HIP_TRY(hipMemcpyAsync(descriptors, m->dBestDesc.p, (size_t)n_mp * 32, hipMemcpyDeviceToHost,
                           s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_distinctive_descriptors_batch(orb_matcher_t* m, int n_mp,
                                               const int32_t* d_obs_offs,
                                               const uint8_t* d_obs_desc, int32_t* d_best_idx,
                                               uint8_t* d_descriptors, void* stream) {
  if (!m || n_mp < 0) return ORB_EINVAL;
  if (n_mp == 0) return ORB_OK;
  if (!d_obs_offs || !d_obs_desc || !d_best_idx) return ORB_EINVAL;
  hipSetDevice(m->device);
  HIP_TRY(orb_k_distinctive(d_obs_offs, d_obs_desc, n_mp, d_best_idx, d_descriptors,
                            stream ? (hipStream_t)stream : m->stream));
  return ORB_OK;
}

// ------------------------------------------- projection-window ORBmatcher variants
// Host-side pose algebra of the reference, in the pinned arithmetic of
// oracle/orb_oracle.cpp (cv::Mat products as float dots left to right,
// scalar scaling through double, norms/dots accumulated in double).
static void rt_xform(const float* R, const float* t, const float* P, float* o) {
  for (int r = 0; r < 3; ++r)
    o[r] = ((R[3 * r] * P[0] + R[3 * r + 1] * P[1]) + R[3 * r + 2] * P[2]) + t[r];
}

static void rt_center(const float* R, const float* t, float* Ow) {  // -R^T t
  for (int i = 0; i < 3; ++i) Ow[i] = -((R[i] * t[0] + R[3 + i] * t[1]) + R[6 + i] * t[2]);
}

static void sim3_normalise(const float* S, float* R, float* t, float* Ow) {
  double ss = 0.0;
  for (int k = 0; k < 3; ++k) ss += (double)S[k] * S[k];
  const float scw = (float)sqrt(ss);  // sqrt(sRcw.row(0).dot(sRcw.row(0))) (:320)
  const double inv = 1.0 / (double)scw;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) R[3 * r + c] = (float)((double)S[4 * r + c] * inv);
    t[r] = (float)((double)S[4 * r + 3] * inv);
  }
  rt_center(R, t, Ow);
}

static orb_status_t pp_base(PPParamsHost& P, const orb_frame_t* K, const orb_camera_t* cam,
                            float logScale, float th, int thr) {
  memset(&P, 0, sizeof(P));
  if (!K || !cam || K->n_levels <= 0 || K->n_levels > ORB_MAX_LEVELS || !K->scale_factors ||
      !(K->max_x > K->min_x) || !(K->max_y > K->min_y))
    return ORB_EINVAL;
  P.fx = cam->fx; P.fy = cam->fy; P.cx = cam->cx; P.cy = cam->cy; P.bf = cam->bf;
  P.minX = K->min_x; P.maxX = K->max_x; P.minY = K->min_y; P.maxY = K->max_y;
  P.invW = (float)ORB_GRID_COLS / (K->max_x - K->min_x);
  P.invH = (float)ORB_GRID_ROWS / (K->max_y - K->min_y);
  P.th = th;
  P.logScale = logScale;
  P.nLevels = K->n_levels;
  P.thr = thr;
  for (int l = 0; l < K->n_levels; ++l) P.scale[l] = K->scale_factors[l];
  return ORB_OK;
}

// upload the searched (key)frame and build its grid; slots 0..3
static orb_status_t pp_frame(orb_matcher_t* m, const orb_frame_t* K, const PPParamsHost& P,
                             int slot, hipStream_t s) {
  orb_status_t st;
  const int n = K->n;
  if (n > 0 && (!K->keys || !K->descriptors)) return ORB_EINVAL;
  if ((st = upload(m->sx[slot], K->keys, (size_t)n * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(m->sx[slot + 1], K->descriptors, (size_t)n * 32, s))) return st;
  if ((st = upload(m->sx[slot + 2], &n, 4, s))) return st;
  if ((st = m->sx[slot + 3].ensure(((size_t)(ORB_GRID_COLS * ORB_GRID_ROWS + 1) + n + 1) * 4)))
    return st;
  int32_t* cs = m->sx[slot + 3].as<int32_t>();
  HIP_TRY(orb_k_grid_build(m->sx[slot].as<orb_keypoint_t>(), m->sx[slot + 2].as<int32_t>(),
                           std::max(n, 1), P.minX, P.minY, P.invW, P.invH, cs,
                           cs + ORB_GRID_COLS * ORB_GRID_ROWS + 1, 1, s));
  return ORB_OK;
}

static int32_t* pp_cells(orb_matcher_t* m, int slot) { return m->sx[slot + 3].as<int32_t>(); }
static int32_t* pp_cellidx(orb_matcher_t* m, int slot) {
  return m->sx[slot + 3].as<int32_t>() + ORB_GRID_COLS * ORB_GRID_ROWS + 1;
}

// Per-point matching of n_mp map points into the frame at `slot`; claiming
// modes replay the first-come order into kp_match (host in/out, nkeys).
static orb_status_t pp_run(orb_matcher_t* m, int mode, const PPParamsHost& P, int slot,
                           const orb_frame_t* K, const uint8_t* kpLocked, int n_mp,
                           const orb_map_point_t* mps, const uint8_t* valid,
                           const uint8_t* skip, const uint8_t* mpDesc, const float* mpAngle,
                           int32_t* best_host, int32_t* kp_match_host, int32_t* count_host,
                           hipStream_t s, int32_t* best_dev = nullptr) {
  orb_status_t st;
  const bool claims = mode <= 1;
  if (n_mp > 0 && (!mps || !mpDesc)) return ORB_EINVAL;
  if ((st = upload(m->sx[8], mps, (size_t)n_mp * sizeof(orb_map_point_t), s))) return st;
  if ((st = upload(m->sx[9], mpDesc, (size_t)n_mp * 32, s))) return st;
  if (valid && (st = upload(m->sx[10], valid, (size_t)n_mp, s))) return st;
  if (skip && (st = upload(m->sx[11], skip, (size_t)n_mp, s))) return st;
  if (mpAngle && (st = upload(m->sx[12], mpAngle, (size_t)n_mp * 4, s))) return st;
  if (K->u_right && (st = upload(m->sx[13], K->u_right, (size_t)K->n * 4, s))) return st;
  if ((st = m->sx[14].ensure((size_t)std::max(n_mp, 1) * orb_k_pp_rec_size()))) return st;
  if ((st = m->sx[15].ensure((size_t)std::max(n_mp, 1) * 16))) return st;   // topk
  if ((st = m->sx[16].ensure((size_t)std::max(n_mp, 1) * 4))) return st;    // ncand
  int32_t* best = best_dev;
  if (!best) {
    if ((st = m->sx[17].ensure((size_t)std::max(n_mp, 1) * 4))) return st;
    best = m->sx[17].as<int32_t>();
  }
  HIP_TRY(orb_k_pp_match(mode, m->sx[8].as<orb_map_point_t>(),
                         valid ? m->sx[10].as<uint8_t>() : nullptr,
                         skip ? m->sx[11].as<uint8_t>() : nullptr, m->sx[9].as<uint8_t>(), n_mp,
                         m->sx[slot].as<orb_keypoint_t>(), m->sx[slot + 1].as<uint8_t>(),
                         K->u_right ? m->sx[13].as<float>() : nullptr, pp_cells(m, slot),
                         pp_cellidx(m, slot), &P, m->sx[14].p, best, m->sx[15].as<uint32_t>(),
                         m->sx[16].as<int32_t>(), s));
  if (claims) {
    const size_t lds = orb_k_pp_resolve_lds(K->n, n_mp);
    if (lds > 160 * 1024) return ORB_ECAPACITY;
    if (kpLocked && (st = upload(m->sx[18], kpLocked, (size_t)K->n, s))) return st;
    if ((st = upload(m->sx[19], kp_match_host, (size_t)K->n * 4, s))) return st;
    if ((st = m->sx[20].ensure(16))) return st;
    HIP_TRY(orb_k_pp_resolve(m->sx[slot].as<orb_keypoint_t>(), m->sx[slot + 1].as<uint8_t>(),
                             K->n, kpLocked ? m->sx[18].as<uint8_t>() : nullptr,
                             m->sx[9].as<uint8_t>(), mpAngle ? m->sx[12].as<float>() : nullptr,
                             n_mp, pp_cells(m, slot), pp_cellidx(m, slot), &P, m->sx[14].p,
                             m->sx[15].as<uint32_t>(), m->sx[16].as<int32_t>(),
                             m->sx[19].as<int32_t>(), m->sx[20].as<int32_t>(), s));
    HIP_TRY(hipMemcpyAsync(kp_match_host, m->sx[19].p, (size_t)K->n * 4, hipMemcpyDeviceToHost,
                           s));
    HIP_TRY(hipMemcpyAsync(count_host, m->sx[20].p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(stream_wait(s));
  } else if (best_host) {
    HIP_TRY(hipMemcpyAsync(best_host, best, (size_t)n_mp * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(stream_wait(s));
    int c = 0;
    for (int i = 0; i < n_mp; ++i) c += best_host[i] >= 0;
    *count_host = c;
  }
  return ORB_OK;
}

orb_status_t orb_search_by_projection_reloc(orb_matcher_t* m, const orb_frame_t* frame,
                                            const uint8_t* kp_locked, const orb_pose_t* pose,
                                            const orb_camera_t* cam, float log_scale_factor,
                                            int n_mp, const orb_map_point_t* mps,
                                            const uint8_t* mp_desc, const float* kf_angle,
                                            float th, int orb_dist, int check_orientation,
                                            int32_t* kp_match, int32_t* nmatches) {
  if (!m || !frame || !pose || !nmatches || n_mp < 0 || frame->n < 0 ||
      (frame->n > 0 && !kp_match) || (n_mp > 0 && check_orientation && !kf_angle))
    return ORB_EINVAL;
  PPParamsHost P;
  orb_status_t st = pp_base(P, frame, cam, log_scale_factor, th, orb_dist);
  if (st) return st;
  memcpy(P.R, pose->rcw, sizeof(P.R));
  memcpy(P.t, pose->tcw, sizeof(P.t));
  memcpy(P.Ow, pose->ow, sizeof(P.Ow));
  P.checkOri = check_orientation ? 1 : 0;
  *nmatches = 0;
  for (int j = 0; j < frame->n; ++j) kp_match[j] = -1;
  if (frame->n == 0 || n_mp == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  if ((st = pp_frame(m, frame, P, 0, s))) return st;
  return pp_run(m, 0, P, 0, frame, kp_locked, n_mp, mps, nullptr, nullptr, mp_desc,
                check_orientation ? kf_angle : nullptr, nullptr, kp_match, nmatches, s);
}

orb_status_t orb_search_by_projection_sim3(orb_matcher_t* m, const orb_frame_t* kf,
                                           const float* scw, const orb_camera_t* cam,
                                           float log_scale_factor, int n_mp,
                                           const orb_map_point_t* mps, const uint8_t* mp_desc,
                                           float th, int32_t* kp_matched, int32_t* nmatches) {
  if (!m || !kf || !scw || !nmatches || n_mp < 0 || kf->n < 0 || (kf->n > 0 && !kp_matched))
    return ORB_EINVAL;
  PPParamsHost P;
  orb_status_t st = pp_base(P, kf, cam, log_scale_factor, th, 50);
  if (st) return st;
  sim3_normalise(scw, P.R, P.t, P.Ow);
  *nmatches = 0;
  if (kf->n == 0 || n_mp == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  if ((st = pp_frame(m, kf, P, 0, s))) return st;
  return pp_run(m, 1, P, 0, kf, nullptr, n_mp, mps, nullptr, nullptr, mp_desc, nullptr, nullptr,
                kp_matched, nmatches, s);
}

orb_status_t orb_fuse(orb_matcher_t* m, const orb_frame_t* kf, const float* inv_level_sigma2,
                      const orb_pose_t* pose, const orb_camera_t* cam, float log_scale_factor,
                      int n_mp, const orb_map_point_t* mps, const uint8_t* mp_desc, float th,
                      int32_t* fuse_idx, int32_t* n_fuse) {
  if (!m || !kf || !pose || !inv_level_sigma2 || !n_fuse || n_mp < 0 || kf->n < 0 ||
      (n_mp > 0 && !fuse_idx))
    return ORB_EINVAL;
  PPParamsHost P;
  orb_status_t st = pp_base(P, kf, cam, log_scale_factor, th, 50);
  if (st) return st;
  memcpy(P.R, pose->rcw, sizeof(P.R));
  memcpy(P.t, pose->tcw, sizeof(P.t));
  memcpy(P.Ow, pose->ow, sizeof(P.Ow));
  for (int l = 0; l < kf->n_levels; ++l) P.invSigma2[l] = inv_level_sigma2[l];
  *n_fuse = 0;
  for (int i = 0; i < n_mp; ++i) fuse_idx[i] = -1;
  if (kf->n == 0 || n_mp == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  if ((st = pp_frame(m, kf, P, 0, s))) return st;
  return pp_run(m, 2, P, 0, kf, nullptr, n_mp, mps, nullptr, nullptr, mp_desc, nullptr,
                fuse_idx, nullptr, n_fuse, s);
}

orb_status_t orb_fuse_sim3(orb_matcher_t* m, const orb_frame_t* kf, const float* scw,
                           const orb_camera_t* cam, float log_scale_factor, int n_mp,
                           const orb_map_point_t* mps, const uint8_t* mp_desc, float th,
                           int32_t* fuse_idx, int32_t* n_fuse) {
  if (!m || !kf || !scw || !n_fuse || n_mp < 0 || kf->n < 0 || (n_mp > 0 && !fuse_idx))
    return ORB_EINVAL;
  PPParamsHost P;
  orb_status_t st = pp_base(P, kf, cam, log_scale_factor, th, 50);
  if (st) return st;
  sim3_normalise(scw, P.R, P.t, P.Ow);
  *n_fuse = 0;
  for (int i = 0; i < n_mp; ++i) fuse_idx[i] = -1;
  if (kf->n == 0 || n_mp == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  if ((st = pp_frame(m, kf, P, 0, s))) return st;
  return pp_run(m, 3, P, 0, kf, nullptr, n_mp, mps, nullptr, nullptr, mp_desc, nullptr,
                fuse_idx, nullptr, n_fuse, s);
}

orb_status_t orb_search_by_sim3(orb_matcher_t* m, const orb_frame_t* kf1, const orb_frame_t* kf2,
                                float log_scale_factor, const orb_camera_t* cam,
                                const float* r1w, const float* t1w, const float* r2w,
                                const float* t2w, const orb_map_point_t* mps1,
                                const uint8_t* valid1, const uint8_t* already1,
                                const uint8_t* mp_desc1, const orb_map_point_t* mps2,
                                const uint8_t* valid2, const uint8_t* already2,
                                const uint8_t* mp_desc2, float s12, const float* r12,
                                const float* t12, float th, int32_t* match12,
                                int32_t* nfound) {
  if (!m || !kf1 || !kf2 || !r1w || !t1w || !r2w || !t2w || !r12 || !t12 || !nfound ||
      kf1->n < 0 || kf2->n < 0 || (kf1->n > 0 && (!mps1 || !valid1 || !mp_desc1 || !match12)) ||
      (kf2->n > 0 && (!mps2 || !valid2 || !mp_desc2)))
    return ORB_EINVAL;
  PPParamsHost P1, P2;  // P1: KF1 points into KF2, P2: KF2 points into KF1
  orb_status_t st;
  if ((st = pp_base(P1, kf2, cam, log_scale_factor, th, 100))) return st;
  if ((st = pp_base(P2, kf1, cam, log_scale_factor, th, 100))) return st;
  float sR12[9], sR21[9], t21[3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      sR12[3 * r + c] = (float)((double)s12 * (double)r12[3 * r + c]);
      sR21[3 * r + c] = (float)((1.0 / (double)s12) * (double)r12[3 * c + r]);
    }
  for (int r = 0; r < 3; ++r)  // t21 = -sR21 * t12 (:1235)
    t21[r] = -((sR21[3 * r] * t12[0] + sR21[3 * r + 1] * t12[1]) + sR21[3 * r + 2] * t12[2]);
  memcpy(P1.R, r1w, 36); memcpy(P1.t, t1w, 12); memcpy(P1.R2, sR21, 36); memcpy(P1.t2, t21, 12);
  memcpy(P2.R, r2w, 36); memcpy(P2.t, t2w, 12); memcpy(P2.R2, sR12, 36); memcpy(P2.t2, t12, 12);
  *nfound = 0;
  for (int i = 0; i < kf1->n; ++i) match12[i] = -1;
  if (kf1->n == 0 || kf2->n == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  if ((st = pp_frame(m, kf2, P1, 0, s))) return st;
  if ((st = pp_frame(m, kf1, P2, 4, s))) return st;
  if ((st = m->sx[21].ensure((size_t)kf1->n * 4))) return st;
  if ((st = m->sx[22].ensure((size_t)kf2->n * 4))) return st;
  if ((st = m->sx[23].ensure((size_t)kf1->n * 4 + 16))) return st;
  // direction 1 runs to completion before its point buffers are reused
  if ((st = pp_run(m, 4, P1, 0, kf2, nullptr, kf1->n, mps1, valid1, already1, mp_desc1, nullptr,
                   nullptr, nullptr, nullptr, s, m->sx[21].as<int32_t>())))
    return st;
  HIP_TRY(stream_wait(s));
  if ((st = pp_run(m, 4, P2, 4, kf1, nullptr, kf2->n, mps2, valid2, already2, mp_desc2, nullptr,
                   nullptr, nullptr, nullptr, s, m->sx[22].as<int32_t>())))
    return st;
  int32_t* out = m->sx[23].as<int32_t>();
  HIP_TRY(orb_k_sim3_mutual(m->sx[21].as<int32_t>(), kf1->n, m->sx[22].as<int32_t>(), out,
                            out + kf1->n, s));
  HIP_TRY(hipMemcpyAsync(match12, out, (size_t)kf1->n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nfound, out + kf1->n, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_match_bow_kf(orb_matcher_t* m, int n1, const uint8_t* desc1,
                              const float* angle1, const int32_t* mp1, const uint8_t* mp1_bad,
                              int nodes1, const uint32_t* node_ids1, const int32_t* offs1,
                              const uint32_t* feats1, int n2, const uint8_t* desc2,
                              const float* angle2, const int32_t* mp2, const uint8_t* mp2_bad,
                              int nodes2, const uint32_t* node_ids2, const int32_t* offs2,
                              const uint32_t* feats2, float nnratio, int check_orientation,
                              int32_t* match12, int32_t* nmatches) {
  if (!m || n1 < 0 || n2 < 0 || nodes1 < 0 || nodes2 < 0 || !nmatches ||
      (n1 > 0 && (!desc1 || !angle1 || !mp1 || !match12)) ||
      (n2 > 0 && (!desc2 || !angle2 || !mp2)) || (nodes1 > 0 && (!node_ids1 || !offs1)) ||
      (nodes2 > 0 && (!node_ids2 || !offs2)))
    return ORB_EINVAL;
  *nmatches = 0;
  for (int i = 0; i < n1; ++i) match12[i] = -1;
  if (n1 == 0 || n2 == 0 || nodes1 == 0 || nodes2 == 0) return ORB_OK;
  if ((size_t)4 * ((n2 + 31) / 32) * 4 > 65536) return ORB_ECAPACITY;
  const int nF1 = offs1[nodes1], nF2 = offs2[nodes2];
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  orb_status_t st;
  DevBuf* b = m->sx;
  if ((st = upload(b[0], desc1, (size_t)n1 * 32, s))) return st;
  if ((st = upload(b[1], angle1, (size_t)n1 * 4, s))) return st;
  if ((st = upload(b[2], mp1, (size_t)n1 * 4, s))) return st;
  if (mp1_bad && (st = upload(b[3], mp1_bad, (size_t)n1, s))) return st;
  if ((st = upload(b[4], node_ids1, (size_t)nodes1 * 4, s))) return st;
  if ((st = upload(b[5], offs1, (size_t)(nodes1 + 1) * 4, s))) return st;
  if ((st = upload(b[6], feats1, (size_t)nF1 * 4, s))) return st;
  if ((st = upload(b[7], desc2, (size_t)n2 * 32, s))) return st;
  if ((st = upload(b[8], angle2, (size_t)n2 * 4, s))) return st;
  if ((st = upload(b[9], mp2, (size_t)n2 * 4, s))) return st;
  if (mp2_bad && (st = upload(b[10], mp2_bad, (size_t)n2, s))) return st;
  if ((st = upload(b[11], node_ids2, (size_t)nodes2 * 4, s))) return st;
  if ((st = upload(b[12], offs2, (size_t)(nodes2 + 1) * 4, s))) return st;
  if ((st = upload(b[13], feats2, (size_t)nF2 * 4, s))) return st;
  if ((st = b[14].ensure((size_t)n1 * 4))) return st;
  if ((st = b[15].ensure((size_t)std::max(nF1, 1) * 4))) return st;
  if ((st = b[16].ensure(16))) return st;
  HIP_TRY(hipMemsetAsync(b[14].p, 0xFF, (size_t)n1 * 4, s));
  HIP_TRY(orb_k_bow(b[0].as<uint8_t>(), b[1].as<float>(), b[2].as<int32_t>(),
                    mp1_bad ? b[3].as<uint8_t>() : nullptr, nodes1, b[4].as<uint32_t>(),
                    b[5].as<int32_t>(), b[6].as<uint32_t>(), nF1, b[7].as<uint8_t>(),
                    b[8].as<float>(), nodes2, b[11].as<uint32_t>(), b[12].as<int32_t>(),
                    b[13].as<uint32_t>(), n2, b[9].as<int32_t>(),
                    mp2_bad ? b[10].as<uint8_t>() : nullptr, 49, nnratio, check_orientation,
                    b[14].as<int32_t>(), b[15].as<int32_t>(), b[16].as<int32_t>(), s));
  HIP_TRY(hipMemcpyAsync(match12, b[14].p, (size_t)n1 * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nmatches, b[16].p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_search_for_triangulation(
    orb_matcher_t* m, const orb_frame_t* kf1, const uint8_t* has_mp1, const orb_frame_t* kf2,
    const uint8_t* has_mp2, const float* level_sigma2, const float* f12,
    const orb_camera_t* cam, const float* cw, const float* r2w, const float* t2w, int nodes1,
    const uint32_t* node_ids1, const int32_t* offs1, const uint32_t* feats1, int nodes2,
    const uint32_t* node_ids2, const int32_t* offs2, const uint32_t* feats2, int only_stereo,
    int check_orientation, int32_t* match12, int32_t* nmatches) {
  if (!m || !kf1 || !kf2 || !level_sigma2 || !f12 || !cam || !cw || !r2w || !t2w || !nmatches ||
      kf1->n < 0 || kf2->n < 0 || nodes1 < 0 || nodes2 < 0 || !kf2->scale_factors ||
      kf2->n_levels <= 0 || kf2->n_levels > ORB_MAX_LEVELS ||
      (kf1->n > 0 && (!kf1->keys || !kf1->descriptors || !has_mp1 || !match12)) ||
      (kf2->n > 0 && (!kf2->keys || !kf2->descriptors || !has_mp2)) ||
      (nodes1 > 0 && (!node_ids1 || !offs1)) || (nodes2 > 0 && (!node_ids2 || !offs2)))
    return ORB_EINVAL;
  TriParamsHost T;
  memset(&T, 0, sizeof(T));
  memcpy(T.F, f12, sizeof(T.F));
  float C2[3];
  rt_xform(r2w, t2w, cw, C2);  // epipole of KF1 in KF2 (:728-733)
  const float invz = 1.0f / C2[2];
  T.ex = cam->fx * C2[0] * invz + cam->cx;
  T.ey = cam->fy * C2[1] * invz + cam->cy;
  T.onlyStereo = only_stereo ? 1 : 0;
  T.checkOri = check_orientation ? 1 : 0;
  for (int l = 0; l < kf2->n_levels; ++l) {
    T.scale[l] = kf2->scale_factors[l];
    T.sigma2[l] = level_sigma2[l];
  }
  *nmatches = 0;
  for (int i = 0; i < kf1->n; ++i) match12[i] = -1;
  if (kf1->n == 0 || kf2->n == 0 || nodes1 == 0 || nodes2 == 0) return ORB_OK;
  const int nF1 = offs1[nodes1], nF2 = offs2[nodes2];
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  orb_status_t st;
  DevBuf* b = m->sx;
  const int n1 = kf1->n, n2 = kf2->n;
  if ((st = upload(b[0], kf1->keys, (size_t)n1 * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(b[1], kf1->descriptors, (size_t)n1 * 32, s))) return st;
  if (kf1->u_right && (st = upload(b[2], kf1->u_right, (size_t)n1 * 4, s))) return st;
  if ((st = upload(b[3], has_mp1, (size_t)n1, s))) return st;
  if ((st = upload(b[4], node_ids1, (size_t)nodes1 * 4, s))) return st;
  if ((st = upload(b[5], offs1, (size_t)(nodes1 + 1) * 4, s))) return st;
  if ((st = upload(b[6], feats1, (size_t)nF1 * 4, s))) return st;
  if ((st = upload(b[7], kf2->keys, (size_t)n2 * sizeof(orb_keypoint_t), s))) return st;
  if ((st = upload(b[8], kf2->descriptors, (size_t)n2 * 32, s))) return st;
  if (kf2->u_right && (st = upload(b[9], kf2->u_right, (size_t)n2 * 4, s))) return st;
  if ((st = upload(b[10], has_mp2, (size_t)n2, s))) return st;
  if ((st = upload(b[11], node_ids2, (size_t)nodes2 * 4, s))) return st;
  if ((st = upload(b[12], offs2, (size_t)(nodes2 + 1) * 4, s))) return st;
  if ((st = upload(b[13], feats2, (size_t)nF2 * 4, s))) return st;
  if ((st = b[14].ensure((size_t)n1 * 4))) return st;
  if ((st = b[15].ensure((size_t)std::max(nF1, 1) * 4))) return st;
  if ((st = b[16].ensure(16))) return st;
  HIP_TRY(hipMemsetAsync(b[14].p, 0xFF, (size_t)n1 * 4, s));
  HIP_TRY(orb_k_triangulation(
      b[0].as<orb_keypoint_t>(), b[1].as<uint8_t>(), kf1->u_right ? b[2].as<float>() : nullptr,
      b[3].as<uint8_t>(), nodes1, b[4].as<uint32_t>(), b[5].as<int32_t>(), b[6].as<uint32_t>(),
      nF1, b[7].as<orb_keypoint_t>(), b[8].as<uint8_t>(),
      kf2->u_right ? b[9].as<float>() : nullptr, b[10].as<uint8_t>(), nodes2,
      b[11].as<uint32_t>(), b[12].as<int32_t>(), b[13].as<uint32_t>(), &T, b[14].as<int32_t>(),
      b[15].as<int32_t>(), b[16].as<int32_t>(), s));
  HIP_TRY(hipMemcpyAsync(match12, b[14].p, (size_t)n1 * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nmatches, b[16].p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

// ------------------------------------------------------- DBoW2 vocabulary
// TemplatedVocabulary<FORB::TDescriptor, FORB> as loaded by loadFromTextFile
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1362-1448) and its transform
// (:1128-1283), the producer of Frame/KeyFrame::mBowVec and mFeatVec
// (src/Frame.cc:439-449, src/KeyFrame.cc:60-71).  The tree lives on the
// device, renumbered breadth-first (vocab_kernels.hip).
struct orb_vocabulary {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  int k = 0, L = 0, scoring = 0, weighting = 0, nNodes = 0, nWords = 0;
  DevBuf dInfo, dDesc, dWord, dWeight, dOrig;
  DevBuf dIn, dCounts, dFWord, dFWeight, dFNode, dBowW, dBowV, dNW, dFvN, dFvO, dFvF, dNFv;
};

static orb_status_t vocab_build(orb_vocabulary* V, int n_nodes, const int32_t* parent,
                                const uint8_t* leaf, const uint8_t* desc, const double* weight) {
  // children in creation order (m_nodes[pid].children.push_back(nid), :1416)
  std::vector<int32_t> ccount(n_nodes, 0), cstart(n_nodes + 1, 0), clist(std::max(n_nodes - 1, 1));
  for (int i = 1; i < n_nodes; ++i) {
    if (parent[i] < 0 || parent[i] >= i) return ORB_EINVAL;
    ++ccount[parent[i]];
  }
  for (int i = 0; i < n_nodes; ++i) cstart[i + 1] = cstart[i] + ccount[i];
  {
    std::vector<int32_t> fill(cstart.begin(), cstart.end() - 1);
    for (int i = 1; i < n_nodes; ++i) clist[fill[parent[i]]++] = i;
  }
  // word ids: leaf-flagged nodes in file order (:1432-1439); others keep 0 (Node())
  std::vector<uint32_t> wordOf(n_nodes, 0);
  int nw = 0;
  for (int i = 1; i < n_nodes; ++i)
    if (leaf[i]) wordOf[i] = (uint32_t)nw++;
  // breadth-first renumbering: children of the node at position p occupy
  // consecutive positions, in child order
  struct Info { int32_t first, count; };
  std::vector<Info> info(n_nodes);
  std::vector<int32_t> orig(n_nodes);
  std::vector<uint8_t> ddesc((size_t)n_nodes * 32);
  std::vector<uint32_t> dword(n_nodes);
  std::vector<double> dweight(n_nodes);
  orig[0] = 0;
  int next = 1;
  for (int p = 0; p < n_nodes; ++p) {
    const int id = orig[p];
    info[p].first = next;
    info[p].count = ccount[id];
    for (int c = cstart[id]; c < cstart[id + 1]; ++c) orig[next++] = clist[c];
    memcpy(&ddesc[(size_t)p * 32], desc + (size_t)id * 32, 32);
    dword[p] = wordOf[id];
    dweight[p] = id == 0 ? 0.0 : weight[id];
  }
  if (next != n_nodes) return ORB_EINVAL;
  V->nNodes = n_nodes;
  V->nWords = nw;
  hipStream_t s = V->stream;
  orb_status_t st;
  if ((st = upload(V->dInfo, info.data(), info.size() * sizeof(Info), s))) return st;
  if ((st = upload(V->dDesc, ddesc.data(), ddesc.size(), s))) return st;
  if ((st = upload(V->dWord, dword.data(), dword.size() * 4, s))) return st;
  if ((st = upload(V->dWeight, dweight.data(), dweight.size() * 8, s))) return st;
  if ((st = upload(V->dOrig, orig.data(), orig.size() * 4, s))) return st;
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

static orb_status_t vocab_new(int device, int k, int L, int scoring, int weighting,
                              orb_vocabulary** out) {
  orb_status_t st = check_device(device);
  if (st) return st;
  orb_vocabulary* V = new orb_vocabulary();
  V->device = device;
  V->k = k; V->L = L; V->scoring = scoring; V->weighting = weighting;
  hipSetDevice(device);
  if (create_own_stream(&V->stream) != hipSuccess) {
    delete V;
    return ORB_EDEVICE;
  }
  *out = V;
  return ORB_OK;
}

orb_status_t orb_vocabulary_create(int device, int k, int L, int scoring, int weighting,
                                   int n_nodes, const int32_t* parent, const uint8_t* leaf_flag,
                                   const uint8_t* descriptors, const double* weights,
                                   orb_vocabulary_t** out) {
  if (!out) return ORB_EINVAL;
  *out = nullptr;
  // loadFromTextFile's header check (:1383)
  if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 ||
      weighting > 3 || n_nodes < 1 ||
      (n_nodes > 1 && (!parent || !leaf_flag || !descriptors || !weights)))
    return ORB_EINVAL;
  orb_vocabulary* V = nullptr;
  orb_status_t st = vocab_new(device, k, L, scoring, weighting, &V);
  if (st) return st;
  std::vector<int32_t> p0(1, 0);
  std::vector<uint8_t> l0(1, 0), d0(32, 0);
  std::vector<double> w0(1, 0.0);
  st = n_nodes > 1 ? vocab_build(V, n_nodes, parent, leaf_flag, descriptors, weights)
                   : vocab_build(V, 1, p0.data(), l0.data(), d0.data(), w0.data());
  if (st) {
    orb_vocabulary_destroy(V);
    return st;
  }
  *out = V;
  return ORB_OK;
}

// Text format of loadFromTextFile: "k L scoring weighting", then one line per
// node "parent isLeaf d0 .. d31 weight" (descriptor bytes as integers,
// FORB::fromString FORB.cpp:120-135).  Lines without a parent field are
// skipped (the reference's eof loop turns a trailing empty line into a root
// child with an uninitialised descriptor).
orb_status_t orb_vocabulary_load_text(int device, const char* path, orb_vocabulary_t** out) {
  if (!out || !path) return ORB_EINVAL;
  *out = nullptr;
  FILE* fp = fopen(path, "rb");
  if (!fp) return ORB_EINVAL;
  std::vector<char> text;
  {
    char buf[1 << 16];
    size_t r;
    while ((r = fread(buf, 1, sizeof(buf), fp)) > 0) text.insert(text.end(), buf, buf + r);
    fclose(fp);
  }
  text.push_back('\0');
  char* c = text.data();
  char* eol = strchr(c, '\n');
  int hdr[4];
  for (int i = 0; i < 4; ++i) {
    char* e;
    const long v = strtol(c, &e, 10);
    if (e == c || (eol && e > eol)) return ORB_EINVAL;
    hdr[i] = (int)v;
    c = e;
  }
  c = eol ? eol + 1 : c + strlen(c);
  std::vector<int32_t> parent(1, 0);
  std::vector<uint8_t> leaf(1, 0), desc(32, 0);
  std::vector<double> weight(1, 0.0);
  while (*c) {
    char* le = strchr(c, '\n');
    if (le) *le = '\0';
    char* e;
    const long pid = strtol(c, &e, 10);
    if (e != c) {
      c = e;
      const long isLeaf = strtol(c, &e, 10);
      c = e;
      uint8_t d[32] = {0};
      for (int i = 0; i < 32; ++i) {
        const long v = strtol(c, &e, 10);
        if (e == c) break;
        d[i] = (uint8_t)v;
        c = e;
      }
      const double w = strtod(c, &e);
      parent.push_back((int32_t)pid);
      leaf.push_back(isLeaf > 0);
      desc.insert(desc.end(), d, d + 32);
      weight.push_back(e == c ? 0.0 : w);
    }
    if (!le) break;
    c = le + 1;
  }
  return orb_vocabulary_create(device, hdr[0], hdr[1], hdr[2], hdr[3], (int)parent.size(),
                               parent.data(), leaf.data(), desc.data(), weight.data(), out);
}

void orb_vocabulary_destroy(orb_vocabulary_t* V) {
  if (!V) return;
  hipSetDevice(V->device);
  hipStreamSynchronize(V->stream);
  DevBuf* bufs[] = {&V->dInfo, &V->dDesc, &V->dWord, &V->dWeight, &V->dOrig, &V->dIn,
                    &V->dCounts, &V->dFWord, &V->dFWeight, &V->dFNode, &V->dBowW, &V->dBowV,
                    &V->dNW, &V->dFvN, &V->dFvO, &V->dFvF, &V->dNFv};
  for (DevBuf* b : bufs) b->release();
  hipStreamDestroy(V->stream);
  delete V;
}

orb_status_t orb_vocabulary_info(const orb_vocabulary_t* V, int32_t* info6) {
  if (!V || !info6) return ORB_EINVAL;
  info6[0] = V->k; info6[1] = V->L; info6[2] = V->scoring; info6[3] = V->weighting;
  info6[4] = V->nNodes; info6[5] = V->nWords;
  return ORB_OK;
}

void* orb_vocabulary_stream(orb_vocabulary_t* V) { return V ? (void*)V->stream : nullptr; }

static orb_status_t vocab_launch(orb_vocabulary* V, int n_frames, const int32_t* d_counts,
                                 int n_single, const uint8_t* d_desc, int stride, int levelsup,
                                 uint32_t* fword, double* fweight, uint32_t* fnode,
                                 uint32_t* bw, double* bv, int32_t* nw, uint32_t* fvn,
                                 int32_t* fvo, uint32_t* fvf, int32_t* nfv, hipStream_t s) {
  int l2 = V->scoring == 1;
  const int must = V->scoring != 5;  // ScoringObject.h:74-89
  const int tf = V->weighting == 0 || V->weighting == 1;
  if (V->nWords == 0) {  // empty(): v, fv cleared (:1136-1140)
    HIP_TRY(hipMemsetAsync(nw, 0, (size_t)n_frames * 4, s));
    HIP_TRY(hipMemsetAsync(nfv, 0, (size_t)n_frames * 4, s));
    for (int f = 0; f < n_frames; ++f)
      HIP_TRY(hipMemsetAsync(fvo + (size_t)f * (stride + 1), 0, 4, s));
    return ORB_OK;
  }
  HIP_TRY(orb_k_voc_descend(V->dInfo.p, V->dDesc.p, V->dWord.as<uint32_t>(),
                            V->dWeight.as<double>(), V->dOrig.as<uint32_t>(), V->L - levelsup,
                            d_desc, d_counts, n_single, stride, n_frames, fword, fweight, fnode,
                            s));
  HIP_TRY(orb_k_voc_vectors(fword, fweight, fnode, d_counts, n_single, stride, tf, must, l2,
                            n_frames, bw, bv, nw, fvn, fvo, fvf, nfv, s));
  return ORB_OK;
}

orb_status_t orb_vocabulary_transform(orb_vocabulary_t* V, int n, const uint8_t* desc,
                                      int levelsup, uint32_t* bow_words, double* bow_values,
                                      int32_t* n_words, uint32_t* fv_nodes, int32_t* fv_offs,
                                      uint32_t* fv_feats, int32_t* n_fv_nodes,
                                      uint32_t* feat_word, uint32_t* feat_node) {
  if (!V || n < 0 || n > orb_k_voc_max_features() || (n > 0 && !desc) || !bow_words ||
      !bow_values || !n_words || !fv_nodes || !fv_offs || !fv_feats || !n_fv_nodes)
    return ORB_EINVAL;
  if (n == 0 || V->nWords == 0) {
    *n_words = 0;
    *n_fv_nodes = 0;
    fv_offs[0] = 0;
    return ORB_OK;
  }
  std::lock_guard<std::mutex> g(V->mu);
  hipSetDevice(V->device);
  hipStream_t s = V->stream;
  orb_status_t st;
  const size_t N = (size_t)n;
  if ((st = upload(V->dIn, desc, N * 32, s))) return st;
  if ((st = V->dFWord.ensure(N * 4)) || (st = V->dFWeight.ensure(N * 8)) ||
      (st = V->dFNode.ensure(N * 4)) || (st = V->dBowW.ensure(N * 4)) ||
      (st = V->dBowV.ensure(N * 8)) || (st = V->dNW.ensure(16)) || (st = V->dFvN.ensure(N * 4)) ||
      (st = V->dFvO.ensure((N + 1) * 4)) || (st = V->dFvF.ensure(N * 4)) ||
      (st = V->dNFv.ensure(16)))
    return st;
  if ((st = vocab_launch(V, 1, nullptr, n, V->dIn.as<uint8_t>(), n, levelsup,
                         V->dFWord.as<uint32_t>(), V->dFWeight.as<double>(),
                         V->dFNode.as<uint32_t>(), V->dBowW.as<uint32_t>(),
                         V->dBowV.as<double>(), V->dNW.as<int32_t>(), V->dFvN.as<uint32_t>(),
                         V->dFvO.as<int32_t>(), V->dFvF.as<uint32_t>(), V->dNFv.as<int32_t>(), s)))
    return st;
  int32_t counts[2];
  HIP_TRY(hipMemcpyAsync(&counts[0], V->dNW.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&counts[1], V->dNFv.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  *n_words = counts[0];
  *n_fv_nodes = counts[1];
  HIP_TRY(hipMemcpyAsync(bow_words, V->dBowW.p, (size_t)counts[0] * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(bow_values, V->dBowV.p, (size_t)counts[0] * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(fv_nodes, V->dFvN.p, (size_t)counts[1] * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(fv_offs, V->dFvO.p, (size_t)(counts[1] + 1) * 4, hipMemcpyDeviceToHost,
                         s));
  HIP_TRY(stream_wait(s));
  const int nfeat = fv_offs[counts[1]];
  if (nfeat > 0)
    HIP_TRY(hipMemcpyAsync(fv_feats, V->dFvF.p, (size_t)nfeat * 4, hipMemcpyDeviceToHost, s));
  if (feat_word) HIP_TRY(hipMemcpyAsync(feat_word, V->dFWord.p, N * 4, hipMemcpyDeviceToHost, s));
  if (feat_node) HIP_TRY(hipMemcpyAsync(feat_node, V->dFNode.p, N * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_vocabulary_transform_batch(orb_vocabulary_t* V, int n_frames,
                                            const int32_t* d_counts, const uint8_t* d_desc,
                                            int stride, int levelsup, uint32_t* d_feat_word,
                                            double* d_feat_weight, uint32_t* d_feat_node,
                                            uint32_t* d_bow_words, double* d_bow_values,
                                            int32_t* d_n_words, uint32_t* d_fv_nodes,
                                            int32_t* d_fv_offs, uint32_t* d_fv_feats,
                                            int32_t* d_n_fv_nodes, void* stream) {
  if (!V || n_frames < 0 || stride <= 0 || stride > orb_k_voc_max_features()) return ORB_EINVAL;
  if (n_frames == 0) return ORB_OK;
  if (!d_counts || !d_desc || !d_feat_word || !d_feat_weight || !d_feat_node || !d_bow_words ||
      !d_bow_values || !d_n_words || !d_fv_nodes || !d_fv_offs || !d_fv_feats || !d_n_fv_nodes)
    return ORB_EINVAL;
  hipSetDevice(V->device);
  return vocab_launch(V, n_frames, d_counts, 0, d_desc, stride, levelsup, d_feat_word,
                      d_feat_weight, d_feat_node, d_bow_words, d_bow_values, d_n_words,
                      d_fv_nodes, d_fv_offs, d_fv_feats, d_n_fv_nodes,
                      stream ? (hipStream_t)stream : V->stream);
}

// ------------------------------------------------------------ undistortion
// cv::undistortPoints(src, dst, mK, mDistCoef, cv::Mat(), mK) as called by
// Frame::UndistortKeyPoints / ComputeImageBounds (src/Frame.cc:452-514); the
// double parameter block of camera_kernels.hip (cvConvert of the CV_32F
// matrices, ifx = 1./fx, RR = mK * I).
struct UndistortParamsHost {
  double fx, fy, cx, cy, ifx, ify;
  double rr[9];
  double k[12];
};

static orb_status_t undistort_params(const float* K, const float* dist, int n_dist,
                                     UndistortParamsHost& P) {
  static_assert(sizeof(UndistortParamsHost) == 27 * 8, "parameter block layout");
  if (orb_k_undistort_params_size() != sizeof(UndistortParamsHost)) return ORB_EINVAL;
  if (!K || !dist || !(n_dist == 4 || n_dist == 5 || n_dist == 8 || n_dist == 12))
    return ORB_EINVAL;
  memset(&P, 0, sizeof(P));
  P.fx = K[0]; P.fy = K[4]; P.cx = K[2]; P.cy = K[5];
  P.ifx = 1. / P.fx;
  P.ify = 1. / P.fy;
  for (int i = 0; i < 9; ++i) P.rr[i] = (double)K[i];
  for (int i = 0; i < n_dist; ++i) P.k[i] = (double)dist[i];
  return ORB_OK;
}

orb_status_t orb_undistort_points(orb_matcher_t* m, int n, const float* xy, const float* K,
                                  const float* dist, int n_dist, float* out_xy) {
  if (!m || n < 0 || (n > 0 && (!xy || !out_xy))) return ORB_EINVAL;
  UndistortParamsHost P;
  orb_status_t st = undistort_params(K, dist, n_dist, P);
  if (st) return st;
  if (n == 0) return ORB_OK;
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  if ((st = upload(m->dA, xy, (size_t)n * 8, s)) || (st = m->dB.ensure((size_t)n * 8))) return st;
  HIP_TRY(orb_k_undistort_points(&P, n, m->dA.as<float>(), m->dB.as<float>(), s));
  HIP_TRY(hipMemcpyAsync(out_xy, m->dB.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_undistort_keypoints(orb_matcher_t* m, int n, const orb_keypoint_t* keys,
                                     const float* K, const float* dist, int n_dist,
                                     orb_keypoint_t* keys_un) {
  if (!m || n < 0 || (n > 0 && (!keys || !keys_un))) return ORB_EINVAL;
  UndistortParamsHost P;
  orb_status_t st = undistort_params(K, dist, n_dist, P);
  if (st) return st;
  if (n == 0) return ORB_OK;
  if (dist[0] == 0.0f) {  // mvKeysUn = mvKeys (:454-458)
    if (keys_un != keys) memmove(keys_un, keys, (size_t)n * sizeof(orb_keypoint_t));
    return ORB_OK;
  }
  std::lock_guard<std::mutex> g(m->mu);
  hipSetDevice(m->device);
  hipStream_t s = m->stream;
  CallOrder order(m->evLast, &m->lastStream, s);
  if (order.status) return order.status;
  const size_t bytes = (size_t)n * sizeof(orb_keypoint_t);
  if ((st = upload(m->dA, keys, bytes, s)) || (st = m->dB.ensure(bytes))) return st;
  HIP_TRY(orb_k_undistort_keys(&P, 1, nullptr, n, n, m->dA.p, m->dB.p, 0, s));
  HIP_TRY(hipMemcpyAsync(keys_un, m->dB.p, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return ORB_OK;
}

orb_status_t orb_compute_image_bounds(orb_matcher_t* m, int cols, int rows, const float* K,
                                      const float* dist, int n_dist, float* bounds) {
  if (!m || !bounds || cols < 0 || rows < 0) return ORB_EINVAL;
  UndistortParamsHost P;
  orb_status_t st = undistort_params(K, dist, n_dist, P);
  if (st) return st;
  if (dist[0] == 0.0f) {  // :506-512
    bounds[0] = 0.0f;
    bounds[1] = (float)cols;
    bounds[2] = 0.0f;
    bounds[3] = (float)rows;
    return ORB_OK;
  }
  const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
  float u[8];
  if ((st = orb_undistort_points(m, 4, c, K, dist, n_dist, u))) return st;
  bounds[0] = std::min(u[0], u[4]);  // mnMinX = min(mat(0,0), mat(2,0)) (:496-499)
  bounds[1] = std::max(u[2], u[6]);
  bounds[2] = std::min(u[1], u[3]);
  bounds[3] = std::max(u[5], u[7]);
  return ORB_OK;
}

orb_status_t orb_undistort_keypoints_batch(orb_matcher_t* m, int n_frames, const int32_t* d_n,
                                           const orb_keypoint_t* d_keys, int stride,
                                           const float* K, const float* dist, int n_dist,
                                           orb_keypoint_t* d_keys_un, void* stream) {
  if (!m || n_frames < 0 || stride <= 0) return ORB_EINVAL;
  UndistortParamsHost P;
  orb_status_t st = undistort_params(K, dist, n_dist, P);
  if (st) return st;
  if (n_frames == 0) return ORB_OK;
  if (!d_n || !d_keys || !d_keys_un) return ORB_EINVAL;
  hipSetDevice(m->device);
  HIP_TRY(orb_k_undistort_keys(&P, n_frames, d_n, 0, stride, d_keys, d_keys_un,
                               dist[0] == 0.0f ? 1 : 0, stream ? (hipStream_t)stream : m->stream));
  return ORB_OK;
}

// ------------------------------------------------------------ synthetic input
void orb_synth_image(uint64_t seed, int frame, int view, int width, int height, uint8_t* out,
                     size_t stride) {
  orb_synth::render(seed, frame, view, width, height, out, stride);
}

void orb_synth_local_map(uint64_t seed, const orb_keypoint_t* keys, const uint8_t* desc,
                         int n_kp, int n_mp, int width, int height, orb_mp_track_t* mps,
                         uint8_t* mp_desc, uint8_t* kp_locked) {
  orb_synth::local_map(seed, keys, desc, n_kp, n_mp, width, height, mps, mp_desc, kp_locked);
}

}  // extern "C"
