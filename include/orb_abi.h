/*
 * orb_abi.h -- C ABI of the MI355X-native ORB front-end (extractor + Hamming matcher).
 *
 * This is the drop-in boundary.  Plain C: pointers, sizes, status codes; no
 * OpenCV, no torch, no HIP types in any signature (streams are passed as
 * `void*`, a hipStream_t, NULL = the handle's own stream).
 *
 * Streams and call order.  A handle's calls are serialised on the host (a
 * mutex per handle) and on the device: every call reuses the handle's device
 * scratch, so a call issued on a different stream from the previous call on
 * the same handle first makes its stream wait for that call (an event wait,
 * no host synchronisation), and a frame-size change, which rewrites the
 * extractor's plan tables, waits on the host for the previous call.  One
 * handle may therefore be driven from any mix of streams (the reference's
 * ORBextractor is not reentrant at all, include/ORBextractor.h:85).  The
 * caller still orders its own data: a batch call's inputs must be ready on
 * the stream passed, and its outputs are ready on that stream only.  Calls
 * issued on a stream being captured into a graph record no event; the caller
 * orders the graph's launches.  The extractor's batch calls also use one
 * device-wide side stream that HIP creates blocking, so work on the legacy
 * null stream waits for its FAST kernels in flight (INTEGRATION.md "Streams").
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference tree, yg838457845/ORB_SLAM2-Chinese-annotation):
 *
 *   orb_extractor_create/destroy   ORBextractor::ORBextractor  include/ORBextractor.h:51-54,
 *                                  src/ORBextractor.cc:428-489
 *   orb_extractor_get_*            ORBextractor::Get*          include/ORBextractor.h:63-83
 *   orb_extractor_extract          ORBextractor::operator()    include/ORBextractor.h:59-61,
 *                                  src/ORBextractor.cc:1091-1169
 *   orb_extractor_pyramid_level    ORBextractor::mvImagePyramid include/ORBextractor.h:85
 *   orb_extractor_extract_batch    (throughput form of operator(), many frames per launch)
 *   orb_descriptor_distance        ORBmatcher::DescriptorDistance src/ORBmatcher.cc:1814-1830
 *   orb_hamming_batch              batched DescriptorDistance (device)
 *   orb_match_projection_local     ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, float)
 *                                  src/ORBmatcher.cc:47-133 (+ Frame::GetFeaturesInArea
 *                                  src/Frame.cc:368-424, AssignFeaturesToGrid :261-276)
 *   orb_match_projection_local_batch  device-batched form of the above
 *   orb_stereo_match               Frame::ComputeStereoMatches src/Frame.cc:516-704
 *   orb_match_projection_frame     ORBmatcher::SearchByProjection(Frame&, const Frame&, float, bool)
 *                                  src/ORBmatcher.cc:1460-1619
 *   orb_match_bow                  ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
 *                                  src/ORBmatcher.cc:164-306
 *   orb_frustum(_batch)            Frame::isInFrustum src/Frame.cc:303-366 over the local map
 *                                  (Tracking::SearchLocalPoints src/Tracking.cc:1360-1377,
 *                                  MapPoint::PredictScale src/MapPoint.cc:435-450)
 *   orb_stereo_match_batch         device-batched ComputeStereoMatches (pairs from two extractors)
 *   orb_search_for_initialization(_batch)  ORBmatcher::SearchForInitialization
 *                                  src/ORBmatcher.cc:429-577
 *   orb_distinctive_descriptors(_batch)    MapPoint::ComputeDistinctiveDescriptors
 *                                  src/MapPoint.cc:250-326
 *   orb_search_by_projection_reloc SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)
 *                                  src/ORBmatcher.cc:1622-1759
 *   orb_search_by_projection_sim3  SearchByProjection(KeyFrame*, Scw, ...) src/ORBmatcher.cc:311-425
 *   orb_fuse / orb_fuse_sim3       Fuse(KeyFrame*, ...) x2   src/ORBmatcher.cc:903-1210
 *   orb_search_by_sim3             SearchBySim3              src/ORBmatcher.cc:1212-1458
 *   orb_match_bow_kf               SearchByBoW(KeyFrame*, KeyFrame*, ...) src/ORBmatcher.cc:581-716
 *   orb_search_for_triangulation   SearchForTriangulation    src/ORBmatcher.cc:718-901
 *   orb_undistort_points / orb_undistort_keypoints(_batch) / orb_compute_image_bounds
 *                                  cv::undistortPoints in Frame::UndistortKeyPoints
 *                                  src/Frame.cc:452-482 and ComputeImageBounds :484-514
 *   orb_vocabulary_create / _load_text / _destroy
 *                                  DBoW2 TemplatedVocabulary ctor + loadFromTextFile
 *                                  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1362-1448
 *                                  (ORBVocabulary, include/ORBVocabulary.h; loaded by
 *                                  System::System src/System.cc)
 *   orb_vocabulary_transform(_batch)  Frame::ComputeBoW src/Frame.cc:439-449,
 *                                  KeyFrame::ComputeBoW src/KeyFrame.cc:60-71 ->
 *                                  TemplatedVocabulary::transform(features, BowVector&,
 *                                  FeatureVector&, levelsup) TemplatedVocabulary.h:1128-1283
 *
 * Error behaviour: the reference has no status codes (an empty image returns
 * silently with outputs untouched, src/ORBextractor.cc:1095-1096; a non-8UC1
 * image asserts, :1100).  Here every call returns an orb_status_t; the C++
 * wrapper (orb_slam2-chinese-annotation_amd/host/orb_amd.hpp) maps
 * ORB_EEMPTY to "return, outputs untouched" and ORB_EINVAL to an assert.
 */
#ifndef ORB_ABI_H
#define ORB_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORB_ABI_VERSION 1
#define ORB_DESC_BYTES 32
#define ORB_GRID_COLS 64 /* FRAME_GRID_COLS, include/Frame.h:39 */
#define ORB_GRID_ROWS 48 /* FRAME_GRID_ROWS, include/Frame.h:40 */

typedef enum orb_status {
  ORB_OK = 0,
  ORB_EEMPTY = 1,     /* empty input: reference returns silently, outputs untouched */
  ORB_EINVAL = -1,    /* bad argument (reference: assert) */
  ORB_ENOMEM = -2,    /* device allocation failed */
  ORB_EDEVICE = -3,   /* HIP runtime / kernel error */
  ORB_ECAPACITY = -4, /* caller buffer too small; *n set to the required size */
  ORB_ENODEV = -5     /* no gfx950 device visible */
} orb_status_t;

/* Mirrors cv::KeyPoint field-for-field (28 bytes). */
typedef struct orb_keypoint {
  float x, y;      /* pt */
  float size;      /* int(31 * scale[octave]) */
  float angle;     /* degrees, [0, 360] */
  float response;  /* FAST-9/16 corner score */
  int32_t octave;  /* pyramid level */
  int32_t class_id;/* always -1 */
} orb_keypoint_t;

typedef struct orb_extractor orb_extractor_t;
typedef struct orb_matcher orb_matcher_t;

/* ---------------------------------------------------------------- extractor */

/* Limits (the reference states none; these are where this build stops, each
 * a status, never a silent change of results):
 *   create: nfeatures >= 0, 1 <= nlevels <= 16, scale_factor > 1 (finite)
 *     (ORB_EINVAL otherwise: at 1 the reference's quota series is 0 / 0,
 *     src/ORBextractor.cc:453-455).  Every scale factor takes the same
 *     integer resize taps; levels whose downscale the staged tiles cannot
 *     hold (beyond ~1.9) take an untiled kernel.
 *   extract: every pyramid level between 33 and 4095 px in each dimension
 *     (at 32 px or less the reference's DistributeOctTree divides by zero or
 *     sizes its root vector negatively, :562-569; keys pack x and y in 12
 *     bits), a level's quota + 4 at most 65,534 (16-bit node labels: nfeatures
 *     up to ~300,000 at 1.2 / 8 levels), FAST cells at most 64 x 64 interior
 *     pixels: ORB_EINVAL from the call (and orb_extractor_capacity < 0).
 *   DistributeOctTree (src/ORBextractor.cc:558-782): node tables hold
 *     quota + 4 nodes per level (the reference's list never exceeds quota + 3,
 *     or 4 x its root count after the first pass), at most 512 passes (distinct
 *     keys separate in about 12; the final phase adds a few) and 2^24 created
 *     nodes.  Exceeding any of them is not reachable with keys the FAST stage
 *     emits; if it happened the image fails as a whole: orb_extractor_extract
 *     returns ORB_EDEVICE and the batch form writes d_counts[i] = ORB_EDEVICE
 *     (negative).  A test-only build of the library with the pass bound
 *     lowered drives that path (tests/test_gpu_extractor.py); the product
 *     reads no environment variable that changes results. */
orb_status_t orb_extractor_create(int nfeatures, float scale_factor, int nlevels,
                                  int ini_th_fast, int min_th_fast, int device,
                                  orb_extractor_t** out);
void orb_extractor_destroy(orb_extractor_t* h);

int orb_extractor_get_levels(const orb_extractor_t* h);
float orb_extractor_get_scale_factor(const orb_extractor_t* h);
/* Each writes nlevels floats. */
void orb_extractor_get_scale_factors(const orb_extractor_t* h, float* out);
void orb_extractor_get_inverse_scale_factors(const orb_extractor_t* h, float* out);
void orb_extractor_get_scale_sigma_squares(const orb_extractor_t* h, float* out);
void orb_extractor_get_inverse_scale_sigma_squares(const orb_extractor_t* h, float* out);
/* Per-level keypoint quotas (mnFeaturesPerLevel, src/ORBextractor.cc:453-464). */
void orb_extractor_get_features_per_level(const orb_extractor_t* h, int32_t* out);
/* Upper bound on keypoints one image of this size can produce. */
int orb_extractor_capacity(const orb_extractor_t* h, int width, int height);

/* ORBextractor::operator(): host image in, host keypoints + N x 32 descriptors out.
 * Synchronous.  `capacity` = rows available in keypoints/descriptors; on
 * ORB_ECAPACITY *n_keypoints holds the required count. */
orb_status_t orb_extractor_extract(orb_extractor_t* h, const uint8_t* image, int width,
                                   int height, size_t stride, orb_keypoint_t* keypoints,
                                   uint8_t* descriptors, int capacity, int* n_keypoints);

/* Host copy of mvImagePyramid[level] of the first image of the last call
 * (orb_extractor_extract, or image 0 of orb_extractor_extract_batch, whose
 * level 0 is read from the caller's d_images: keep it alive until then).
 * The copy waits for the last call's stream.  dst may be NULL to query the size. */
orb_status_t orb_extractor_pyramid_level(orb_extractor_t* h, int level, uint8_t* dst,
                                         size_t dst_stride, int* width, int* height);
/* mvImagePyramid[level] of the last orb_extractor_extract call without a copy
 * out: a pointer into pinned host memory the library owns, valid until the
 * next call on this handle (the reference rebuilds mvImagePyramid on every
 * call too, src/ORBextractor.cc:1172-1207; its only reader is
 * Frame::ComputeStereoMatches, src/Frame.cc:524,619,633,639, right after the
 * extraction).  Level 0 is the call's pinned staging of the image; levels 1..
 * come from one DMA of the device pyramid, which the first request makes
 * synchronously and which from then on rides in every call's graph after the
 * keypoint copy.  ORB_EINVAL after a batch call. */
orb_status_t orb_extractor_host_pyramid(orb_extractor_t* h, int level, const uint8_t** data,
                                        int* width, int* height, size_t* stride);
/* Stops the per-call DMA of levels 1.. that orb_extractor_host_pyramid turned
 * on (for a caller that no longer reads the mirror): later calls move no
 * pyramid bytes until the next request, which again copies once and turns the
 * per-call copy back on. */
orb_status_t orb_extractor_host_pyramid_off(orb_extractor_t* h);
/* The 7x7 Gaussian-blurred copy of level `level` of the first image of the
 * last call (the image computeDescriptors samples, src/ORBextractor.cc:1143-1145);
 * same conventions as orb_extractor_pyramid_level. */
orb_status_t orb_extractor_blurred_level(orb_extractor_t* h, int level, uint8_t* dst,
                                         size_t dst_stride, int* width, int* height);

/* Throughput form: n_images device-resident images (image i at
 * d_images + i*image_pitch, rows `stride` apart), all width x height.
 * Outputs per image i: d_keypoints[i*capacity ...], d_descriptors[(i*capacity) * 32 ...],
 * d_counts[i].  Asynchronous on `stream` (NULL = handle stream). */
orb_status_t orb_extractor_extract_batch(orb_extractor_t* h, const uint8_t* d_images,
                                         int n_images, int width, int height, size_t stride,
                                         size_t image_pitch, orb_keypoint_t* d_keypoints,
                                         uint8_t* d_descriptors, int capacity,
                                         int32_t* d_counts, void* stream);

/* Device pointer to pyramid level `level` of batch image `image` after
 * orb_extractor_extract_batch (valid until the next call on this handle).
 * Level 0 is the caller's own image memory (d_images of that call): it is
 * valid only while the caller keeps it.  Readers on another stream must order
 * themselves after the batch's stream. */
orb_status_t orb_extractor_batch_level(orb_extractor_t* h, int image, int level,
                                       const uint8_t** d_level, int* width, int* height,
                                       size_t* stride);

/* Stream the handle launches on (a hipStream_t). */
void* orb_extractor_stream(orb_extractor_t* h);

/* Kernel timing with HIP events recorded on the stream each stage is launched
 * on (no synchronisation in the launch path).  profile(h, 1) resets and
 * enables; profile_read drains the recorded events and returns the summed
 * milliseconds, launch count and kernel name of `stage`:
 * 0 k_pyr_resize (nlevels-1 launches per call), 1 k_blur_levels (split mode
 * only), 2 FAST (k_fast_cells on the levels the main stream runs, or
 * k_fast_band on all levels), 3 k_octree, 4 k_orient_desc,
 * 5 k_fast_cells_side (the cells of level 0, then of levels 1-2, on the
 * handle's side stream beside the resize chain; durations summed; 0 launches
 * when not split off), 6 = the whole extraction call.
 * enable = 2 times every stage alone: while it is set the batch form runs all
 * stages one after another on the caller's stream (no side stream), so each
 * stage's events bracket its own kernels only (bench.py's isolated table). */
orb_status_t orb_extractor_profile(orb_extractor_t* h, int enable);
orb_status_t orb_extractor_profile_read(orb_extractor_t* h, int stage, double* total_ms,
                                        int* launches, const char** name);

/* ------------------------------------------------------------------ matcher */

/* A frame as the matcher sees it (Frame members used by ORBmatcher). */
typedef struct orb_frame {
  int32_t n;                     /* N */
  const orb_keypoint_t* keys;    /* mvKeysUn (== mvKeys at zero distortion) */
  const uint8_t* descriptors;    /* mDescriptors, N x 32 */
  const float* u_right;          /* mvuRight (N) or NULL for monocular (-1) */
  float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
  int32_t n_levels;
  const float* scale_factors;    /* mvScaleFactors */
} orb_frame_t;

/* MapPoint fields written by Frame::isInFrustum (include/MapPoint.h:92-97). */
typedef struct orb_mp_track {
  float proj_x, proj_y, proj_xr;  /* mTrackProjX, mTrackProjY, mTrackProjXR */
  float view_cos;                 /* mTrackViewCos */
  int32_t level;                  /* mnTrackScaleLevel */
  uint8_t in_view;                /* mbTrackInView */
  uint8_t bad;                    /* isBad() */
  uint8_t has_obs;                /* Observations() > 0 (a claim by it locks the keypoint) */
  uint8_t _pad;
} orb_mp_track_t;

/* MapPoint state read by Frame::isInFrustum and Tracking::SearchLocalPoints
 * (src/Frame.cc:303-366, src/Tracking.cc:1360-1377, src/MapPoint.cc:404-450). */
typedef struct orb_map_point {
  float pos[3];        /* GetWorldPos() */
  float normal[3];     /* GetNormal() */
  float min_distance;  /* mfMinDistance (GetMinDistanceInvariance = 0.8f * it) */
  float max_distance;  /* mfMaxDistance (GetMaxDistanceInvariance = 1.2f * it) */
  uint8_t bad;         /* isBad() */
  uint8_t seen;        /* mnLastFrameSeen == mCurrentFrame.mnId (already matched) */
  uint8_t has_obs;     /* Observations() > 0 */
  uint8_t _pad;
} orb_map_point_t;     /* 36 bytes */

/* Pinhole camera (Frame::fx, fy, cx, cy, mbf, mb). */
typedef struct orb_camera {
  float fx, fy, cx, cy, bf, mb;
} orb_camera_t;

/* Frame pose (Frame::UpdatePoseMatrices, src/Frame.cc:294-300). */
typedef struct orb_pose {
  float rcw[9];        /* mRcw, row-major */
  float tcw[3];        /* mtcw */
  float ow[3];         /* mOw = -mRcw^T * mtcw (camera centre) */
} orb_pose_t;

int orb_descriptor_distance(const uint8_t* a, const uint8_t* b);

orb_status_t orb_matcher_create(int device, orb_matcher_t** out);
void orb_matcher_destroy(orb_matcher_t* m);
void* orb_matcher_stream(orb_matcher_t* m);
/* Same scheme for the batched local-map matcher: stage 0 k_grid_build,
 * 1 k_proj_candidates, 2 k_proj_resolve, 3 = whole call. */
orb_status_t orb_matcher_profile(orb_matcher_t* m, int enable);
orb_status_t orb_matcher_profile_read(orb_matcher_t* m, int stage, double* total_ms,
                                      int* launches, const char** name);

/* Resolve schedule of SearchByProjection(F, vpMapPoints)'s first-come claims
 * (src/ORBmatcher.cc:90-93,127: a keypoint claimed by an earlier MapPoint of
 * the same call is skipped).  Every schedule returns the reference's result;
 * they differ in how the ordered resolve is spread over the chip (DESIGN.md
 * §4.2).  AUTO (the default) picks by problem count and map size; JACOBI runs
 * `jacobi_rounds` (1-48) chip-wide rounds first, then the fixed-point windows
 * for any problem not yet settled.  Schedules that need more LDS than the
 * frame's keypoint count allows fall back to the prefix windows. */
#define ORB_RESOLVE_AUTO 0
#define ORB_RESOLVE_PREFIX 1      /* speculative windows, longest conflict-free prefix kept */
#define ORB_RESOLVE_FIXED_POINT 2 /* 1024-point windows iterated to their fixed point */
#define ORB_RESOLVE_JACOBI 3      /* chip-wide rounds + fixed-point windows */
orb_status_t orb_matcher_set_resolve(orb_matcher_t* m, int schedule, int jacobi_rounds);
/* The resolve kernel the local-map matcher launches for a call of n_problems
 * problems at these strides under the handle's schedule. */
#define ORB_RESOLVE_KERNEL_PREFIX_W1 1   /* k_proj_resolve<1>: one wave per problem */
#define ORB_RESOLVE_KERNEL_PREFIX_W4 4   /* k_proj_resolve<4> */
#define ORB_RESOLVE_KERNEL_PREFIX_W8 8   /* k_proj_resolve<8> */
#define ORB_RESOLVE_KERNEL_FIXED_POINT 16 /* k_proj_resolve_fp<1024> */
#define ORB_RESOLVE_KERNEL_JACOBI 32     /* k_proj_jacobi rounds + k_proj_resolve_fp */
orb_status_t orb_matcher_resolve_kernel(orb_matcher_t* m, int n_problems, int kp_stride,
                                        int mp_stride, int* kernel);

/* dist[i] = DescriptorDistance(a + 32 i, b + 32 i), device pointers. */
orb_status_t orb_hamming_batch(orb_matcher_t* m, const uint8_t* d_a, const uint8_t* d_b,
                               int n, int32_t* d_dist, void* stream);

/* SearchByProjection(F, vpMapPoints, th) with ORBmatcher(nnratio).
 * kp_locked[i] != 0  <=>  F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0
 * on entry.  Output kp_match[i] = index of the MapPoint assigned to keypoint i
 * by THIS call (last writer wins, as F.mvpMapPoints[bestIdx]=pMP), or -1.
 * Returns the reference's nmatches. Host buffers. */
orb_status_t orb_match_projection_local(orb_matcher_t* m, const orb_frame_t* frame,
                                        const uint8_t* kp_locked, int n_mp,
                                        const orb_mp_track_t* mps, const uint8_t* mp_desc,
                                        float th, float nnratio, int32_t* kp_match,
                                        int32_t* nmatches);

/* Zero-copy form of orb_match_projection_local, for a caller that flattens its
 * Frame and MapPoints anyway (the reference-typed drop-in's SearchByProjection,
 * integration/ORBmatcher.cc): _stage returns pointers into the handle's pinned
 * input block laid out for n_keys keypoints and n_mp map points, the caller
 * writes keys, descriptors, the map-point tracks and descriptors there (and
 * u_right / kp_locked when it passes stereo / locked), and _staged runs the
 * match on them: one DMA in, no library-side copy.  `frame` supplies n (==
 * n_keys), the bounds, levels and scale factors; its keys / descriptors /
 * u_right pointers are not read.  The pointers are valid until the next call
 * on this handle; the pair must not interleave with other calls on it (one
 * handle per thread, as the reference's per-call-site ORBmatcher objects).
 * Optional _begin, between _stage and _staged, once the frame's part (keys,
 * descriptors, u_right, kp_locked) is written and before the map points are:
 * it sends that part and builds the keypoint grid on the device while the
 * caller flattens its map; stereo / locked must equal _staged's.  A _stage
 * after a _begin without its _staged waits for the _begin's work first. */
typedef struct orb_local_stage {
  orb_keypoint_t* keys;        /* n_keys */
  uint8_t* descriptors;        /* n_keys x 32 */
  float* u_right;              /* n_keys (read only with stereo != 0) */
  uint8_t* kp_locked;          /* n_keys (read only with locked != 0) */
  orb_mp_track_t* mps;         /* n_mp */
  uint8_t* mp_desc;            /* n_mp x 32 */
} orb_local_stage_t;
orb_status_t orb_match_projection_local_stage(orb_matcher_t* m, int n_keys, int n_mp,
                                              orb_local_stage_t* out);
orb_status_t orb_match_projection_local_begin(orb_matcher_t* m, const orb_frame_t* frame,
                                              int stereo, int locked);
orb_status_t orb_match_projection_local_staged(orb_matcher_t* m, const orb_frame_t* frame,
                                               int n_mp, int stereo, int locked, float th,
                                               float nnratio, int32_t* kp_match,
                                               int32_t* nmatches);

/* Device-batched form: P independent (frame, local map) problems.
 * Problem p: keypoints d_keys + p*kp_stride (count d_nkeys[p]), descriptors
 * d_desc + p*kp_stride*32, locks d_locked + p*kp_stride (may be NULL),
 * map points d_mps + p*mp_stride (count d_nmps[p]), their descriptors
 * d_mp_desc + p*mp_stride*32.  Monocular (u_right = -1).  Frame bounds and
 * scale factors are shared.  Outputs d_kp_match + p*kp_stride, d_nmatches[p]. */
orb_status_t orb_match_projection_local_batch(
    orb_matcher_t* m, int n_problems, const orb_keypoint_t* d_keys, const uint8_t* d_desc,
    const int32_t* d_nkeys, const uint8_t* d_locked, int kp_stride,
    const orb_mp_track_t* d_mps, const uint8_t* d_mp_desc, const int32_t* d_nmps,
    int mp_stride, float min_x, float max_x, float min_y, float max_y, int n_levels,
    const float* scale_factors, float th, float nnratio, int32_t* d_kp_match,
    int32_t* d_nmatches, void* stream);

/* Tracking::SearchLocalPoints' frustum pass: for each local MapPoint in order,
 * skip it if seen or bad, else Frame::isInFrustum(pMP, viewing_cos_limit)
 * (src/Tracking.cc:1360-1377, src/Frame.cc:303-366, MapPoint::PredictScale
 * src/MapPoint.cc:435-450).  Writes tracks[i] (proj_x, proj_y, proj_xr,
 * view_cos, level, in_view; bad and has_obs copied through; all-zero
 * projection fields when not in view) and n_in_view = nToMatch.  The tracks
 * feed orb_match_projection_local unchanged.  log_scale_factor =
 * Frame::mfLogScaleFactor.  Host buffers. */
orb_status_t orb_frustum(orb_matcher_t* m, int n_mp, const orb_map_point_t* mps,
                         const orb_pose_t* pose, const orb_camera_t* cam, float min_x,
                         float max_x, float min_y, float max_y, float viewing_cos_limit,
                         float log_scale_factor, int n_levels, orb_mp_track_t* tracks,
                         int32_t* n_in_view);

/* Device-batched form: problem p uses d_poses[p], map points d_mps + p*mp_stride
 * (count d_nmps[p]); writes d_tracks + p*mp_stride and d_n_in_view[p]. */
orb_status_t orb_frustum_batch(orb_matcher_t* m, int n_problems, const orb_map_point_t* d_mps,
                               const int32_t* d_nmps, int mp_stride, const orb_pose_t* d_poses,
                               const orb_camera_t* cam, float min_x, float max_x, float min_y,
                               float max_y, float viewing_cos_limit, float log_scale_factor,
                               int n_levels, orb_mp_track_t* d_tracks, int32_t* d_n_in_view,
                               void* stream);

/* Frame::ComputeStereoMatches for one rectified pair.  Left/right keypoints
 * and descriptors as produced by the two extractors, plus both pyramids
 * (level l of side s at pyr[s][l] with the given stride/size).  Writes
 * mvuRight / mvDepth (-1 = no match). Host buffers. */
typedef struct orb_stereo_input {
  const orb_frame_t* left;       /* mvKeys, mDescriptors (u_right ignored) */
  int32_t n_right;
  const orb_keypoint_t* right_keys;
  const uint8_t* right_desc;
  int32_t n_levels;
  const uint8_t* const* left_levels;   /* n_levels host pointers */
  const uint8_t* const* right_levels;
  const int32_t* level_width;    /* n_levels */
  const int32_t* level_height;
  const int64_t* level_stride;
  const float* inv_scale_factors;/* mvInvScaleFactors */
  float bf;                      /* mbf */
  float fx;                      /* fx; mb = bf / fx */
} orb_stereo_input_t;

orb_status_t orb_stereo_match(orb_matcher_t* m, const orb_stereo_input_t* in,
                              float* u_right, float* depth);

/* Device-batched ComputeStereoMatches for n_pairs rectified pairs whose left
 * and right images went through orb_extractor_extract_batch on left_ext and
 * right_ext (pyramids are read from those handles).  Keypoints/descriptors as
 * written by the two batches (pair i at i*kp_stride), counts d_left_n/d_right_n.
 * Writes d_u_right / d_depth (-1 = none) and d_sad (SAD of kept matches, -1). */
orb_status_t orb_stereo_match_batch(orb_matcher_t* m, int n_pairs, orb_extractor_t* left_ext,
                                    orb_extractor_t* right_ext, const orb_keypoint_t* d_left_keys,
                                    const uint8_t* d_left_desc, const int32_t* d_left_n,
                                    const orb_keypoint_t* d_right_keys,
                                    const uint8_t* d_right_desc, const int32_t* d_right_n,
                                    int kp_stride, float bf, float fx, float* d_u_right,
                                    float* d_depth, int32_t* d_sad, void* stream);

/* Frame::ComputeStereoMatches (src/Frame.cc:516-704) for the pair whose left
 * and right images were extracted last by orb_extractor_extract on left_ext and
 * right_ext (the stereo Frame constructor's two ExtractORB calls,
 * src/Frame.cc:81-93): keypoints, descriptors and both pyramids are read where
 * the extractions left them in device memory, so only mvuRight / mvDepth
 * (-1 = no match) are copied back.  *n_left = the left keypoint count; the
 * outputs need n_left entries (ORB_ECAPACITY if capacity is smaller; both
 * outputs NULL = size query).
 * ORB_EINVAL if either handle's last call was not orb_extractor_extract, or
 * if the matcher and the two extractors were not created on one device.
 * Synchronous. */
orb_status_t orb_stereo_match_extracted(orb_matcher_t* m, orb_extractor_t* left_ext,
                                        orb_extractor_t* right_ext, float bf, float fx,
                                        float* u_right, float* depth, int capacity,
                                        int* n_left);

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono) with ORBmatcher(nnratio, checkOri).
 * The last frame's map points are given already projected with the current
 * pose (the float camera-space coordinates xc, yc and invzc computed exactly
 * as src/ORBmatcher.cc:1500-1505).  valid[i]=0 for NULL or outlier entries.
 * kp_match[i] (out) = MapPoint id assigned to current keypoint i by this call,
 * -1 untouched, -2 reset to NULL by the rotation-consistency filter
 * (src/ORBmatcher.cc:1597-1616). */
typedef struct orb_last_mp {
  float xc, yc, invzc;          /* Rcw*x3Dw + tcw, 1/z */
  int32_t last_octave;          /* LastFrame.mvKeys[i].octave */
  float last_angle;             /* LastFrame.mvKeysUn[i].angle */
  uint8_t valid;                /* pMP && !mvbOutlier[i] */
  uint8_t has_obs;              /* pMP->Observations() > 0 */
  uint8_t _pad[2];
  int32_t mp_id;                /* identity of pMP (same id => same MapPoint) */
} orb_last_mp_t;


orb_status_t orb_match_projection_frame(orb_matcher_t* m, const orb_frame_t* current,
                                        const uint8_t* kp_locked, int n_last,
                                        const orb_last_mp_t* last, const uint8_t* last_desc,
                                        const orb_camera_t* cam, float tlc_z, float th,
                                        int mono, int check_orientation,
                                        int32_t* kp_match, int32_t* nmatches);

/* SearchByBoW(pKF, F, vpMapPointMatches) with ORBmatcher(nnratio, checkOri).
 * FeatureVectors are CSR: node ids ascending (nodes_*), feature lists
 * offs_*[k]..offs_*[k+1] in feats_*.  kf_mp[i] = MapPoint id of KF keypoint i
 * or -1 (NULL); kf_mp_bad[i] = isBad().  Output f_match[j] = MapPoint id or -1. */
orb_status_t orb_match_bow(orb_matcher_t* m, int n_kf, const uint8_t* kf_desc,
                           const float* kf_angle, const int32_t* kf_mp,
                           const uint8_t* kf_mp_bad, int kf_nodes, const uint32_t* kf_node_ids,
                           const int32_t* kf_offs, const uint32_t* kf_feats, int n_f,
                           const uint8_t* f_desc, const float* f_angle, int f_nodes,
                           const uint32_t* f_node_ids, const int32_t* f_offs,
                           const uint32_t* f_feats, float nnratio, int check_orientation,
                           int32_t* f_match, int32_t* nmatches);

/* ORBmatcher(nnratio, checkOri).SearchForInitialization(F1, F2, vbPrevMatched,
 * vnMatches12, windowSize), src/ORBmatcher.cc:429-577 (called from
 * Tracking::MonocularInitialization, src/Tracking.cc:698-701).  Level-0
 * keypoints of f1 are matched to level-0 keypoints of f2 within windowSize of
 * prev_matched[i] (x, y pairs); f2's grid bounds are min_x..max_y.
 * matches12[i] = F2 index or -1; prev_matched is updated in place for matched
 * keypoints (:571-574); *nmatches = the reference's return value.  Host buffers;
 * both frames must have fewer than 2^19 keypoints and 4 * 4 * max(N1, N2) bytes
 * must fit the 160 KiB LDS of one CU (N <= 10240), else ORB_ECAPACITY. */
orb_status_t orb_search_for_initialization(orb_matcher_t* m, const orb_frame_t* f1,
                                           const orb_frame_t* f2, float* prev_matched,
                                           int window_size, float nnratio,
                                           int check_orientation, int32_t* matches12,
                                           int32_t* nmatches);

/* Device-batched form: problem p uses d_keys1/d_desc1/d_prev_matched/d_matches12
 * at offset p*kp_stride (keypoints; x2 floats, x32 bytes as applicable), counts
 * d_n1[p], d_n2[p] <= kp_stride, shared frame bounds. */
orb_status_t orb_search_for_initialization_batch(
    orb_matcher_t* m, int n_problems, const orb_keypoint_t* d_keys1, const uint8_t* d_desc1,
    const int32_t* d_n1, const orb_keypoint_t* d_keys2, const uint8_t* d_desc2,
    const int32_t* d_n2, int kp_stride, float min_x, float max_x, float min_y, float max_y,
    int window_size, float nnratio, int check_orientation, float* d_prev_matched,
    int32_t* d_matches12, int32_t* d_nmatches, void* stream);

/* MapPoint::ComputeDistinctiveDescriptors, src/MapPoint.cc:250-326, for n_mp
 * points at once.  Point p's candidate descriptors are obs_desc rows
 * obs_offs[p] .. obs_offs[p+1]-1: its observations in mObservations (map) order,
 * bad KeyFrames left out (:279-283).  best_idx[p] = BestIdx within that list,
 * -1 for an empty list (the reference returns without touching mDescriptor).
 * If descriptors != NULL, row p is overwritten with the chosen descriptor
 * (left untouched for empty lists).  Host buffers. */
orb_status_t orb_distinctive_descriptors(orb_matcher_t* m, int n_mp, const int32_t* obs_offs,
                                         const uint8_t* obs_desc, int32_t* best_idx,
                                         uint8_t* descriptors);

/* Device-batched form (device pointers, asynchronous on `stream`). */
orb_status_t orb_distinctive_descriptors_batch(orb_matcher_t* m, int n_mp,
                                               const int32_t* d_obs_offs,
                                               const uint8_t* d_obs_desc, int32_t* d_best_idx,
                                               uint8_t* d_descriptors, void* stream);

/* ---- projection-window ORBmatcher variants.  Map points use
 * orb_map_point_t; its `seen` flag marks the variant's "already found" set
 * (documented per call).  Host buffers; log_scale_factor = mfLogScaleFactor;
 * KeyFrame bounds come from the orb_frame_t (KeyFrame::IsInImage is
 * half-open, Frame bounds closed, as in the reference). */

/* SearchByProjection(Frame& F, KeyFrame* pKF, sAlreadyFound, th, ORBdist),
 * src/ORBmatcher.cc:1622-1759 (Tracking::Relocalization).  Point i = the
 * MapPoint of KF keypoint i (NULL -> bad = 1; seen = in sAlreadyFound),
 * kf_angle[i] = pKF->mvKeysUn[i].angle, pose = F.mTcw (+ mOw).
 * kp_locked[j] = F.mvpMapPoints[j] != NULL on entry.  kp_match[j] (out) = point
 * assigned to frame keypoint j by this call, -1 none, -2 reset by the rotation
 * filter.  *nmatches = the reference's return value. */
orb_status_t orb_search_by_projection_reloc(orb_matcher_t* m, const orb_frame_t* frame,
                                            const uint8_t* kp_locked, const orb_pose_t* pose,
                                            const orb_camera_t* cam, float log_scale_factor,
                                            int n_mp, const orb_map_point_t* mps,
                                            const uint8_t* mp_desc, const float* kf_angle,
                                            float th, int orb_dist, int check_orientation,
                                            int32_t* kp_match, int32_t* nmatches);

/* SearchByProjection(KeyFrame* pKF, Scw, vpPoints, vpMatched, th),
 * src/ORBmatcher.cc:311-425 (LoopClosing::ComputeSim3).  scw = the top 3 rows of
 * Scw, row-major.  seen = in spAlreadyFound (vpMatched's points).
 * kp_matched[j] (in/out) = index into vpPoints of vpMatched[j], -1 = NULL. */
orb_status_t orb_search_by_projection_sim3(orb_matcher_t* m, const orb_frame_t* kf,
                                           const float* scw, const orb_camera_t* cam,
                                           float log_scale_factor, int n_mp,
                                           const orb_map_point_t* mps, const uint8_t* mp_desc,
                                           float th, int32_t* kp_matched, int32_t* nmatches);

/* Fuse(KeyFrame* pKF, vpMapPoints, th), src/ORBmatcher.cc:903-1077: the match
 * half.  fuse_idx[i] (out) = keypoint of pKF point i fuses into (bestIdx) or
 * -1; seen = pMP->IsInKeyFrame(pKF); pose = pKF's Tcw with Ow = camera centre;
 * kf->u_right = mvuRight.  The caller applies Replace / AddObservation in
 * point order (:1048-1070), re-checking isBad() / IsInKeyFrame() first: the
 * targets only depend on entry state for points the reference still visits. */
orb_status_t orb_fuse(orb_matcher_t* m, const orb_frame_t* kf, const float* inv_level_sigma2,
                      const orb_pose_t* pose, const orb_camera_t* cam, float log_scale_factor,
                      int n_mp, const orb_map_point_t* mps, const uint8_t* mp_desc, float th,
                      int32_t* fuse_idx, int32_t* n_fuse);

/* Fuse(KeyFrame* pKF, Scw, vpPoints, th, vpReplacePoint),
 * src/ORBmatcher.cc:1079-1210: fuse_idx[i] = bestIdx or -1 (seen = in
 * pKF->GetMapPoints() at entry); vpReplacePoint / AddMapPoint stay with the
 * caller. */
orb_status_t orb_fuse_sim3(orb_matcher_t* m, const orb_frame_t* kf, const float* scw,
                           const orb_camera_t* cam, float log_scale_factor, int n_mp,
                           const orb_map_point_t* mps, const uint8_t* mp_desc, float th,
                           int32_t* fuse_idx, int32_t* n_fuse);

/* SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th),
 * src/ORBmatcher.cc:1212-1458.  mpsX[i] / mp_descX[i] = the MapPoint of
 * keypoint i of KF X (validX[i] = non-NULL), alreadyX = vbAlreadyMatchedX
 * (:1240-1252).  rXw / tXw = KF rotations (row-major) and translations.
 * match12[i1] (out) = idx2 with vpMatches12[i1] = vpMapPoints2[idx2], or -1. */
orb_status_t orb_search_by_sim3(orb_matcher_t* m, const orb_frame_t* kf1, const orb_frame_t* kf2,
                                float log_scale_factor, const orb_camera_t* cam,
                                const float* r1w, const float* t1w, const float* r2w,
                                const float* t2w, const orb_map_point_t* mps1,
                                const uint8_t* valid1, const uint8_t* already1,
                                const uint8_t* mp_desc1, const orb_map_point_t* mps2,
                                const uint8_t* valid2, const uint8_t* already2,
                                const uint8_t* mp_desc2, float s12, const float* r12,
                                const float* t12, float th, int32_t* match12, int32_t* nfound);

/* SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vpMatches12),
 * src/ORBmatcher.cc:581-716 (FeatureVectors as in orb_match_bow).
 * match12[i] (out) = MapPoint id of the KF2 keypoint matched to KF1 keypoint i,
 * or -1. */
orb_status_t orb_match_bow_kf(orb_matcher_t* m, int n1, const uint8_t* desc1,
                              const float* angle1, const int32_t* mp1, const uint8_t* mp1_bad,
                              int nodes1, const uint32_t* node_ids1, const int32_t* offs1,
                              const uint32_t* feats1, int n2, const uint8_t* desc2,
                              const float* angle2, const int32_t* mp2, const uint8_t* mp2_bad,
                              int nodes2, const uint32_t* node_ids2, const int32_t* offs2,
                              const uint32_t* feats2, float nnratio, int check_orientation,
                              int32_t* match12, int32_t* nmatches);

/* SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo),
 * src/ORBmatcher.cc:718-901.  has_mpX[i] = GetMapPoint(i) != NULL;
 * level_sigma2 = pKF2->mvLevelSigma2; f12 row-major; cw = pKF1 camera centre,
 * r2w/t2w = pKF2 pose.  match12[i] (out) = KF2 index or -1; vMatchedPairs =
 * the (i, match12[i]) with match12[i] >= 0 in ascending i. */
orb_status_t orb_search_for_triangulation(
    orb_matcher_t* m, const orb_frame_t* kf1, const uint8_t* has_mp1, const orb_frame_t* kf2,
    const uint8_t* has_mp2, const float* level_sigma2, const float* f12,
    const orb_camera_t* cam, const float* cw, const float* r2w, const float* t2w, int nodes1,
    const uint32_t* node_ids1, const int32_t* offs1, const uint32_t* feats1, int nodes2,
    const uint32_t* node_ids2, const int32_t* offs2, const uint32_t* feats2, int only_stereo,
    int check_orientation, int32_t* match12, int32_t* nmatches);

/* -------------------------------------------------------- undistortion */

/* cv::undistortPoints(src, dst, mK, mDistCoef, cv::Mat(), mK), the call in
 * Frame::UndistortKeyPoints and Frame::ComputeImageBounds (src/Frame.cc:452-514),
 * with OpenCV's cvUndistortPoints arithmetic (double, 5 fixed iterations,
 * RR = mK): K = mK as 9 floats row-major, dist = mDistCoef (n_dist 4, 5, 8 or
 * 12: k1 k2 p1 p2 [k3 [k4 k5 k6 [s1 s2 s3 s4]]]; the tilted 14-term model is
 * not supported).  Points as (x, y) float pairs.  Host buffers. */
orb_status_t orb_undistort_points(orb_matcher_t* m, int n, const float* xy, const float* K,
                                  const float* dist, int n_dist, float* out_xy);
/* Frame::UndistortKeyPoints: mvKeysUn from mvKeys (dist[0] == 0 -> copy,
 * :454-458); every field but pt is copied.  keys_un may equal keys. */
orb_status_t orb_undistort_keypoints(orb_matcher_t* m, int n, const orb_keypoint_t* keys,
                                     const float* K, const float* dist, int n_dist,
                                     orb_keypoint_t* keys_un);
/* Frame::ComputeImageBounds: bounds = {mnMinX, mnMaxX, mnMinY, mnMaxY}. */
orb_status_t orb_compute_image_bounds(orb_matcher_t* m, int cols, int rows, const float* K,
                                      const float* dist, int n_dist, float* bounds);
/* Device-batched UndistortKeyPoints: frame f has d_n[f] keypoints at
 * d_keys + f * stride (e.g. the output of orb_extractor_extract_batch);
 * writes d_keys_un at the same offsets.  Asynchronous on `stream`. */
orb_status_t orb_undistort_keypoints_batch(orb_matcher_t* m, int n_frames, const int32_t* d_n,
                                           const orb_keypoint_t* d_keys, int stride,
                                           const float* K, const float* dist, int n_dist,
                                           orb_keypoint_t* d_keys_un, void* stream);

/* ------------------------------------------------------ DBoW2 vocabulary */

typedef struct orb_vocabulary orb_vocabulary_t;

/* ScoringType / WeightingType values (Thirdparty/DBoW2/DBoW2/BowVector.h:36-53). */
#define ORB_VOC_L1_NORM 0
#define ORB_VOC_L2_NORM 1
#define ORB_VOC_CHI_SQUARE 2
#define ORB_VOC_KL 3
#define ORB_VOC_BHATTACHARYYA 4
#define ORB_VOC_DOT_PRODUCT 5
#define ORB_VOC_TF_IDF 0
#define ORB_VOC_TF 1
#define ORB_VOC_IDF 2
#define ORB_VOC_BINARY 3

/* A vocabulary tree from the node table loadFromTextFile builds
 * (TemplatedVocabulary.h:1400-1444): node 0 is the root; node i >= 1 has
 * parent[i] < i (its children are ordered by id), leaf_flag[i] (word ids go to
 * flagged nodes in id order), descriptor 32 bytes at descriptors + 32 i and
 * weight[i].  Entry 0 of each array is ignored.  k, L, scoring, weighting as in
 * the text header (validated as at :1383).  The tree is copied to the device. */
orb_status_t orb_vocabulary_create(int device, int k, int L, int scoring, int weighting,
                                   int n_nodes, const int32_t* parent, const uint8_t* leaf_flag,
                                   const uint8_t* descriptors, const double* weights,
                                   orb_vocabulary_t** out);
/* loadFromTextFile(path) (ORBvoc.txt format). */
orb_status_t orb_vocabulary_load_text(int device, const char* path, orb_vocabulary_t** out);
void orb_vocabulary_destroy(orb_vocabulary_t* v);
/* info6 = {k, L, scoring, weighting, nodes (incl. root), words}. */
orb_status_t orb_vocabulary_info(const orb_vocabulary_t* v, int32_t* info6);
void* orb_vocabulary_stream(orb_vocabulary_t* v);

/* transform(desc rows, mBowVec, mFeatVec, levelsup) for one frame of n <= 8192
 * descriptors.  BowVector (std::map<WordId, double>) as bow_words ascending +
 * bow_values; FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR in
 * the orb_match_bow layout: fv_nodes ascending, fv_offs[n_fv_nodes + 1],
 * fv_feats.  Every output holds up to n entries (fv_offs n + 1).  Optional
 * per-feature feat_word (0xFFFFFFFF = stopped, weight <= 0) and feat_node. */
orb_status_t orb_vocabulary_transform(orb_vocabulary_t* v, int n, const uint8_t* desc,
                                      int levelsup, uint32_t* bow_words, double* bow_values,
                                      int32_t* n_words, uint32_t* fv_nodes, int32_t* fv_offs,
                                      uint32_t* fv_feats, int32_t* n_fv_nodes,
                                      uint32_t* feat_word, uint32_t* feat_node);
/* Device-batched form: frame f has d_counts[f] descriptors at
 * d_desc + 32 * f * stride (stride <= 8192).  Per-frame outputs at offset
 * f * stride (fv_offs: f * (stride + 1)); d_feat_* are per-feature scratch
 * (also outputs) of n_frames * stride entries.  Asynchronous on `stream`. */
orb_status_t orb_vocabulary_transform_batch(orb_vocabulary_t* v, int n_frames,
                                            const int32_t* d_counts, const uint8_t* d_desc,
                                            int stride, int levelsup, uint32_t* d_feat_word,
                                            double* d_feat_weight, uint32_t* d_feat_node,
                                            uint32_t* d_bow_words, double* d_bow_values,
                                            int32_t* d_n_words, uint32_t* d_fv_nodes,
                                            int32_t* d_fv_offs, uint32_t* d_fv_feats,
                                            int32_t* d_n_fv_nodes, void* stream);

/* ---------------------------------------------------------- synthetic input */

/* Deterministic synthetic grayscale images (integer-only generator, identical
 * everywhere).  view 0 = left / mono, 1 = right (shapes shifted by their
 * disparity, bf-consistent).  Frame `frame` of sequence `seed` applies the
 * cumulative ego-motion of frames 0..frame-1. */
void orb_synth_image(uint64_t seed, int frame, int view, int width, int height,
                     uint8_t* out, size_t stride);

/* Synthetic local map of n_mp points derived from one frame's keypoints
 * (SURVEY §8(d) C5 recipe).  Writes mps[n_mp], mp_desc[n_mp*32],
 * kp_locked[n_kp]. */
void orb_synth_local_map(uint64_t seed, const orb_keypoint_t* keys,
                         const uint8_t* desc, int n_kp, int n_mp, int width, int height,
                         orb_mp_track_t* mps, uint8_t* mp_desc, uint8_t* kp_locked);

/* Library / device info. */
int orb_abi_version(void);
orb_status_t orb_device_count(int* n);
const char* orb_status_string(orb_status_t s);

#ifdef __cplusplus
}
#endif
#endif /* ORB_ABI_H */
