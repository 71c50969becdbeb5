/*
 * orbx.h — C-ABI of the MI355X-native ORB front-end and Hamming matchers (liborbx.so).
 *
 * Drop-in boundary for the hot path of andresenwc/MultiAgent_ORB_SLAM2 (reference paths below are
 * relative to the reference root).  The reference's C++ classes ORB_SLAM2::ORBextractor
 * (include/ORBextractor.h:45-111) and ORB_SLAM2::ORBmatcher (include/ORBmatcher.h:37-102) keep their
 * signatures; their bodies call the functions below (adapter in INTEGRATION.md).  Plain pointers and
 * sizes only; every function returns an int status (ORBX_OK = 0, < 0 on error; text via
 * orbx_last_error()) and never throws.  Host buffers are owned by the caller, device buffers made by
 * a context are owned by the context.  Threads:
 *   - an extractor or a fusion object is used by one host thread at a time (the reference constructs one
 *     ORBextractor per camera per agent, Tracking.cc:119-125);
 *   - a matcher and a keyframe database may be shared by any number of threads, like the reference's
 *     KeyFrameDatabase (its mMutex, KeyFrameDatabase.cc:42-316): each call holds the object's lock while it
 *     runs, and a call's stream is ordered after the previous call's device work on the object's state
 *     (matcher scratch; database BowVectors, membership, scratch fields), whatever stream that ran on -- so
 *     operations take effect in the order their calls took the lock;
 *   - distinct objects may be used concurrently from different threads.
 *
 * "_device" entry points take device pointers and a hipStream_t (passed as void*; NULL = the HIP
 * null stream, as in the HIP API) and do not synchronise; all other entry points take host pointers,
 * run on the context's own stream and return after the results are in host memory.
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORBX_OK = 0,
    ORBX_ERR_ARG = -1,        /* invalid argument */
    ORBX_ERR_HIP = -2,        /* HIP runtime error (no device, launch failure, OOM) */
    ORBX_ERR_CAPACITY = -3,   /* output capacity too small; *n_out holds the required count */
    ORBX_ERR_UNSUPPORTED = -4 /* configuration outside the compiled limits */
};

/* Layout-identical to cv::KeyPoint (28 B): pt.x, pt.y, size, angle, response, octave, class_id. */
typedef struct orbx_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbx_keypoint;

/* Last error message of the calling thread ("" if none). */
const char* orbx_last_error(void);
/* Library version string. */
const char* orbx_version(void);
/* Number of visible HIP devices (0 when none; never fails). */
int orbx_device_count(void);
/* Waits for every stream of `device` and returns ORBX_ERR_HIP (message in orbx_last_error) if the device holds a
 * pending error -- a kernel fault, an illegal address.  For a caller's shutdown path: a fault after the last result
 * must not end in exit status 0. */
int orbx_device_check(int device);

/* A non-blocking stream on `device` (no reference counterpart: scheduling plumbing for device-API callers).
 * cu_exclude > 0 leaves that many compute units out of the stream's CU mask (spread over the device), so that
 * streams without a mask keep free CUs for latency-bound work; cu_exclude = -k keeps only k CUs (every (CUs / k)-th);
 * cu_exclude = 0: a plain stream of `priority`.
 * *out receives the hipStream_t. */
int orbx_stream_create(int device, int priority, int cu_exclude, void** out);
int orbx_stream_destroy(void* stream);

/* ------------------------------------------------------------------------------------------------
 * Extractor — replaces ORBextractor (src/ORBextractor.cc:410-1132)
 * ---------------------------------------------------------------------------------------------- */
typedef struct orbx_extractor orbx_extractor;

/* ORBextractor::ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
 * (src/ORBextractor.cc:410-470).  Binds the context to 'device' (HIP ordinal) and creates its stream. */
int orbx_extractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                          int device, orbx_extractor** out);
int orbx_extractor_destroy(orbx_extractor* ex);

/* Getters — ORBextractor::GetLevels/GetScaleFactor/GetScaleFactors/GetInverseScaleFactors/
 * GetScaleSigmaSquares/GetInverseScaleSigmaSquares (include/ORBextractor.h:63-83).  Arrays hold nlevels. */
int orbx_extractor_get_levels(const orbx_extractor* ex);
float orbx_extractor_get_scale_factor(const orbx_extractor* ex);
int orbx_extractor_get_scale_factors(const orbx_extractor* ex, float* out);
int orbx_extractor_get_inverse_scale_factors(const orbx_extractor* ex, float* out);
int orbx_extractor_get_scale_sigma_squares(const orbx_extractor* ex, float* out);
int orbx_extractor_get_inverse_scale_sigma_squares(const orbx_extractor* ex, float* out);
/* mnFeaturesPerLevel (src/ORBextractor.cc:435-446). */
int orbx_extractor_get_features_per_level(const orbx_extractor* ex, int* out);

/* Configure the context for images of rows x cols, up to max_batch images per device call
 * (allocates HBM once).  Called implicitly by orbx_extract with max_batch 1.  Limits (ORBX_ERR_UNSUPPORTED past
 * them): < 2^15 FAST cells and < 2^24 candidate slots per level (3840 x 2160 is tested), < 8,192 DistributeOctTree
 * nodes per level (about nfeatures 37,000 at scaleFactor 1.2 / 8 levels); the stereo calls take <= 4,096 keypoints
 * per image. */
int orbx_extractor_reserve(orbx_extractor* ex, int rows, int cols, int max_batch);
/* Maximum keypoints one image can yield for rows x cols (output capacity to allocate). */
int orbx_extractor_max_keypoints(orbx_extractor* ex, int rows, int cols);
/* Pyramid geometry for rows x cols: level sizes (nlevels each). */
int orbx_extractor_level_sizes(orbx_extractor* ex, int rows, int cols, int* level_rows, int* level_cols);

/* ORBextractor::operator()(image, mask, keypoints, descriptors) (src/ORBextractor.cc:1043-1105).
 * image: host 8UC1, rows x cols, row stride 'step' bytes.  Writes *n_out keypoints (level-major,
 * quadtree order within a level, coordinates scaled to level 0) and n_out x 32 descriptor bytes.
 * An empty image (rows or cols 0) returns ORBX_OK with *n_out = 0 (reference: :1046-1047).
 * If capacity < needed, returns ORBX_ERR_CAPACITY with *n_out = needed and writes nothing. */
int orbx_extract(orbx_extractor* ex, const uint8_t* image, int rows, int cols, size_t step,
                 orbx_keypoint* keypoints, uint8_t* descriptors, int capacity, int* n_out);
/* The stereo Frame constructor's two extractions (src/Frame.cc:78-81: mpORBextractorLeft on the left image and
 * mpORBextractorRight on the right one, in two threads) from ONE host thread: both are enqueued before either is
 * waited for, so they run together on the two extractors' streams.  Same outputs and error behaviour as two
 * orbx_extract calls (an empty image gives 0 keypoints for its side); left and right must be distinct extractors. */
int orbx_extract_pair(orbx_extractor* left, orbx_extractor* right, const uint8_t* image_left, size_t step_left,
                      const uint8_t* image_right, size_t step_right, int rows, int cols, orbx_keypoint* keypoints_left,
                      uint8_t* descriptors_left, int capacity_left, int* n_left, orbx_keypoint* keypoints_right,
                      uint8_t* descriptors_right, int capacity_right, int* n_right);

/* mvImagePyramid (include/ORBextractor.h:85): copy level 'level' of image 'index' of the last call
 * into a host buffer with row stride dst_step (unpadded level view, as Frame::ComputeStereoMatches
 * reads it, src/Frame.cc:563-580). */
int orbx_extractor_copy_level(orbx_extractor* ex, int index, int level, uint8_t* dst, size_t dst_step);

/* Batched device entry: 'batch' images of rows x cols at d_images + i*image_stride (row stride 'step').
 * Outputs per image i: d_keypoints[i*capacity ...], d_descriptors[(i*capacity ...)*32], d_counts[i].
 * capacity must be >= orbx_extractor_max_keypoints(). */
int orbx_extract_batch_device(orbx_extractor* ex, const uint8_t* d_images, int batch, int rows, int cols,
                              size_t step, size_t image_stride, orbx_keypoint* d_keypoints,
                              uint8_t* d_descriptors, int32_t* d_counts, int capacity, void* stream);
/* The same with two streams: the inputs are read in in_stream order and the outputs (keypoints, descriptors,
 * counts) are complete in out_stream order.  Everything up to DistributeOctTree runs on in_stream (and the
 * extractor's side stream); the descriptor stage runs on out_stream, so a caller that issues call k+1 on
 * in_stream overlaps it with call k's descriptor stage.  The extractor orders its own buffer reuse across calls
 * (call k+1's quadtree / blur wait for call k's descriptor stage; a pyramid set's resize waits for the last
 * descriptor stage that read it); the pyramid of the call (orbx_extractor_pyramid_device) is complete in
 * out_stream order too.  out_stream == in_stream is orbx_extract_batch_device. */
int orbx_extract_batch_device_split(orbx_extractor* ex, const uint8_t* d_images, int batch, int rows, int cols,
                                    size_t step, size_t image_stride, orbx_keypoint* d_keypoints,
                                    uint8_t* d_descriptors, int32_t* d_counts, int capacity, void* in_stream,
                                    void* out_stream);

/* The image pyramids of the last extraction call, as one device-side description (what
 * ORBextractor::mvImagePyramid exposes, include/ORBextractor.h:85): level 0 of image i is the caller's
 * image at level0 + i*level0_image_stride (row step level0_step); level l >= 1 of image i is at
 * levels + i*image_stride + offset[l] with row step cols[l].  scale / inv_scale: mvScaleFactor /
 * mvInvScaleFactor.  Valid until the next call on the extractor (and while the caller keeps level 0);
 * with a pyramid ring of n sets (orbx_extractor_set_pyramid_ring), until the n-th next call. */
#define ORBX_MAX_LEVELS 32
typedef struct orbx_pyramid {
    int nlevels, batch;
    const uint8_t* level0;
    size_t level0_step, level0_image_stride;
    const uint8_t* levels;
    size_t image_stride;
    size_t offset[ORBX_MAX_LEVELS];
    int rows[ORBX_MAX_LEVELS], cols[ORBX_MAX_LEVELS];
    float scale[ORBX_MAX_LEVELS], inv_scale[ORBX_MAX_LEVELS];
} orbx_pyramid;
int orbx_extractor_pyramid_device(const orbx_extractor* ex, orbx_pyramid* out);

/* Number of pyramid sets the extractor cycles through (1..8, default 1).  In the reference each Frame
 * owns its extractor's mvImagePyramid until the next Frame is built (src/Frame.cc:78-81, used by
 * ComputeStereoMatches :598-640); a ring of 2 lets the caller run step k's stereo SAD refinement on
 * another stream while step k+1 extracts.  Reallocates the extractor's buffers. */
int orbx_extractor_set_pyramid_ring(orbx_extractor* ex, int n);

/* Device pointer and row step of pyramid level 'level' of image 'index' of the last call.  Level 0 is
 * the caller's input image itself (read in place, never copied): valid while the caller keeps it. */
int orbx_extractor_level_device(orbx_extractor* ex, int index, int level, const uint8_t** d_level,
                                int* rows, int* cols, size_t* step);

/* Diagnostics: host copy of the GaussianBlur'd level 'level' of image 'index' of the last call -- the whole level,
 * borders (REFLECT_101) included: what computeDescriptors reads (src/ORBextractor.cc:1085-1086 blurs a clone of
 * mvImagePyramid[level] with GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101)).  The reference keeps it internal; the
 * parity tests read it to check every blurred pixel, not only those around keypoints.  Waits for the extractor's
 * work.  ORBX_ERR_ARG before the first call. */
int orbx_extractor_copy_blurred_level(orbx_extractor* ex, int index, int level, uint8_t* dst, size_t dst_step);

/* Device-side error word of the extractor, after every call issued so far has finished (waits for them).
 * Bits: 1 = a level's quadtree exceeded its node capacity; 4 = ordering canary -- a descriptor stage found another
 * call's kept-keypoint stamp (a missing cross-call ordering edge; the host API returns ORBX_ERR_HIP for it).  The
 * device entry points cannot return these; a device-API caller polls them here.  reset != 0 clears the word. */
int orbx_extractor_status(orbx_extractor* ex, int* flags, int reset);

/* Diagnostics: a kernel occupying 'stream' for about 'ms' milliseconds (<= 2000), used by the ordering tests to
 * delay one stream so that a missing cross-stream edge shows deterministically. */
int orbx_debug_spin_device(void* stream, double ms);

/* Optional per-stage timing of device calls (HIP events on the launch stream).  When enabled, each
 * orbx_extract_batch_device records events around every stage; orbx_extractor_stage_times returns
 * the accumulated milliseconds per stage and the number of recorded calls.  Stage names via
 * orbx_extractor_stage_name. */
int orbx_extractor_enable_timing(orbx_extractor* ex, int enable);
int orbx_extractor_stage_count(void);
const char* orbx_extractor_stage_name(int stage);
int orbx_extractor_stage_times(orbx_extractor* ex, double* ms_per_stage, int* calls);

/* ------------------------------------------------------------------------------------------------
 * Matchers — replace ORBmatcher (src/ORBmatcher.cc) and the descriptor search of
 * Frame::ComputeStereoMatches (src/Frame.cc:466-552)
 * ---------------------------------------------------------------------------------------------- */
typedef struct orbx_matcher orbx_matcher;

/* ORBmatcher::ORBmatcher(nnratio, checkOri) (src/ORBmatcher.cc:41-43), bound to 'device'. */
int orbx_matcher_create(float nnratio, int checkOri, int device, orbx_matcher** out);
int orbx_matcher_destroy(orbx_matcher* m);

/* ORBmatcher::TH_HIGH / TH_LOW / HISTO_LENGTH (src/ORBmatcher.cc:37-39). */
int orbx_th_high(void);
int orbx_th_low(void);
int orbx_histo_length(void);

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1649-1665) for n row pairs (a_i, b_i), device. */
int orbx_descriptor_distance_device(orbx_matcher* m, const uint8_t* d_a, const uint8_t* d_b, int n,
                                    int32_t* d_dist, void* stream);

/* Brute-force all-pairs 256-bit Hamming: for each query row the smallest distance, the lowest train
 * index attaining it and the second smallest distance (multiset), with the reference's
 * best/second update rule (init 256, strict <; src/ORBmatcher.cc:568-598).  Host and device forms. */
int orbx_bf_match(orbx_matcher* m, const uint8_t* query, int nq, const uint8_t* train, int nt,
                  int32_t* best_idx, int32_t* best_dist, int32_t* second_dist);
int orbx_bf_match_device(orbx_matcher* m, const uint8_t* d_query, int nq, const uint8_t* d_train, int nt,
                         int32_t* d_best_idx, int32_t* d_best_dist, int32_t* d_second_dist, void* stream);
/* n_problems independent all-pairs matches in one launch (e.g. the L x R descriptor sets of a batch of stereo pairs,
 * or a query keyframe against many candidates): problem z reads nq queries at d_query + z*query_stride and nt train
 * rows at d_train + z*train_stride (bytes, multiples of 16) and writes outputs at z*nq.  nt = 0: every query gets
 * (-1, 256, 256). */
int orbx_bf_match_batch_device(orbx_matcher* m, const uint8_t* d_query, int nq, size_t query_stride, const uint8_t* d_train,
                               int nt, size_t train_stride, int n_problems, int32_t* d_best_idx, int32_t* d_best_dist,
                               int32_t* d_second_dist, void* stream);

/* Stereo L<->R descriptor search of Frame::ComputeStereoMatches (src/Frame.cc:466-552): for each left
 * keypoint, the right keypoint in the row band of (int)vL (+-2*scale[octave] rows), octave within +-1
 * and uR in [uL - bf/b, uL] with the smallest distance (init TH_HIGH, strict <, ties -> lowest right
 * index).  best_idx = -1 unless best_dist < (TH_HIGH+TH_LOW)/2.  scale_factors: nlevels entries;
 * rows = level-0 image rows.  Returns the number of accepted matches in *n_matched. */
int orbx_stereo_match(orbx_matcher* m, const orbx_keypoint* kpl, const uint8_t* desc_l, int nl,
                      const orbx_keypoint* kpr, const uint8_t* desc_r, int nr, const float* scale_factors,
                      int nlevels, int rows, float bf, float b, int32_t* best_idx, int32_t* best_dist,
                      int* n_matched);
/* Batched device form over 'batch' stereo pairs laid out like orbx_extract_batch_device output
 * (keypoints/descriptors at i*capacity, counts per image).  Outputs at i*capacity. */
int orbx_stereo_match_batch_device(orbx_matcher* m, const orbx_keypoint* d_kpl, const uint8_t* d_desc_l,
                                   const int32_t* d_nl, const orbx_keypoint* d_kpr, const uint8_t* d_desc_r,
                                   const int32_t* d_nr, int batch, int capacity, const float* scale_factors,
                                   int nlevels, int rows, float bf, float b, int32_t* d_best_idx,
                                   int32_t* d_best_dist, void* stream);

/* The sub-pixel half of Frame::ComputeStereoMatches (src/Frame.cc:554-639) over 'batch' stereo pairs, after
 * orbx_stereo_match_batch_device: for each left keypoint with an accepted right match, the 11x11 SAD
 * window slid over +-5 px on the left keypoint's pyramid level (left image left_first+i of 'left', right
 * image right_first+i of 'right' -- the same pyramid when one extractor made both), parabola fit,
 * disparity check in [0, bf/b), then the median-SAD outlier rejection per pair (thDist = 1.5*1.4*median).
 * Outputs mvuRight / mvDepth (-1 = no stereo) at i*capacity + iL for iL < capacity. */
int orbx_stereo_refine_batch_device(orbx_matcher* m, const orbx_keypoint* d_kpl, const int32_t* d_nl,
                                    const orbx_keypoint* d_kpr, const int32_t* d_best_idx, int batch, int capacity,
                                    const orbx_pyramid* left, int left_first, const orbx_pyramid* right,
                                    int right_first, float bf, float b, float* d_uright, float* d_depth,
                                    void* stream);

/* The stereo Frame constructor's ORB work in one call (src/Frame.cc:61-117: ExtractORB(0) / ExtractORB(1) on two
 * threads, :78-81, then ComputeStereoMatches, :101): the two extractions of orbx_extract_pair, then the stereo search
 * and SAD refinement on their device outputs (no host round trip of the keypoints between them), host keypoints /
 * descriptors / uright / depth out -- the same values as orbx_extract_pair + orbx_compute_stereo_matches.  uright /
 * depth hold n_left entries.  An empty image on either side: the extractions only, no stereo matches. */
int orbx_stereo_frame(orbx_matcher* m, orbx_extractor* left, orbx_extractor* right, const uint8_t* image_left,
                      size_t step_left, const uint8_t* image_right, size_t step_right, int rows, int cols,
                      orbx_keypoint* kps_left, uint8_t* desc_left, int capacity_left, int* n_left, orbx_keypoint* kps_right,
                      uint8_t* desc_right, int capacity_right, int* n_right, float bf, float b, float* uright, float* depth,
                      int* n_stereo);
/* Frame::ComputeStereoMatches (src/Frame.cc:466-639) as one host call: the keypoints/descriptors the two
 * extractors returned from their last host orbx_extract, whose pyramids (image 0) it reads, like the
 * reference reads mpORBextractorLeft/Right->mvImagePyramid.  uright/depth: nl floats (-1 = none);
 * *n_stereo = keypoints with depth. */
int orbx_compute_stereo_matches(orbx_matcher* m, const orbx_extractor* left, const orbx_extractor* right,
                                const orbx_keypoint* kpl, const uint8_t* desc_l, int nl, const orbx_keypoint* kpr,
                                const uint8_t* desc_r, int nr, float bf, float b, float* uright, float* depth,
                                int* n_stereo);

/* DBoW2::FeatureVector (Thirdparty/DBoW2/DBoW2/FeatureVector.h:21-22) as CSR: node ids ascending,
 * offsets[n_nodes+1], feature indices (ascending within a node). */
typedef struct orbx_featvec {
    const uint32_t* node_ids;
    const int32_t* offsets;
    int n_nodes;
    const int32_t* indices;
} orbx_featvec;

/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (src/ORBmatcher.cc:524-657).
 * valid1/valid2[i] != 0 when keypoint i has a non-bad MapPoint.  match12[i] = KF2 index or -1. */
int orbx_search_by_bow_kfkf(orbx_matcher* m, const uint8_t* desc1, const float* angle1, const uint8_t* valid1,
                            int n1, orbx_featvec fv1, const uint8_t* desc2, const float* angle2,
                            const uint8_t* valid2, int n2, orbx_featvec fv2, int32_t* match12, int* n_matches);

/* A keyframe store on the device: slot k's field F lives at (const uint8_t*)F + k * F_stride (bytes), so the
 * same struct describes the batch outputs of orbx_extract_batch_device / orbx_vocab_transform_batch_device
 * (field-major: desc_stride = capacity*32, ...) and an array of exchanged keyframe packets (slot-major: every
 * stride = packet bytes).  desc and kps must be 16- and 4-byte aligned per slot.
 *   desc[capacity][32], kps[capacity] (KeyPoint::angle used), valid[capacity] (keypoint has a non-bad
 *   MapPoint), FeatureVector CSR fv_nodes[n_fv] / fv_offsets[n_fv+1] / fv_indices, n_fv (int32). */
typedef struct orbx_kf_store {
    const uint8_t* desc;        size_t desc_stride;
    const orbx_keypoint* kps;   size_t kps_stride;
    const uint8_t* valid;       size_t valid_stride;
    const uint32_t* fv_nodes;   size_t fv_nodes_stride;
    const int32_t* fv_offsets;  size_t fv_offsets_stride;
    const int32_t* fv_indices;  size_t fv_indices_stride;
    const int32_t* n_fv;        size_t n_fv_stride;
    int capacity;
} orbx_kf_store;

/* Many SearchByBoW(KeyFrame*, KeyFrame*) pairs in one launch over a device keyframe store — MapFusion's
 * cross-agent matches (src/MapFusion.cc:275 ComputeSim3, :849 CovisibilityDiscovery) and LoopClosing's
 * (src/LoopClosing.cc ComputeSim3).  d_pairs: n_pairs (kf1, kf2) slot pairs (int32; a pair with a negative
 * slot is padding and gets no matches); max_fv_nodes is the
 * launch width per pair (workgroups stride over kf1's FeatureVector nodes, so any value >= 1 is correct; the
 * largest node count is the fastest).  Outputs: d_match12[p*capacity + i1] = KF2 index or -1, d_nmatches[p]. */
int orbx_search_by_bow_kfkf_pairs_device(orbx_matcher* m, const orbx_kf_store* store, const int32_t* d_pairs,
                                         int n_pairs, int max_fv_nodes, int32_t* d_match12, int32_t* d_nmatches,
                                         void* stream);
/* orbx_distinctive_descriptors over a keyframe store (see above): observation o = (slot d_obs[2o], keypoint
 * d_obs[2o+1]). */
int orbx_distinctive_descriptors_store_device(orbx_matcher* m, const orbx_kf_store* store, const int32_t* d_obs,
                                              const int32_t* d_offsets, int n_mappoints, int32_t* d_best,
                                              uint8_t* d_out_desc, void* stream);

/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:246-311) for n_mappoints MapPoints at once.  MapPoint p's
 * observed descriptors -- the rows of its non-bad observing keyframes, in mObservations order (the caller
 * flattens them) -- are desc[offsets[p] .. offsets[p+1]) (32 B each).  best[p] = the index, within p's list, of
 * the descriptor with the least median distance to the others (the reference's first strict minimum of
 * vDists[(size_t)(0.5*(N-1))] over rows of the all-pairs Hamming table), -1 for a MapPoint without observations
 * (the reference returns, leaving mDescriptor unchanged).  out_desc[p] (may be NULL) = that descriptor
 * (mDescriptor; the device forms write a zero row for a MapPoint without observations).  Host form and device forms; the _store_ form reads observation o as keypoint obs[2o+1] of
 * keyframe slot obs[2o] of a device keyframe store (e.g. MapFusion's packet ring). */
int orbx_distinctive_descriptors(orbx_matcher* m, const uint8_t* desc, const int32_t* offsets, int n_mappoints, int32_t* best,
                                 uint8_t* out_desc);
int orbx_distinctive_descriptors_device(orbx_matcher* m, const uint8_t* d_desc, const int32_t* d_offsets, int n_mappoints,
                                        int32_t* d_best, uint8_t* d_out_desc, void* stream);

/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:161-290).
 * validk[i] != 0 when KF keypoint i has a non-bad MapPoint.  matchf[j] = KF index or -1. */
int orbx_search_by_bow_kff(orbx_matcher* m, const uint8_t* desck, const float* anglek, const uint8_t* validk,
                           int nk, orbx_featvec fvk, const uint8_t* descf, const float* anglef, int nf,
                           orbx_featvec fvf, int32_t* matchf, int* n_matches);

/* ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:659-825).  has_mp1/2: keypoint already has a
 * MapPoint; uright1/2 >= 0 marks stereo keypoints; F12 row-major 3x3; sigma2_2/scale_2: KF2 level
 * tables; (ex, ey): epipole of KF1 in KF2.  match12[i] = KF2 index or -1 (pairs in idx1 order). */
int orbx_search_for_triangulation(orbx_matcher* m, const uint8_t* desc1, const orbx_keypoint* kp1,
                                  const uint8_t* has_mp1, const float* uright1, int n1, orbx_featvec fv1,
                                  const uint8_t* desc2, const orbx_keypoint* kp2, const uint8_t* has_mp2,
                                  const float* uright2, int n2, orbx_featvec fv2, const float* F12,
                                  const float* sigma2_2, const float* scale_2, int nlevels, float ex, float ey,
                                  int only_stereo, int32_t* match12, int* n_matches);

/* SearchForTriangulation for many (kf1, kf2) slot pairs of a device keyframe store in one launch -- LocalMapping::
 * CreateNewMapPoints' loop over the new keyframe's best covisible neighbours (src/LocalMapping.cc:243-274).
 * d_has_mp: per-slot "keypoint already has a MapPoint" rows at d_has_mp + k*has_mp_stride bytes (NULL = the store's
 * valid field; stride 0 = one row for every slot); d_uright: per-slot mvuRight rows likewise (NULL = no stereo keypoints); d_geom[p]: F12 (row-major) and the epipole of KF1 in KF2 for pair p; sigma2_2 / scale_2: KF2's
 * level tables (host).  Outputs d_match12[p*capacity + i1] = KF2 index or -1, d_nmatches[p]; the matcher's
 * checkOri applies (CreateNewMapPoints uses ORBmatcher(0.6, false)). */
typedef struct orbx_tri_geom {
    float F12[9];
    float ex, ey;
    float pad;
} orbx_tri_geom;
int orbx_search_for_triangulation_pairs_device(orbx_matcher* m, const orbx_kf_store* store, const uint8_t* d_has_mp,
                                               size_t has_mp_stride, const float* d_uright, size_t uright_stride, const int32_t* d_pairs, const orbx_tri_geom* d_geom,
                                               int n_pairs, int max_fv_nodes, const float* sigma2_2, const float* scale_2,
                                               int nlevels, int only_stereo, int32_t* d_match12, int32_t* d_nmatches,
                                               void* stream);

/* ComputeDistinctiveDescriptors of the MapPoints CreateNewMapPoints makes after the batched SearchForTriangulation
 * above (LocalMapping.cc:440-448), read from the match table itself: keypoint i of keyframe d_new_slots[j] becomes
 * MapPoint j*capacity + i with the first neighbour k (in order, d_neighbours[j*n_neighbours + k] >= 0) whose match
 * d_match12[(j*n_neighbours + k)*capacity + i] >= 0 -- a keypoint becomes a MapPoint at most once -- and observations
 * [(that neighbour, its match), (the new keyframe, i)] in creation order (mObservations is keyed by KeyFrame*; pinned
 * to creation order).  Two descriptors: both medians are 0, row 0 wins (MapPoint.cc:293-306).  d_best[mp]
 * = 0, or -1 without a MapPoint (a zero row written then); d_out_desc[mp] (or NULL) = the chosen descriptor.
 * n_neighbours <= 64. */
int orbx_distinctive_descriptors_neighbours_device(orbx_matcher* m, const orbx_kf_store* store, const int32_t* d_new_slots,
                                                   const int32_t* d_neighbours, int n_new, int n_neighbours,
                                                   const int32_t* d_match12, int32_t* d_best, uint8_t* d_out_desc,
                                                   void* stream);

/* ------------------------------------------------------------------------------------------------
 * Keypoint grid and the projection / radius matchers.
 * The reference's callers project each MapPoint before searching (cv::Mat products, PredictScale,
 * src/ORBmatcher.cc); a query carries what that projection hands to the search: the window of
 * GetFeaturesInArea and the values the reference's inner loop tests.
 * ---------------------------------------------------------------------------------------------- */
/* Frame grid (FRAME_GRID_COLS 64 x FRAME_GRID_ROWS 48, include/Frame.h:37-38): image bounds and inverse
 * cell size as the Frame constructor computes them (src/Frame.cc:99-104, :436-464). */
typedef struct orbx_grid {
    float min_x, min_y, max_x, max_y;
    float inv_w, inv_h;          /* mfGridElementWidthInv, mfGridElementHeightInv */
    int32_t cols, rows;
} orbx_grid;

enum {
    ORBX_PROJ_MAPPOINTS = 0, /* SearchByProjection(Frame&, vpMapPoints, th)             src/ORBmatcher.cc:45-131 */
    ORBX_PROJ_LASTFRAME = 1, /* SearchByProjection(Frame&, const Frame&, th, bMono)     :1330-1472 */
    ORBX_PROJ_KEYFRAME = 2,  /* SearchByProjection(Frame&, KeyFrame*, sFound, th, ORBdist) :1474-1601 */
    ORBX_PROJ_SIM3 = 3,      /* SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) :292-405 */
    ORBX_PROJ_FUSE = 4,      /* Fuse(KeyFrame*, vpMapPoints, th), its search             :894-951 */
    ORBX_PROJ_BEST = 5,      /* Fuse(KeyFrame*, Scw, ...) :1053-1081; SearchBySim3's two searches :1193-1226, :1273-1306 */
    ORBX_PROJ_INIT = 6       /* SearchForInitialization                                  :407-522 */
};
enum { ORBX_QF_SKIP = 1,     /* query absent (bad MapPoint, not in view, already found, level > 0 for INIT) */
       ORBX_QF_BLOCKS = 2 }; /* an assignment by this query excludes the keypoint from later queries
                                (MAPPOINTS/LASTFRAME: the MapPoint has Observations() > 0; KEYFRAME/SIM3: always) */

/* One projected MapPoint (or, for INIT, one F1 keypoint). 40 bytes. */
typedef struct orbx_proj_query {
    float x, y, r;                /* GetFeaturesInArea(x, y, r, ...) window: projection u, v and radius */
    int32_t min_level, max_level; /* Frame::GetFeaturesInArea level arguments (tested iff min > 0 || max >= 0) */
    float ur, ur_tol;             /* MAPPOINTS/LASTFRAME: skip candidates with uright > 0 && |ur - uright| > ur_tol
                                     (ur_tol < 0: off); FUSE: ur = u - bf/z for the stereo reprojection error */
    float angle;                  /* the query keypoint's angle (rotation-consistency histogram) */
    int32_t level;                /* reserved (predicted level) */
    int32_t flags;                /* ORBX_QF_* */
} orbx_proj_query;

typedef struct orbx_proj_params {
    int32_t mode;                 /* ORBX_PROJ_* */
    int32_t accept_max;           /* accept if bestDist <= accept_max: TH_HIGH, TH_LOW or ORBdist */
    float nnratio;                /* MAPPOINTS same-level ratio (:122) / INIT ratio (:463) */
    int32_t check_ori;            /* rotation-consistency filter (LASTFRAME, KEYFRAME, INIT) */
    int32_t nlevels;
    float inv_sigma2[32];         /* mvInvLevelSigma2 of the target view (FUSE reprojection test :927, :938) */
} orbx_proj_params;

/* One search problem on the device: a query set against one target view with its grid (CSR cells
 * from orbx_grid_build_device).  blocked[idx] != 0: the target keypoint already holds an excluding
 * MapPoint (MAPPOINTS/LASTFRAME: Observations() > 0; KEYFRAME: any; SIM3: vpMatched[idx]); NULL = none.
 * Outputs: q_idx/q_dist per query (accepted keypoint or -1; INIT: vnMatches12); owner[idx] for modes
 * MAPPOINTS..SIM3 (-1 untouched, q = the MapPoint of query q, -2 = set to NULL by the rotation filter);
 * *nmatches as the reference returns it. */
typedef struct orbx_proj_problem {
    const orbx_proj_query* queries; const uint8_t* qdesc; int32_t nq;
    const orbx_keypoint* kps; const uint8_t* desc; const float* uright; const uint8_t* blocked; int32_t n;
    const int32_t* cell_start; const int32_t* cell_idx;
    int32_t* q_idx; int32_t* q_dist; int32_t* owner; int32_t* nmatches;
} orbx_proj_problem;

/* Frame::UndistortKeyPoints (src/Frame.cc:404-434): mvKeysUn = mvKeys with pt replaced by cv::undistortPoints(pt, K,
 * DistCoef, R = I, P = K), pinned to OpenCV 3.2's cvUndistortPoints (double precision, five fixed iterations; the
 * oracle restates it).  K: 3x3 row-major float (mK); dist: n_dist = 0, 4, 5, 8 or 12 coefficients (k1 k2 p1 p2 [k3
 * [k4 k5 k6 [s1..s4]]]); dist[0] == 0 copies the keypoints unchanged (:406-410), as the reference does. */
int orbx_undistort_keypoints(orbx_matcher* m, const orbx_keypoint* kps, int n, const float* K, const float* dist, int n_dist,
                             orbx_keypoint* out);
/* Device form over an extractor batch (keypoints at i*capacity, d_counts[i]); K / dist are host arrays. */
int orbx_undistort_keypoints_device(orbx_matcher* m, const orbx_keypoint* d_kps, const int32_t* d_counts, int batch, int capacity,
                                    const float* K, const float* dist, int n_dist, orbx_keypoint* d_out, void* stream);
/* Frame::ComputeImageBounds (src/Frame.cc:436-464): bounds = {mnMinX, mnMaxX, mnMinY, mnMaxY} of the undistorted image
 * corners (or the image rectangle when dist[0] == 0). */
int orbx_compute_image_bounds(orbx_matcher* m, const float* K, const float* dist, int n_dist, int cols, int rows,
                              float* bounds);

/* Frame::AssignFeaturesToGrid (src/Frame.cc:230-245) for 'batch' keypoint sets laid out like the
 * orbx_extract_batch_device output: cell (ix, iy) -> CSR row ix*rows + iy at d_cell_start + i*(cols*rows+1),
 * keypoint indices ascending inside a cell at d_cell_idx + i*capacity.  capacity <= 8192. */
int orbx_grid_build_device(orbx_matcher* m, orbx_grid grid, const orbx_keypoint* d_kps, const int32_t* d_counts,
                           int batch, int capacity, int32_t* d_cell_start, int32_t* d_cell_idx, void* stream);
/* The searches of n_problems problems (device array) in one launch; max_n / max_nq bound the target
 * keypoints / queries of any problem (they size the launch's LDS plan).  A problem above either bound is not
 * searched: its q_idx / q_dist are -1 and its *nmatches is -1. */
int orbx_proj_search_batch_device(orbx_matcher* m, const orbx_proj_params* params, orbx_grid grid,
                                  const orbx_proj_problem* d_problems, int n_problems, int max_n, int max_nq,
                                  void* stream);
/* As orbx_proj_search_batch_device, with each problem's grid built inside its search: problem p's cell_start /
 * cell_idx are OUTPUTS, Frame::AssignFeaturesToGrid (src/Frame.cc:230-245) of its first d_grid_counts[p] (<= n) target
 * keypoints -- the same CSR arrays as orbx_grid_build_device, for later searches of the frame -- so a frame's first
 * search (Tracking::TrackWithMotionModel's, on a fresh Frame) needs no separate grid launch.  A problem with
 * d_grid_counts[p] < 0 reads its grid (inputs, as orbx_proj_search_batch_device); problems of one launch that build the
 * grid of the same keypoint set write identical arrays.  Not for
 * ORBX_PROJ_INIT; ORBX_ERR_UNSUPPORTED when the grid and the keypoints do not fit the launch's LDS plan.  A problem
 * above max_n / max_nq is not searched (as above) and its grid is written empty: every cell_start entry 0. */
int orbx_proj_search_grid_batch_device(orbx_matcher* m, const orbx_proj_params* params, orbx_grid grid,
                                       const orbx_proj_problem* d_problems, int n_problems, int max_n, int max_nq,
                                       const int32_t* d_grid_counts, void* stream);
/* Host form: one query set against one view (host buffers; uright / blocked / owner may be NULL). */
int orbx_proj_search(orbx_matcher* m, const orbx_proj_params* params, orbx_grid grid, const orbx_proj_query* queries,
                     const uint8_t* qdesc, int nq, const orbx_keypoint* kps, const uint8_t* desc, const float* uright,
                     const uint8_t* blocked, int n, int32_t* q_idx, int32_t* q_dist, int32_t* owner, int* n_matches);

/* The projection step in front of the search: the per-MapPoint arithmetic the reference runs before it calls
 * GetFeaturesInArea, producing the orbx_proj_query the search consumes.
 *   ORBX_PROJ_LASTFRAME  SearchByProjection(Frame&, const Frame&, th, bMono)   src/ORBmatcher.cc:1363-1392, :1418-1426
 *   ORBX_PROJ_MAPPOINTS  Frame::isInFrustum (src/Frame.cc:269-325, viewingCosLimit) + the window of
 *                        SearchByProjection(Frame&, vpMapPoints, th)           src/ORBmatcher.cc:62-71, :92-98
 *   ORBX_PROJ_FUSE       Fuse(KeyFrame*, vpMapPoints, th)                       src/ORBmatcher.cc:854-893
 * A point that fails a test (negative depth, outside the image, outside the scale-invariance distances, viewing angle)
 * gets ORBX_QF_SKIP; a point whose flags already hold ORBX_QF_SKIP (NULL, bad, outlier, already matched, IsInKeyFrame)
 * stays skipped.  Pinned arithmetic: Rcw * X + tcw as float products summed left to right, cv::norm and
 * Mat::dot with float products accumulated in double, PredictScale (src/MapPoint.cc:389-421) with a double log. */
typedef struct orbx_map_point {
    float x, y, z;                /* GetWorldPos */
    float nx, ny, nz;             /* GetNormal (MAPPOINTS, FUSE) */
    float min_dist, max_dist;     /* mfMinDistance, mfMaxDistance (GetMin/MaxDistanceInvariance apply 0.8 / 1.2) */
    float angle;                  /* LASTFRAME: LastFrame.mvKeysUn[i].angle (the rotation histogram) */
    int32_t octave;               /* LASTFRAME: LastFrame.mvKeys[i].octave */
    int32_t flags;                /* ORBX_QF_*: carried into the query (BLOCKS = Observations() > 0) */
    int32_t pad;
} orbx_map_point;                 /* 48 bytes */

/* The view a set of MapPoints is projected into (the current Frame, or the KeyFrame of a Fuse). */
typedef struct orbx_view {
    float R[9], t[3], Ow[3];      /* Rcw (row-major), tcw, camera centre (GetCameraCenter / mOw) */
    float fx, fy, cx, cy, bf;     /* intrinsics and mbf */
    float min_x, max_x, min_y, max_y;   /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float th;                     /* the call's th (LASTFRAME radius factor, MAPPOINTS factor if != 1, Fuse radius) */
    float view_cos_limit;         /* MAPPOINTS: isInFrustum's viewingCosLimit (Tracking::SearchLocalPoints: 0.5) */
    int32_t level_mode;           /* LASTFRAME: 1 bForward, -1 bBackward, 0 neither (from the two poses, :1344-1352) */
    int32_t pad;
} orbx_view;                      /* 112 bytes */

/* n_views projections: view v projects point set s = d_view_points ? d_view_points[v] : v (points at
 * d_points + s * capacity, d_counts[s] of them) into d_views[v]; its queries are written at d_queries + v * capacity,
 * the rows past the set's count as ORBX_QF_SKIP (so a search may take nq = capacity).  Many views of one point set is
 * Fuse's shape (one KeyFrame's MapPoints into each of its neighbours, LocalMapping.cc:486-496).  scale_factors:
 * mvScaleFactors (nlevels); log_scale_factor: mfLogScaleFactor.  d_found (optional, laid out as the queries): points
 * with d_found[v * capacity + i] >= 0 are skipped -- the MapPoints the current frame already matched
 * (Tracking::SearchLocalPoints skips them, src/Tracking.cc:1160-1182). */
int orbx_proj_project_device(orbx_matcher* m, int mode, const orbx_map_point* d_points, const int32_t* d_counts, int n_views,
                             int capacity, const orbx_view* d_views, const int32_t* d_view_points, const float* scale_factors,
                             int nlevels, float log_scale_factor, const int32_t* d_found, orbx_proj_query* d_queries,
                             void* stream);

/* What SearchLocalPoints skips after SearchByProjection(CurrentFrame, LastFrame) (src/Tracking.cc:1160-1182), for
 * n_sets (query set, frame) pairs in one launch: d_found[s * n_queries + q] = 0 when MapPoint q is in the frame --
 * it was assigned a keypoint (k = d_q_idx[s * n_queries + q] >= 0) and that keypoint still holds it
 * (d_owner[s * n_keypoints + k] == q; the rotation filter resets the entries it drops, ORBmatcher.cc:1456-1466) --
 * else -1 (the d_found layout of orbx_proj_project_device); d_blocked[s * n_keypoints + i] (optional) = 1 when keypoint
 * i holds a MapPoint (owner >= 0), else 0 (a problem's `blocked` bytes).  Replaces the host loop over
 * mCurrentFrame.mvpMapPoints that sets mbTrackInView = false. */
int orbx_proj_found_device(orbx_matcher* m, const int32_t* d_q_idx, const int32_t* d_owner, int n_sets, int n_queries,
                           int n_keypoints, int32_t* d_found, uint8_t* d_blocked, void* stream);

/* MapPoints of stereo frames (Frame::UnprojectStereo src/Frame.cc:666-680 + MapPoint::MapPoint(Pos, pMap, pFrame, idxF)
 * src/MapPoint.cc:47-68, as Tracking::StereoInitialization / CreateNewKeyFrame / UpdateLastFrame create them):
 * for keypoint i of frame b with depth z > 0, X = Rwc * ((u - cx) z / fx, (v - cy) z / fy, z) + Ow, the normal
 * (X - Ow) / |X - Ow|, mfMaxDistance = |X - Ow| * mvScaleFactors[octave], mfMinDistance = max / mvScaleFactors[nlevels - 1],
 * octave and angle from the keypoint, flags = 'flags'; a keypoint without depth gets ORBX_QF_SKIP.  Keypoints at
 * d_kps + b * capacity (d_counts[b] each), depths at d_depth + b * capacity; d_twc: per frame Rwc (9, row-major) then
 * Ow (3) -- 12 floats; camera = {fx, fy, cx, cy}.  Output at d_points + b * capacity. */
int orbx_stereo_mappoints_device(orbx_matcher* m, const orbx_keypoint* d_kps, const float* d_depth, const int32_t* d_counts,
                                 int batch, int capacity, const float* d_twc, const float* camera, const float* scale_factors,
                                 int nlevels, int flags, orbx_map_point* d_points, void* stream);
/* A batch of new keyframes' orbx_stereo_mappoints_device and orbx_grid_build_device (same outputs) in one launch of
 * one workgroup per keyframe -- LocalMapping's keyframe insertion (src/LocalMapping.cc:157-200 with the KeyFrame's grid
 * of src/KeyFrame.cc:44-49) before SearchInNeighbors' Fuse reads both.  Grid outputs at d_cell_start + b *
 * (cols * rows + 1) and d_cell_idx + b * capacity. */
int orbx_keyframe_prep_device(orbx_matcher* m, const orbx_keypoint* d_kps, const float* d_depth, const int32_t* d_counts,
                              int batch, int capacity, const float* d_twc, const float* camera, const float* scale_factors,
                              int nlevels, int flags, orbx_map_point* d_points, orbx_grid grid, int32_t* d_cell_start,
                              int32_t* d_cell_idx, void* stream);
/* Host form: one point set, one view. */
int orbx_proj_project(orbx_matcher* m, int mode, const orbx_map_point* points, int n, const orbx_view* view,
                      const float* scale_factors, int nlevels, float log_scale_factor, orbx_proj_query* queries);

/* ------------------------------------------------------------------------------------------------
 * DBoW2 vocabulary — replaces TemplatedVocabulary<FORB>::transform (Thirdparty/DBoW2/DBoW2/
 * TemplatedVocabulary.h:1125-1259), i.e. Frame::ComputeBoW / KeyFrame::ComputeBoW (src/Frame.cc:395-402),
 * which produce the FeatureVector that SearchByBoW buckets on.  Supported: L1/L2 scoring with any
 * weighting (ORBvoc.txt is "10 6 0 0": k 10, L 6, L1_NORM, TF_IDF).
 * ---------------------------------------------------------------------------------------------- */
typedef struct orbx_vocab orbx_vocab;

/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424). */
int orbx_vocab_load_text(const char* path, int device, orbx_vocab** out);
/* The same tree from arrays: n_lines node lines in file order (node id = line + 1, root = 0): parent id,
 * is_leaf, 32-byte descriptor, weight. */
int orbx_vocab_create(int k, int L, int scoring, int weighting, int n_lines, const int32_t* parent,
                      const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device, orbx_vocab** out);
int orbx_vocab_destroy(orbx_vocab* v);
int orbx_vocab_info(const orbx_vocab* v, int* k, int* L, int* n_nodes, int* n_words);

/* transform(features, BowVector&, FeatureVector&, levelsup) for n descriptors (host buffers, n <= 4096).
 * BowVector: *n_words (word id ascending, value); FeatureVector: CSR with *n_fv_nodes node ids ascending,
 * fv_offsets[n_fv_nodes + 1], fv_indices (feature indices ascending within a node).  Capacities: n. */
int orbx_vocab_transform(orbx_vocab* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                         double* bow_values, int* n_words, uint32_t* fv_nodes, int32_t* fv_offsets,
                         int32_t* fv_indices, int* n_fv_nodes);
/* Per-descriptor transform(feature, word_id, weight, &nid, levelsup) (:1218-1259), device buffers. */
int orbx_vocab_words_device(orbx_vocab* v, const uint8_t* d_desc, int n, int levelsup, int32_t* d_word,
                            double* d_weight, int32_t* d_node, void* stream);
/* Batched device transform of 'batch' descriptor sets laid out like orbx_extract_batch_device output
 * (descriptors at i*capacity, d_counts[i]).  Per set i: words/weights/nodes and BoW arrays at i*capacity,
 * fv offsets at i*(capacity+1); d_n_words[i], d_n_fv_nodes[i].  capacity <= 4096. */
int orbx_vocab_transform_batch_device(orbx_vocab* v, const uint8_t* d_desc, const int32_t* d_counts, int batch,
                                      int capacity, int levelsup, int32_t* d_word, double* d_weight,
                                      int32_t* d_node, uint32_t* d_bow_words, double* d_bow_values,
                                      int32_t* d_n_words, uint32_t* d_fv_nodes, int32_t* d_fv_offsets,
                                      int32_t* d_fv_indices, int32_t* d_n_fv_nodes, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Keyframe database — replaces KeyFrameDatabase (src/KeyFrameDatabase.cc) and ORBVocabulary::score
 * (DBoW2 L1Scoring, Thirdparty/DBoW2/DBoW2/ScoringObject.cpp:23-66).  SURVEY §8f row 4: the inverted-
 * file candidate search that precedes every cross-agent SearchByBoW.
 *
 * A database is a table of max_slots keyframe slots.  A slot holds the keyframe's BowVector (word ids
 * ascending, DBoW2 values), its GetBestCovisibilityKeyFrames(10) list (src/KeyFrame.cc:189-197) and, per
 * query kind, the scratch fields the reference keeps on KeyFrame: mn*Query, mn*Words, m*Score
 * (include/KeyFrame.h:155-163; the scores are never initialised by the reference: here they start at 0
 * unless set with orbx_kfdb_set_state).  Membership (add / erase / clear) defines the inverted file.
 * A query names a slot for its BowVector (a Frame's BowVector for relocalisation goes in a spare slot) and
 * its id (KeyFrame::mnId / Frame::mnId).  Only L1 scoring is implemented (ORBvoc.txt: "10 6 0 0").
 * ---------------------------------------------------------------------------------------------- */
typedef struct orbx_kfdb orbx_kfdb;

enum {
    ORBX_KFDB_LOOP = 0,   /* DetectLoopCandidates (src/KeyFrameDatabase.cc:76-197): exclusions = GetConnectedKeyFrames() */
    ORBX_KFDB_COVIS = 1,  /* DetectCovisibilityCandidates (:199-308): exclusions = vpKFsToIgnore */
    ORBX_KFDB_RELOC = 2   /* DetectRelocalizationCandidates (:310-420): no exclusions, no minScore */
};

/* KeyFrameDatabase(voc) (:33-37): n_vocab_words = voc.size(); max_words <= 4096 BowVector entries per slot. */
int orbx_kfdb_create(int n_vocab_words, int max_slots, int max_words, int device, orbx_kfdb** out);
int orbx_kfdb_destroy(orbx_kfdb* db);
int orbx_kfdb_info(const orbx_kfdb* db, int* n_vocab_words, int* max_slots, int* max_words, int* n_members);
/* How a query finds the keyframes sharing its words (results are identical):
 * ORBX_KFDB_INVERTED walks the inverted file (rebuilt on the device after membership changes), as the
 * reference does; ORBX_KFDB_PAIRWISE intersects the query with every member's BowVector (no rebuild, cheaper
 * for small databases); ORBX_KFDB_WORDMAP reads, per query word, that word's row of a word x slot bit matrix
 * the database keeps beside the BowVectors (databases of <= 2048 slots whose matrix is <= 1 GB, e.g. 156 MB for
 * 1,224 slots over a 10^6-word vocabulary; ORBX_ERR_UNSUPPORTED otherwise); ORBX_KFDB_AUTO (default) picks the
 * word map when the database has one, else pairwise up to 2048 members, else the inverted file. */
enum { ORBX_KFDB_AUTO = 0, ORBX_KFDB_INVERTED = 1, ORBX_KFDB_PAIRWISE = 2, ORBX_KFDB_WORDMAP = 3 };
int orbx_kfdb_set_strategy(orbx_kfdb* db, int strategy);
/* Store a slot's BowVector (KeyFrame::mBowVec); word ids strictly ascending and < n_vocab_words. */
int orbx_kfdb_set_bow(orbx_kfdb* db, int slot, const uint32_t* words, const double* values, int n);
/* Device form: BowVector i (words at d_words + i*word_stride, values at d_values + i*value_stride, size
 * d_n_words[i*n_stride]; strides in elements) into slot d_slots[i], for i < n: an
 * orbx_vocab_transform_batch_device output (strides capacity, capacity, 1) or an array of exchanged
 * keyframe packets.  Word ids must satisfy the rules above. */
int orbx_kfdb_set_bow_device(orbx_kfdb* db, const int32_t* d_slots, int n, const uint32_t* d_words, long long word_stride,
                             const double* d_values, long long value_stride, const int32_t* d_n_words, long long n_stride,
                             void* stream);
/* GetBestCovisibilityKeyFrames(10) of slots[i]: best[i*10 .. i*10+9], best first, -1 padded. */
int orbx_kfdb_set_covisibility(orbx_kfdb* db, const int32_t* slots, int n, const int32_t* best);
/* KeyFrameDatabase::add (:40-46) in order (adding a slot already in the database is ORBX_ERR_ARG),
 * erase (:48-67; slots not in the database are ignored), clear (:69-73). */
int orbx_kfdb_add(orbx_kfdb* db, const int32_t* slots, int n);
int orbx_kfdb_erase(orbx_kfdb* db, const int32_t* slots, int n);
int orbx_kfdb_clear(orbx_kfdb* db);
/* The scratch fields of one query kind for all max_slots slots. */
int orbx_kfdb_get_state(orbx_kfdb* db, int kind, uint64_t* query, int32_t* words, float* score);
int orbx_kfdb_set_state(orbx_kfdb* db, int kind, const uint64_t* query, const int32_t* words, const float* score);
/* ORBVocabulary::score(bow[pairs[2i]], bow[pairs[2i+1]]) (first = v1), e.g. the minScore bound of
 * src/MapFusion.cc:800-815 and src/LoopClosing.cc DetectLoop. */
int orbx_kfdb_score(orbx_kfdb* db, const int32_t* pairs, int n, double* scores);
int orbx_kfdb_score_device(orbx_kfdb* db, const int32_t* d_pairs, int n, double* d_scores, void* stream);
/* nq queries of one kind, evaluated in order as the reference would evaluate them one after another.
 * min_scores[q]: minScore (ignored for RELOC, may be NULL).  Exclusions of query q:
 * excl_slots[excl_offsets[q] .. excl_offsets[q+1]) (excl_offsets NULL = none).  Candidates of query q:
 * out[out_offsets[q] .. out_offsets[q+1]) in the reference's order; ORBX_ERR_CAPACITY if out_cap is too
 * small or a query retains more than 2048 candidates. */
int orbx_kfdb_detect(orbx_kfdb* db, int kind, const int32_t* query_slots, const uint64_t* query_ids, const float* min_scores,
                     int nq, const int32_t* excl_offsets, const int32_t* excl_slots, int32_t* out_offsets, int32_t* out,
                     int out_cap);
/* Device form (device pointers, no synchronisation).  Outputs: d_out[q*out_stride ...], d_out_n[q];
 * *d_status |= 2 when a query exceeds out_stride or 2048 retained candidates, |= 1 when the queries of the
 * batch interact through the scratch fields (a query id equal to one already recorded in a slot another
 * query of the batch updates, or repeated ids): then the results are not the sequential ones, the scratch
 * fields hold the batched (not the sequential) updates, and the caller must treat the batch as failed (a
 * device caller cannot restore them; orbx_kfdb_detect snapshots and re-runs one query at a time itself).
 * Distinct, fresh query ids (monotonic mnId, as in the reference) never interact. */
int orbx_kfdb_detect_device(orbx_kfdb* db, int kind, const int32_t* d_query_slots, const uint64_t* d_query_ids,
                            const float* d_min_scores, int nq, const int32_t* d_excl_offsets, const int32_t* d_excl_slots,
                            int32_t* d_out, int out_stride, int32_t* d_out_n, int32_t* d_status, void* stream);
/* MapFusion's query-then-add order (src/MapFusion.cc:133 DetectFusionCandidates, then the keyframe is added to the
 * database, :149 / :222) for a whole batch in one call: the caller first adds the query slots with orbx_kfdb_add in
 * query order; query q then sees only the members added before its own slot (its own slot and every later query
 * slot are invisible to it), so the results equal detect(q0); add(q0); detect(q1); add(q1); ...  A query slot that
 * is not a member sees every member.  Otherwise as orbx_kfdb_detect / orbx_kfdb_detect_device. */
int orbx_kfdb_detect_sequential(orbx_kfdb* db, int kind, const int32_t* query_slots, const uint64_t* query_ids,
                                const float* min_scores, int nq, const int32_t* excl_offsets, const int32_t* excl_slots,
                                int32_t* out_offsets, int32_t* out, int out_cap);
int orbx_kfdb_detect_sequential_device(orbx_kfdb* db, int kind, const int32_t* d_query_slots, const uint64_t* d_query_ids,
                                       const float* d_min_scores, int nq, const int32_t* d_excl_offsets,
                                       const int32_t* d_excl_slots, int32_t* d_out, int out_stride, int32_t* d_out_n,
                                       int32_t* d_status, void* stream);
/* MapFusion's use of the candidates (src/MapFusion.cc:136-144, :275): for query q, the first k of its
 * candidates d_cand[q*cand_stride ..+ d_n_cand[q]) whose map differs from the query's
 * (d_slot_group[cand] != d_query_group[q]; both NULL = keep all, LoopClosing's own-map case) become
 * SearchByBoW pairs d_pairs[(q*k + j)*2 ..] = (query slot, candidate slot), padded with (query slot, -1)
 * (orbx_search_by_bow_kfkf_pairs_device skips those: no matches). */
int orbx_kfdb_candidate_pairs_device(const int32_t* d_cand, int cand_stride, const int32_t* d_n_cand, const int32_t* d_query_slots,
                                     int nq, const int32_t* d_slot_group, const int32_t* d_query_group, int k, int32_t* d_pairs,
                                     void* stream);


/* ------------------------------------------------------------------------------------------------
 * Keyframe fusion — one agent's keyframe path into MapFusion as one native object:
 * KeyFrame::ComputeBoW, the LoopClosing -> MultiAgentServer::InsertKeyFrame -> MapFusion::InsertKeyFrame hand-off
 * (src/LoopClosing.cc:83-94, src/MultiAgentServer.cc:78-80, src/MapFusion.cc:83-88), DetectLoopCandidates then
 * add (src/MapFusion.cc:133, :149 / :222), the same-map discard (:136-144) and SearchByBoW with the 20-match gate
 * (:275-281).  A keyframe is a fixed-size packet (orbx_packet_layout) in a device ring of 'slots' packets that the
 * agents' packets are all-gathered into (rank-major: the order MapFusion processes them in); each agent answers
 * its own keyframes' queries on its replica of the database.
 * ---------------------------------------------------------------------------------------------- */
typedef struct orbx_fusion orbx_fusion;
typedef struct orbx_exchange orbx_exchange;

/* Packet byte layout for 'capacity' keypoints: offsets of kps, desc, fv_nodes, fv_offsets, fv_indices, valid,
 * bow_words, bow_values (8 entries, after a 32-byte header: int32 count, agent, frame, n_fv, n_words) and the
 * packet size. */
int orbx_packet_layout(int capacity, size_t* offsets, size_t* bytes);

/* vocab / matcher stay owned by the caller (the matcher's nnratio / checkOri are MapFusion's 0.75 / true); the
 * fusion owns its KeyFrameDatabase over the ring.  max_keyframes: keyframes per agent per step; slots >=
 * world * max_keyframes; candidates: SearchByBoW pairs per query (first k other-map candidates). */
int orbx_fusion_create(orbx_vocab* vocab, orbx_matcher* matcher, int capacity, int slots, int max_keyframes, int candidates,
                       int levelsup, int min_matches, int agent, int world, int device, orbx_fusion** out);
int orbx_fusion_destroy(orbx_fusion* f);
/* Packet size, ring slots, ring base pointer and the ring as an orbx_kf_store (any may be NULL). */
int orbx_fusion_info(const orbx_fusion* f, size_t* packet_bytes, int* slots, void** d_ring, orbx_kf_store* store);
/* Phase 1: this agent's n new keyframes are rows first_row + j*row_step of an orbx_extract_batch_device output
 * (d_kps / d_desc at row*capacity, d_counts[row]); MapPoint-valid = d_valid[row*capacity+i] != 0, else
 * d_depth[row*capacity+i] > 0 (stereo keypoints get MapPoints, Tracking::CreateNewKeyFrame), else all; frame id of
 * keyframe j = frame_base + j*frame_step.  BoW + packets.  With world == 1 the packets go straight into the ring;
 * otherwise into d_send_out (n packets; NULL = an internal buffer), returned in *d_send, which the caller
 * all-gathers (world*n packets, rank-major) into *d_exchange_dst -- this exchange's ring slots -- or elsewhere and
 * hands to phase 2 as d_exchanged. */
int orbx_fusion_pack_device(orbx_fusion* f, const orbx_keypoint* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                            const float* d_depth, const uint8_t* d_valid, int capacity, int first_row, int row_step, int n,
                            long long frame_base, int frame_step, void* d_send_out, void** d_exchange_dst, void** d_send,
                            void* stream);
/* Phase 2: (d_exchanged: the gathered packets when they were not gathered into the ring, else NULL) ring slots leave
 * and rejoin the database in processing order, the sequential DetectLoopCandidates of this agent's keyframes, the
 * first k other-map candidates as SearchByBoW pairs ((query, -1) padded), the batched SearchByBoW.  Outputs, each
 * optional (NULL = not returned): d_pairs [n*k][2] slot pairs, d_match12 [n*k][capacity] (KF2 index or -1),
 * d_nmatches [n*k]. */
int orbx_fusion_commit_device(orbx_fusion* f, const void* d_exchanged, int32_t* d_pairs, int32_t* d_match12,
                              int32_t* d_nmatches, void* stream);
/* Both phases with the all-gather over a native exchange in between (x = NULL for a single agent). */
int orbx_fusion_step_device(orbx_fusion* f, orbx_exchange* x, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                            const int32_t* d_counts, const float* d_depth, const uint8_t* d_valid, int capacity, int first_row,
                            int row_step, int n, long long frame_base, int frame_step, int32_t* d_pairs, int32_t* d_match12,
                            int32_t* d_nmatches, void* stream);
/* Host copy of the whole ring (slots x packet bytes; synchronises). */
int orbx_fusion_read_ring(orbx_fusion* f, uint8_t* host_dst);
/* Ring slots of the last commit: the new slots [first_slot, first_slot + n_new) and this agent's queries. */
int orbx_fusion_last_step(const orbx_fusion* f, int* first_slot, int* n_new, int* query_first, int* n_queries);
/* Synchronises the device; candidates that passed the 20-match gate so far, and the database status word (bit 1:
 * queries interacted, bit 2: candidate capacity exceeded -- either means the results are not the reference's). */
int orbx_fusion_stats(orbx_fusion* f, long long* gate_passed, int* status);

/* RCCL communicator for the keyframe all-gather (librccl opened at run time; ncclUniqueId is 128 bytes: rank 0
 * creates it and the caller distributes it to every rank, e.g. over the process launcher). */
int orbx_exchange_unique_id(void* id128);
int orbx_exchange_create(const void* id128, int world, int rank, int device, orbx_exchange** out);
int orbx_exchange_destroy(orbx_exchange* x);
/* ncclAllGather of 'bytes' per rank: d_recv receives world * bytes, rank-major. */
int orbx_exchange_allgather_device(orbx_exchange* x, const void* d_send, size_t bytes, void* d_recv, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ORBX_H */
