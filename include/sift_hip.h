/*
 * sift_hip.h -- C ABI of libsift_hip.so, the MI355X (gfx950) SIFT detect+compute
 * library.  Plain C types only: no OpenCV, no C++ and no torch types cross
 * this boundary, so any FFI (ctypes, cgo, JNI, N-API) can bind it.
 *
 * Each entry point names the reference interface it replaces
 * (canhld94/SIFT-GPU include/sift.hpp, src/sift.cpp).  The C++ drop-in that
 * restores the reference's own signatures on top of this ABI is
 * include/sift.hpp (implemented in sift-gpu_amd/cpp/sift_shim.cpp).
 *
 * Conventions
 *  - Every function returns SIFT_OK (0) or a negative SIFT_E_* code; the
 *    message is available from sift_last_error(ctx).  Nothing calls exit().
 *  - A context owns device workspace sized at creation for images up to
 *    max_rows x max_cols and batches up to max_batch, plus one HIP stream.
 *    A context is not thread-safe: use one per host thread.
 *  - "host" entry points take and return host memory and synchronise; the
 *    "_device" / "_batch" entry points take device pointers, enqueue on the
 *    context stream and return immediately (call sift_sync to wait).
 *  - Results equal the reference CPU path bit for bit in the default (exact)
 *    mode.  SIFT_FLAG_FAST selects the separable LDS-tiled pyramid, which is
 *    not bit-exact.
 */
#ifndef SIFT_HIP_H_
#define SIFT_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIFT_OK 0
#define SIFT_E_INVALID (-1)   /* bad argument */
#define SIFT_E_HIP (-2)       /* HIP runtime error */
#define SIFT_E_CAPACITY (-3)  /* output capacity too small; required count reported */
#define SIFT_E_SIZE (-4)      /* image/batch larger than the context was created for */
#define SIFT_E_NOMEM (-5)     /* device allocation failed */
#define SIFT_E_WORKSPACE (-6) /* the context's internal candidate workspace overflowed
                                 (an input far more textured than the context was sized
                                 for): no result is held, *n_out = -1; create the context
                                 with a larger max size.  Not the two-call sizing case. */

#define SIFT_FLAG_FAST 0x1u     /* separable fused pyramid (not bit-exact) */
#define SIFT_FLAG_PROFILE 0x2u  /* per-stage HIP-event timing, see sift_get_stage_stats */
#define SIFT_FLAG_VERBOSE 0x4u  /* print the reference's phase timings (src/sift.cpp:70,80,88) */
#define SIFT_FLAG_NO_GRAPH 0x8u /* launch every kernel directly instead of replaying the context's
                                   cached hipGraph of the compute sequence (graphs are also off
                                   under SIFT_FLAG_PROFILE / SIFT_FLAG_VERBOSE) */

#define SIFT_DESC_LEN 128
#define SIFT_N_SCALES 5         /* Gaussian planes per octave */
#define SIFT_N_DOG 4            /* DoG planes per octave */

/* Layout-identical to cv::KeyPoint {Point2f pt; float size, angle, response;
 * int octave, class_id;} = 28 bytes.  octave packs o | layer<<8 | xi<<16
 * exactly as src/sift.cpp:383 does. */
typedef struct sift_keypoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} sift_keypoint;

typedef struct sift_ctx sift_ctx;

typedef struct sift_stage_stat {
  char name[32];
  int launches;
  double ms;     /* summed device time over launches (HIP events) */
  double flops;  /* algorithmic flops summed over launches */
  double bytes;  /* algorithmic HBM bytes summed over launches */
} sift_stage_stat;

/* ---- context ------------------------------------------------------------ */
int sift_ctx_create(int device, int max_rows, int max_cols, int max_batch, unsigned flags,
                    sift_ctx** out);
int sift_ctx_destroy(sift_ctx* ctx);
const char* sift_last_error(const sift_ctx* ctx);
/* Use an external HIP stream (hipStream_t) instead of the context's own. */
int sift_set_stream(sift_ctx* ctx, void* hip_stream);
void* sift_get_stream(sift_ctx* ctx);
int sift_set_flags(sift_ctx* ctx, unsigned flags);
/* Number of octaves (default 5, the literal at src/sift.cpp:67,68,78). */
int sift_set_octaves(sift_ctx* ctx, int n_octaves);
/* Waits for the context stream, then reports the sticky device status of the
 * calls since the last report: SIFT_E_WORKSPACE (candidate workspace
 * overflow), SIFT_E_CAPACITY (a batch call's keypoint total exceeded its
 * kp_cap), SIFT_E_INVALID (calDescriptor's CV_Assert, src/sift.cpp:744). */
int sift_sync(sift_ctx* ctx);
/* Candidate (26-neighbour extremum) slots per image of the batch; the default
 * is max(16384, max_rows * max_cols / 32), about 5x the extrema of a textured
 * 1080p image.  Reallocates the workspace (synchronises). */
int sift_set_candidate_capacity(sift_ctx* ctx, int per_image);
const char* sift_version(void);
/* hipGraph cache counters of this context: sequences captured, cached
 * executables patched in place (hipGraphExecUpdate: same shape, other
 * buffers) and executables instantiated.  The cache holds 4 shapes; a call
 * whose shape (batch, dims, strides, kp_cap, octaves, flags) and buffers both
 * match a cached entry replays it with no capture at all, so callers that can
 * keep their device buffers stable (or rotate among a few) pay no capture. */
int sift_graph_stats(const sift_ctx* ctx, long long* captures, long long* updates, long long* instantiations);

/* ---- layout helpers ----------------------------------------------------- */
/* Octave shapes: octave o+1 = Size(cols/2, rows/2) of octave o (src/sift.cpp:254). */
int sift_octave_shapes(int rows, int cols, int n_octaves, int* orows, int* ocols);
/* Elements of a packed pyramid (planes back to back, no padding): per = 5
 * (Gaussian, index o*5+s) or 4 (DoG, index o*4+s). */
size_t sift_packed_size(int rows, int cols, int n_octaves, int per);

/* ---- full detect + compute ---------------------------------------------- */
/* Replaces SIFT_NCL (include/sift.hpp:41, src/sift.cpp:59-91).
 * img: host, rows x cols CV_32FC1 values, row_stride_bytes apart.
 * kpts/desc: host, capacity cap keypoints / cap x 128 floats.  *n_out gets the
 * keypoint count; if it exceeds cap, nothing is copied and SIFT_E_CAPACITY is
 * returned (call again with cap >= *n_out). */
int sift_detect_compute(sift_ctx* ctx, const float* img, int rows, int cols,
                        size_t row_stride_bytes, sift_keypoint* kpts, float* desc, int cap,
                        int* n_out);

/* Copies the keypoints/descriptors of the last host-API call that produced
 * them (sift_detect_compute or sift_find_scale_space_extrema) without
 * recomputing: the second half of the two-call sizing pattern.  desc may be
 * NULL (extrema only).  SIFT_E_CAPACITY if cap < count (*n_out = count). */
int sift_copy_results(sift_ctx* ctx, sift_keypoint* kpts, float* desc, int cap, int* n_out);

/* Batch mode on device-resident images.  d_imgs: batch images
 * of rows x cols, row_stride elements between rows and img_stride elements
 * between images.  Outputs (device, caller-owned): keypoints of image b occupy
 * [d_img_offsets[b], d_img_offsets[b+1]) of d_kpts/d_desc (rows of 128).  Only
 * the first kp_cap keypoints are written; d_img_offsets[batch] holds the true
 * total, so a caller detects overflow after sift_sync.  Asynchronous. */
int sift_detect_compute_batch(sift_ctx* ctx, const float* d_imgs, int batch, int rows, int cols,
                              size_t row_stride, size_t img_stride, sift_keypoint* d_kpts,
                              float* d_desc, int kp_cap, int* d_img_offsets);

/* Synthetic integer-exact test images, written on device:
 * image b uses seed 0x5EED0000 + seed_base + b.  Asynchronous. */
int sift_synth_images(sift_ctx* ctx, float* d_out, int batch, int rows, int cols,
                      size_t row_stride, size_t img_stride, int seed_base);

/* ---- multi-GPU batch mode (BASELINE configs[3]) ----------
 * The reference's only parallelism is OpenMP over descriptors
 * (src/sift.cpp:738); here the images of a batch are sharded over the GPUs of
 * one node by contiguous ranges, each device runs sift_detect_compute_batch on
 * its shard, and the keypoint records are gathered to the first device over
 * RCCL (ncclSend / ncclRecv, xGMI) one step behind the compute.  One process
 * drives every device (ncclCommInitAll); a multi context is not thread-safe. */
typedef struct sift_multi sift_multi;
#define SIFT_MULTI_SELF_P2P 0x100u /* sift_multi_create flag: device 0's own records also go through RCCL
                                      (self send/recv) instead of a DMA copy -- tests the p2p path on one GPU */
/* Shard arithmetic: device `index` of n takes the contiguous images
 * [*first, *first + *count) = [floor(index * batch / n), floor((index + 1) * batch / n)).
 * No GPU needed. */
int sift_multi_shard(int batch, int n_devices, int index, int* first, int* count);
/* Global per-image offsets [sum(counts) + 1] from each shard's own offsets
 * [counts[i] + 1] (records concatenated in device order).  No GPU needed. */
int sift_multi_merge_offsets(const int* const* shard_offsets, const int* counts, int n_devices,
                             int* global_offsets);
/* Per device: streams_per_device sift_ctx contexts, each with its own HIP
 * stream (0 = the default, 2: each step's shard runs as that many contiguous
 * sub-batches whose stages overlap, as bench.py's streams do), two result
 * slots per context sharing kp_cap_per_device records per slot, and a
 * gather stream; on devices[0] the gather buffers (n_devices x
 * kp_cap_per_device records, and descriptors when gather_desc); RCCL
 * communicators over the devices.  Device indices must be distinct (RCCL:
 * one rank per device). */
int sift_multi_create(const int* devices, int n_devices, int max_rows, int max_cols, int max_batch_per_device,
                      unsigned flags, int streams_per_device, int kp_cap_per_device, int gather_desc,
                      sift_multi** out);
int sift_multi_destroy(sift_multi* m);
const char* sift_multi_last_error(const sift_multi* m);
/* The first context of device index i (sift_synth_images on that device, ...). */
sift_ctx* sift_multi_context(sift_multi* m, int index);
/* sift_set_octaves / sift_set_flags on every context. */
int sift_multi_set_octaves(sift_multi* m, int n_octaves);
int sift_multi_set_flags(sift_multi* m, unsigned flags);
/* One step: device i detects + describes counts[i] images resident on it
 * (d_imgs[i], strides in elements as in sift_detect_compute_batch) into its
 * result slots, and the previous step's records are gathered to devices[0].
 * The images must be complete when the step is enqueued (the contexts'
 * streams do not wait for the caller's producers: synchronise them first).
 * Asynchronous, except that the host waits for the previous step's per-image
 * offsets (one step behind, so normally without blocking). */
int sift_multi_step(sift_multi* m, const float* const* d_imgs, const int* counts, int rows, int cols,
                    size_t row_stride, size_t img_stride);
/* Gathers the last step, drains every stream and reports the contexts' sticky
 * status (as sift_sync).  A step or flush that fails after enqueueing work
 * (a device error, a keypoint count above a context's share of
 * kp_cap_per_device) leaves the result slots undefined: later steps and
 * flushes return SIFT_E_INVALID and the multi context must be destroyed. */
int sift_multi_flush(sift_multi* m);
/* The last gathered step on devices[0]: device pointers to its records (and
 * descriptors, or NULL without gather_desc) in global image order, and the
 * global per-image offsets [batch_total + 1] into host memory (offsets may be
 * NULL).  Valid until the next sift_multi_step. */
int sift_multi_gathered(sift_multi* m, const sift_keypoint** d_kpts, const float** d_desc, int* offsets,
                        int offsets_cap, int* batch_total, long long* step);
/* Host copy of the last gathered step's records (and descriptors, desc may be
 * NULL): *n_out gets the record count; SIFT_E_CAPACITY if cap < count.
 * Synchronous. */
int sift_multi_copy_gathered(sift_multi* m, sift_keypoint* kpts, float* desc, int cap, int* n_out);
/* Steps enqueued, records gathered and RCCL p2p transfers posted so far
 * (device 0's own pieces are DMA copies unless SIFT_MULTI_SELF_P2P). */
int sift_multi_stats(const sift_multi* m, long long* steps, long long* records, long long* transfers);
/* RCCL's NCCL_VERSION_CODE at run time (ncclGetVersion), -1 on error. */
int sift_multi_rccl_version(void);

/* ---- sub-module entry points (host memory, synchronous) ----------------- */
/* Gaussian_Blur (include/sift.hpp:47, src/sift.cpp:123-153). */
int sift_gaussian_blur(sift_ctx* ctx, const float* src, int rows, int cols, double sigma,
                       float* dst);
/* Gaussian_Blur_1D (include/sift.hpp:49, src/sift.cpp:170-217). */
int sift_gaussian_blur_1d(sift_ctx* ctx, const float* src, int rows, int cols, double sigma,
                          float* dst);
/* buildGaussianPyramid (include/sift.hpp:51, src/sift.cpp:229-263); gpyr is
 * packed, sift_packed_size(rows, cols, n_octaves, 5) floats. */
int sift_build_gaussian_pyramid(sift_ctx* ctx, const float* img, int rows, int cols,
                                int n_octaves, float* gpyr);
/* buildDoGPyramid (include/sift.hpp:55, src/sift.cpp:265-283); packed in/out. */
int sift_build_dog_pyramid(sift_ctx* ctx, const float* gpyr, int rows, int cols, int n_octaves,
                           float* dog);
/* findScaleSpaceExtrema (include/sift.hpp:59, src/sift.cpp:547-577); packed
 * pyramids in; keypoints out with the same count/capacity rule as above. */
int sift_find_scale_space_extrema(sift_ctx* ctx, const float* gpyr, const float* dog, int rows,
                                  int cols, int n_octaves, sift_keypoint* kpts, int cap,
                                  int* n_out);
/* calDescriptor (include/sift.hpp:64, src/sift.cpp:733-753). */
int sift_calc_descriptors(sift_ctx* ctx, const float* gpyr, int rows, int cols, int n_octaves,
                          const sift_keypoint* kpts, int n, float* desc, int first_octave);

/* ---- image front end ----------------------------------- */
/* Replaces the conversion half of the application's readImage
 * (src/main.cpp:79-87): decoded 8-bit BGR bytes (imread's layout) ->
 * optional INTER_LINEAR resize to out_rows x out_cols (the scene's
 * Size(960, 960); no resize when the sizes are equal) -> cvtColor
 * COLOR_RGB2GRAY on those BGR bytes -> CV_32F.  Decoding stays with the
 * caller.  Host buffers (synchronous), gray is out_rows x out_cols floats: */
int sift_bgr8_to_gray(sift_ctx* ctx, const uint8_t* bgr, int rows, int cols, size_t row_stride, int out_rows,
                      int out_cols, float* gray);
/* Device buffers, a batch of images, enqueued on the context stream (the
 * output can be the input of sift_detect_compute_batch). Strides in bytes. */
int sift_bgr8_to_gray_device(sift_ctx* ctx, const uint8_t* d_bgr, int batch, int rows, int cols,
                             size_t row_stride, size_t img_stride, int out_rows, int out_cols, float* d_gray,
                             size_t out_row_stride, size_t out_img_stride);

/* ---- matching ------------------------------------------ */
/* Replaces `BFMatcher(NORM_L1).knnMatch(query, train, matches, k)` of the
 * reference application (src/main.cpp:25-27; the 0.86 ratio test at :28-40
 * stays with the caller).  query [n_query][128], train [n_train][128] floats;
 * for each query the k (1 or 2) nearest train rows by float L1 distance
 * (OpenCV normL1_ summation order, see match.hip), ascending, an earlier train
 * index first at equal distance.  idx / dist are [n_query][k]; when
 * n_train < k the missing entries are idx -1, dist +inf.
 * Host buffers (synchronous): */
int sift_knn_match_l1(sift_ctx* ctx, const float* query, int n_query, const float* train, int n_train, int k,
                      int* idx, float* dist);
/* Device buffers (16-byte aligned rows), enqueued on the context's stream: */
int sift_knn_match_l1_device(sift_ctx* ctx, const float* d_query, int n_query, const float* d_train,
                             int n_train, int k, int* d_idx, float* d_dist);

/* ---- homography ---------------------------------------- */
/* Replaces `findHomography(obj, scene, RANSAC)` and `perspectiveTransform`
 * (src/main.cpp:54-62): n point pairs as interleaved (x, y) floats, OpenCV's
 * defaults are ransac_thresh 3, max_iters 2000, confidence 0.995.  H is a
 * row-major 3x3 with H[8] = 1; inlier_mask (n bytes, may be NULL) gets the
 * RANSAC inliers.  Host code, no context.  SIFT_E_INVALID (H zeroed) when no
 * model is found or n < 4 -- OpenCV's empty Mat.
 * Not bit-compatible with OpenCV: the final refinement is 10 steps of a plain
 * Levenberg-Marquardt on H[0..7] (normal equations, Gaussian elimination), not
 * OpenCV's LMSolver, so H can differ from cv::findHomography's in the last
 * digits (the RANSAC sampling and inlier mask follow OpenCV's order).  Parity
 * is pinned only against oracle/homography.py, which restates the same steps. */
int sift_find_homography(const float* src_xy, const float* dst_xy, int n, double ransac_thresh, int max_iters,
                         double confidence, double* H, unsigned char* inlier_mask);
int sift_perspective_transform(const double* H, const float* xy, int n, float* out_xy);

/* ---- self-test ------------------------------------------------------------ */
/* Evaluates one device arithmetic helper element-wise on host arrays (n
 * values), for bit-exact checks of the GPU math against the CPU oracle:
 * op 0 exp32f(a), 1 fastAtan2(a, b) (y = a, x = b, degrees), 2 magnitude(a, b),
 * 3 (float)cos((double)a), 4 (float)sin((double)a), 5 (float)exp2((double)a),
 * 6 cvRound(a) (as float), 7 cvFloor(a) (as float). */
int sift_selftest_math(sift_ctx* ctx, int op, const float* a, const float* b, float* out, int n);

/* ---- profiling ------------------------------------------------------------ */
/* With SIFT_FLAG_PROFILE: per-stage device time accumulated since the last
 * reset (synchronises).  Writes up to cap entries, *n gets the count. */
int sift_get_stage_stats(sift_ctx* ctx, sift_stage_stat* out, int cap, int* n, int reset);

#ifdef __cplusplus
}
#endif
#endif /* SIFT_HIP_H_ */
