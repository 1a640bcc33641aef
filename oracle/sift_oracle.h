/*
 * sift_oracle.h -- CPU restatement of the reference SIFT hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped library links, loads or
 * calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker / CPU baseline.
 *
 * What it restates: canhld94/SIFT-GPU src/sift.cpp (the whole SIFT_NCL path,
 * file:line cited per function in sift_oracle.c) plus the OpenCV-4.0
 * internals that file calls (cvRound, cvFloor, saturate_cast<uchar>,
 * hal::exp32f, hal::fastAtan2, hal::magnitude32f, Matx33f::solve(DECOMP_LU),
 * resize(INTER_NEAREST)) as documented in SURVEY.md Appendix A.
 *
 * PARITY UNPINNED: the reference cannot be compiled in this image (it needs
 * OpenCV 4.0 + opencv_contrib, which are absent, and stand-in headers are not
 * allowed), and it ships no tests, golden vectors or known-answer fixtures.
 * The restatement is therefore checked only against independent math
 * (numpy double-precision re-derivations of each helper) and the fixtures in
 * tests/golden/ are regression vectors produced by this oracle.
 *
 * Arithmetic contract: compiled with -O2 -ffp-contract=off, no -march, no
 * -ffast-math -- the reference's own makefile:25 flags (-O3, no -march) give
 * IEEE single precision with separate multiply and add on x86-64 (SSE2).
 */
#ifndef SIFT_ORACLE_H_
#define SIFT_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Layout-identical to cv::KeyPoint (5 floats + 2 int32 = 28 bytes). */
typedef struct so_keypoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} so_keypoint;

#define SO_N_SCALES 5  /* nOctaveLayers + 3, src/sift.cpp:5 */
#define SO_N_DOG 4     /* nScales - 1 */

/* Octave shapes: octave o+1 is Size(cols/2, rows/2) of octave o
 * (src/sift.cpp:254).  Fills rows[o], cols[o] for o < n_octaves. */
void so_octave_shapes(int rows, int cols, int n_octaves, int* orows, int* ocols);

/* Packed pyramid layout: plane (o, s) starts at element off[o*per+s] where
 * per = 5 for the Gaussian pyramid and 4 for DoG.  Returns total elements. */
size_t so_pyramid_offsets(int rows, int cols, int n_octaves, int per, size_t* off);

/* 2-D Gaussian coefficients x8192 (src/sift.cpp:95-108).  coeff must hold
 * ksize*ksize floats (ksize <= 2*floor(3*sigma)+1).  Returns ksize. */
int so_gaussian_kernel(float sigma, float* coeff);

/* Gaussian_Blur (src/sift.cpp:123-153). */
void so_gaussian_blur(const float* src, int rows, int cols, double sigma, float* dst);

/* Gaussian_Blur_1D (src/sift.cpp:157-217), taps k in [-w, w-1]. */
void so_gaussian_blur_1d(const float* src, int rows, int cols, double sigma, float* dst);

/* resize(..., INTER_NEAREST) to (drows, dcols) (src/sift.cpp:254). */
void so_resize_nn(const float* src, int srows, int scols, float* dst, int drows, int dcols);

/* buildGaussianPyramid (src/sift.cpp:229-263), packed output (5 planes per
 * octave, correct o*5+s indexing -- identical to the reference at 5). */
void so_build_gaussian_pyramid(const float* img, int rows, int cols, int n_octaves, float* gpyr);

/* The library's SIFT_FLAG_FAST separable pyramid (agreement mode, not the
 * reference's arithmetic), in its exact operation order; packed like
 * so_build_gaussian_pyramid. */
void so_fast_pyramid(const float* img, int rows, int cols, int n_octaves, float* gpyr);

/* buildDoGPyramid (src/sift.cpp:265-283), packed output (4 planes/octave). */
void so_build_dog_pyramid(const float* gpyr, int rows, int cols, int n_octaves, float* dog);

/* findScaleSpaceExtrema (src/sift.cpp:547-577).  Writes up to cap keypoints
 * and returns the total count found (may exceed cap). */
int so_find_scale_space_extrema(const float* gpyr, const float* dog, int rows, int cols,
                                int n_octaves, so_keypoint* kps, int cap);

/* calDescriptor (src/sift.cpp:733-753): n rows of 128 floats. */
void so_calc_descriptors(const float* gpyr, int rows, int cols, int n_octaves,
                         const so_keypoint* kps, int n, float* desc, int first_octave);

/* SIFT_NCL (src/sift.cpp:59-91).  *kps / *desc are malloc'd; caller frees
 * with so_free.  Returns the keypoint count. */
int so_sift(const float* img, int rows, int cols, int n_octaves, so_keypoint** kps, float** desc);
void so_free(void* p);

/* Number of OpenMP threads for the descriptor loop (src/sift.cpp:738). */
void so_set_threads(int n);

/* Synthetic integer-exact test image, SURVEY.md 8(d) row d2. */
void so_synth_image(int b, int rows, int cols, float* out);

/* OpenCV-internal helpers, exported for unit tests. */
void so_exp32f(const float* x, float* y, int n);
void so_fast_atan2(const float* y, const float* x, float* out, int n);
void so_magnitude32f(const float* x, const float* y, float* out, int n);
int so_solve3(const float* a9, const float* b3, float* x3); /* 1 ok, 0 singular (x=0) */
int so_cv_round(float v);
/* Element-wise helper evaluation with the same op codes as the library's
 * sift_selftest_math: 0 exp32f, 1 fastAtan2(a,b), 2 magnitude(a,b),
 * 3 (float)cos((double)a), 4 (float)sin((double)a), 5 (float)exp2((double)a),
 * 6 cvRound(a), 7 cvFloor(a). */
void so_helper(int op, const float* a, const float* b, float* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* SIFT_ORACLE_H_ */
