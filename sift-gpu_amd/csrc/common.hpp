// common.hpp -- shared host/device definitions for the gfx950 SIFT library.
//
// Everything here that computes is an exact restatement of the reference
// arithmetic (canhld94/SIFT-GPU src/sift.cpp) and of the OpenCV-4.0 helpers it
// calls, so that device results equal the CPU path bit for bit.  The whole
// library is compiled with -ffp-contract=off: every a*b+c below is a separate
// multiply and add, like the reference's x86-64 build (makefile:25, no -march).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/sift_hip.h"
#include "gauss_host.hpp"

namespace sift {

// ---- tuning constants, src/sift.cpp:4-47 ---------------------------------
constexpr int kScales = 5;          // nScales = nOctaveLayers + 3
constexpr int kDogPer = 4;          // DoG planes per octave
constexpr int kBorder = 5;          // SIFT_IMG_BORDER
constexpr int kMaxInterp = 5;       // SIFT_MAX_INTERP_STEPS
constexpr int kOriBins = 36;        // SIFT_ORI_HIST_BINS
constexpr int kMaxPeaks = 18;       // strict local maxima of a 36-bin circle
constexpr int kDescW = 4;           // SIFT_DESCR_WIDTH
constexpr int kDescBins = 8;        // SIFT_DESCR_HIST_BINS
constexpr int kDescLen = 128;
constexpr int kMaxOctaves = 12;
constexpr float kDogThreshold = 8.f;  // literal at src/sift.cpp:564
constexpr double kCvPi = 3.1415926535897932384626433832795;

// ---- pyramid layout in HBM ------------------------------------------------
// Per image: octave-major, 5 Gaussian planes then (separately) 4 DoG planes,
// each plane rows x pitch floats, pitch = cols rounded up to 32 floats (128 B,
// one L2 line), so every plane row, plane and image block starts on a line
// boundary: a 64-column strip's row is two whole lines, never a partial-line
// write.  (With 64-B pitches the 1080p image block was 55,251,520 B, an odd
// number of half lines, so every odd image of a batch was misaligned.)
// Invariant: the pitch padding columns [cols, pitch) of every plane hold
// unspecified values.  SIFT_FLAG_FAST's dwordx4 / dwordx2 plane stores
// (pyramid_pc.hip) write whole 4-column groups past cols there, and no kernel
// reads a column >= cols of a Gaussian or DoG plane (every reader bounds its
// columns by cols, and the sub-module API copies planes out row by row with
// cols columns); tests/test_gpu_fast.py::test_pitch_padding_is_never_read
// poisons the padding with NaN and requires unchanged results.
constexpr int kPitchAlign = 32;
struct Octave {
  int rows, cols, pitch;
  int pad_;
  long long g_off[kScales];   // element offset of Gaussian plane s in the image block
  long long d_off[kDogPer];   // element offset of DoG plane s in the image block
};

struct Layout {
  int n_oct;
  int rows, cols;
  int pad_;
  long long g_img;  // elements per image, Gaussian pyramid
  long long d_img;  // elements per image, DoG pyramid
  Octave oct[kMaxOctaves];
};

inline int round_up(int v, int m) { return (v + m - 1) / m * m; }

Layout make_layout(int rows, int cols, int n_oct);

// ---- candidate / keypoint work records -----------------------------------
struct Cand {            // one 26-neighbour extremum, in reference scan order
  int b, ol, r, c;       // image, octave | layer<<8, row, col
};

struct CandOut {         // result of refine + orientation for one candidate
  float x, y, size, response;
  int octave, npeaks, img, ref_r;  // npeaks: 1 if refinement kept it (the count is in DetectBufs::npeaks)
  float angle[kMaxPeaks];
  int ref_c, ref_layer;            // refined integer position / layer (orientation input)
};

// ---- OpenCV scalar helpers --------------------------
__device__ __forceinline__ int cv_round(float v) { return __float2int_rn(v); }
__device__ __forceinline__ int cv_round_d(double v) { return __double2int_rn(v); }
__device__ __forceinline__ int cv_floor(float v) {
  int i = (int)v;
  return i - (i > v);
}
__device__ __forceinline__ float sat_u8(float v) {
  int iv = cv_round(v);
  return (float)(iv < 0 ? 0 : iv > 255 ? 255 : iv);
}

// libm calls on the path, evaluated as (float)f((double)x) on CPU and GPU
// alike (see oracle/sift_oracle.c for the measured glibc deviation).
__device__ __forceinline__ float pow2f_cr(float y) { return (float)exp2((double)y); }
__device__ __forceinline__ float cosf_cr(float x) { return (float)cos((double)x); }
__device__ __forceinline__ float sinf_cr(float x) { return (float)sin((double)x); }

// hal::exp32f, scalar form (EXPTAB_SCALE = 6); tab = 64 floats 2^(j/64)*A0.
struct ExpConsts {
  float A1, A2, A3, A4, lo, hi, post, prescale;
};

template <bool CLAMP = true>  // false: see exp32f_v
__device__ __forceinline__ float exp32f(float v, const float* __restrict__ tab,
                                        const ExpConsts& k) {
  if (CLAMP) {
    v = v < k.lo ? k.lo : v;
    v = k.hi < v ? k.hi : v;
    v = v * k.prescale;
    int vi = cv_round(v);
    v = (v - (float)vi) * k.post;
    int t = (vi >> 6) + 127;
    t = !(t & ~255) ? t : t < 0 ? 0 : 255;
    float sc = __int_as_float(t << 23);
    float poly = (((v + k.A1) * v + k.A2) * v + k.A3) * v + k.A4;
    return sc * tab[vi & 63] * poly;
  } else {
    // see exp32f_v: same bits inside the argument range the callers state
    v = v * k.prescale;
    const float r = rintf(v);  // cv_round's value, kept as a float
    const int vi = (int)r;
    v = (v - r) * k.post;
    float poly = (((v + k.A1) * v + k.A2) * v + k.A3) * v + k.A4;
    return __builtin_amdgcn_ldexpf(tab[vi & 63], vi >> 6) * poly;
  }
}

// The same with the table held one entry per lane (lane j: tab[j]) and read
// with a cross-lane permute instead of an LDS gather; every lane of the wave
// must execute it.
// CLAMP = false is for callers whose argument lies in (-87, 0] (the
// descriptor's -(c^2 + r^2) / 8 over a window: > -1.6; the orientation's:
// > -36): exp32f's input clamp to [lo, hi] never acts there, and the exponent
// t = (vi >> 6) + 127 stays in [1, 127], so its clamp to [0, 255] does not
// act either and 2^(vi >> 6) * tab[...] is an exact power-of-two scaling of a
// normal float -- one v_ldexp_f32 gives the same bits as building the scale
// and multiplying.  (float)cv_round(v) is rintf(v) for |v| < 2^24, so the
// rounded value is kept as a float.  Outside that range the result is
// finite garbage (callers mask it).  The lane permute uses address bits [7:2]
// only, so vi << 2 indexes lane vi & 63.
template <bool CLAMP = true>
__device__ __forceinline__ float exp32f_v(float v, float tab_lane, const ExpConsts& k) {
  if (CLAMP) {
    v = v < k.lo ? k.lo : v;
    v = k.hi < v ? k.hi : v;
    v = v * k.prescale;
    int vi = cv_round(v);
    v = (v - (float)vi) * k.post;
    int t = (vi >> 6) + 127;
    t = !(t & ~255) ? t : t < 0 ? 0 : 255;
    float sc = __int_as_float(t << 23);
    float poly = (((v + k.A1) * v + k.A2) * v + k.A3) * v + k.A4;
    const float tv = __int_as_float(__builtin_amdgcn_ds_bpermute((vi & 63) << 2, __float_as_int(tab_lane)));
    return sc * tv * poly;
  } else {
    v = v * k.prescale;
    const float r = rintf(v);
    const int vi = (int)r;
    v = (v - r) * k.post;
    float poly = (((v + k.A1) * v + k.A2) * v + k.A3) * v + k.A4;
    const float tv = __int_as_float(__builtin_amdgcn_ds_bpermute(vi << 2, __float_as_int(tab_lane)));
    return __builtin_amdgcn_ldexpf(tv, vi >> 6) * poly;
  }
}

// hal::fastAtan2 in degrees.
struct AtanConsts {
  float p1, p3, p5, p7, eps;
};

__device__ __forceinline__ float fast_atan2(float y, float x, const AtanConsts& k) {
  float ax = fabsf(x), ay = fabsf(y);
  float mn = ax < ay ? ax : ay, mx = ax < ay ? ay : ax;
  float c = mn / (mx + k.eps);
  float c2 = c * c;
  float a = (((k.p7 * c2 + k.p5) * c2 + k.p3) * c2 + k.p1) * c;
  if (!(ax >= ay)) a = 90.f - a;
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

__device__ __forceinline__ float magnitude(float x, float y) { return sqrtf(x * x + y * y); }

// Matx33f::solve(b, DECOMP_LU): Cramer's rule with float determinant; a
// singular matrix yields 0 (OpenCV returns Matx::zeros()).
__device__ __forceinline__ void solve3(const float a[9], const float b[3], float x[3]) {
#define A_(i, j) a[(i)*3 + (j)]
  float d = (float)(A_(0, 0) * (A_(1, 1) * A_(2, 2) - A_(2, 1) * A_(1, 2)) -
                    A_(0, 1) * (A_(1, 0) * A_(2, 2) - A_(2, 0) * A_(1, 2)) +
                    A_(0, 2) * (A_(1, 0) * A_(2, 1) - A_(2, 0) * A_(1, 1)));
  if (d == 0) {
    x[0] = x[1] = x[2] = 0;
    return;
  }
  d = 1 / d;
  x[0] = d * (b[0] * (A_(1, 1) * A_(2, 2) - A_(1, 2) * A_(2, 1)) -
              A_(0, 1) * (b[1] * A_(2, 2) - A_(1, 2) * b[2]) +
              A_(0, 2) * (b[1] * A_(2, 1) - A_(1, 1) * b[2]));
  x[1] = d * (A_(0, 0) * (b[1] * A_(2, 2) - A_(1, 2) * b[2]) -
              b[0] * (A_(1, 0) * A_(2, 2) - A_(1, 2) * A_(2, 0)) +
              A_(0, 2) * (A_(1, 0) * b[2] - b[1] * A_(2, 0)));
  x[2] = d * (A_(0, 0) * (A_(1, 1) * b[2] - b[1] * A_(2, 1)) -
              A_(0, 1) * (A_(1, 0) * b[2] - b[1] * A_(2, 0)) +
              b[0] * (A_(1, 0) * A_(2, 1) - A_(1, 1) * A_(2, 0)));
#undef A_
}

// Host-computed constant block shared by every kernel that needs it.
struct MathConsts {
  ExpConsts e;
  AtanConsts t;
  float exptab[64];
};

void host_math_consts(MathConsts* mc);

// ---- persistent-grid sizing ------------------------------------------------
// The work-loop kernels (refinement, orientation, descriptors) split their
// items evenly over the grid.  A grid larger than what the device holds at
// once runs in rounds, and the last, partial round idles the rest of the chip
// (8192 orientation waves on 6144 wave slots = 2 rounds for 1.33 rounds of
// work).  So the grid is the resident count: occupancy API x CUs, a multiple
// of 8 (the kernels' XCD split), cached per kernel; fixed_grid is the
// fallback when the occupancy query fails.
int resident_grid(const void* kernel, int block, size_t lds, int fixed_grid);

// ---- host launchers (defined in the .hip files) --------------------------
struct Plane {          // a device plane (or the input image)
  const float* p;
  long long pitch;      // elements per row
  long long img_stride; // elements per image of the batch
};

// blur.hip
void launch_blur_plane(hipStream_t st, int w, const float* coef, Plane src, float* dst,
                       long long dpitch, long long dimg, int rows, int cols, int batch);
// fuse_next: also write octave o+1's plane 0 (the INTER_NEAREST half of plane
// 2) when blur_fuses_decimation(L, o + 1); the caller then skips the decimation.
void launch_blur_octave(hipStream_t st, const Layout& L, int o, float* gpyr, const float* coefs,
                        const int* wsz, int batch, bool fuse_next = false);
bool blur_fuses_decimation(const Layout& L, int o);
// The same planes for small launches (2 outputs per lane, 32 x 16 tiles;
// round 3): picked when blur_octave_tiles(...) is below the context's limit.
void launch_blur_octave_small(hipStream_t st, const Layout& L, int o, float* gpyr, const float* coefs,
                              const int* wsz, int batch, bool fuse_next = false);
long long blur_octave_tiles(const Layout& L, int o, int batch);
// Exact blur in symmetric scatter form for SIFT_NCL's five fixed tables
// (compile-time constants); sym_tables_match(coefs) checks them against the
// context's base + octave tables before these are used.
bool sym_tables_match(const float* coefs);
void launch_blur_base_sym(hipStream_t st, Plane src, float* dst, long long dpitch, long long dimg, int rows,
                          int cols, int batch);
void launch_blur_octave_sym(hipStream_t st, const Layout& L, int o, float* gpyr, int batch, bool fuse_next);
void launch_decimate(hipStream_t st, const Layout& L, int o, float* gpyr, int batch);
void launch_dog(hipStream_t st, const Layout& L, int o, const float* gpyr, float* dog, int batch);
void launch_blur_1d(hipStream_t st, int w, const float* coef1d, Plane src, float* tmp, float* dst,
                    long long pitch, long long img, int rows, int cols, int batch);
void launch_synth(hipStream_t st, float* out, int batch, int rows, int cols, long long pitch,
                  long long img_stride, int seed_base);

void launch_bgr8_gray(hipStream_t st, const uint8_t* src, long long sstride, long long simg, int srows, int scols,
                      float* dst, long long dpitch, long long dimg, int drows, int dcols, int batch);
int find_homography_ransac(const float* src_xy, const float* dst_xy, int n, double thr, int max_iters,
                           double confidence, double* H, unsigned char* mask_out);
void perspective_transform(const double* H, const float* xy, int n, float* out);
int knn_splits(int nq, int nt);
void launch_knn_l1(hipStream_t st, const float* q, int nq, const float* t, int nt, int k, int splits,
                   float2* part_d, int2* part_i, int* idx, float* dist);
// pyramid_pc.hip (SIFT_FLAG_FAST): octave o's five planes by the separable
// form, plus octave o+1's plane 0 when pyramid_fuses_decimation(L, o + 1)
// (else decimate first), from a producer wave and three consumer waves
// synchronised by LDS counters; err = the context's sticky word err[3]
// (kErrStall).  fast_taps_match: the compiled-in 1-D taps equal
// fast_taps_host's for these sigmas; pyramid_fast_fits: every plane and the
// input rows below the kernel's dropped-offset range.
void launch_pyramid_pc(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch, int* err,
                       bool stall_test = false);  // stall_test: the pc_stall_once test hook
bool pyramid_fuses_decimation(const Layout& L, int o);
bool fast_taps_match(float sigma_base, const float* sig);
bool pyramid_fast_fits(const Layout& L, long long src_row_stride);
// Work items of one separable-pyramid launch: n_full strip columns walked
// whole, then the rest in `chunks` row chunks of `chunk` rows.
struct FastPlan {
  int n_full, chunk, chunks;
};
FastPlan fast_plan(int columns, int rows, int slots, int halo);

// One image small enough that the per-keypoint kernels are latency-bound (a
// 1080p image: ~13 K candidates, a few waves per SIMD) runs their one-image
// variants (orient_bin_kernel, the descriptor budgeted for 2 waves per SIMD);
// a batch, or one image above kOneImagePx (an 8K image: 214 K keypoints),
// fills the chip with the batch variants.  SIFT_HIP_ONE_IMAGE_PX overrides the
// limit (A/B runs).
constexpr long long kOneImagePx = 4ll << 20;
bool one_image_variants(const Layout& L, int batch);

// detect.hip
struct DetectBufs {
  unsigned* mask;       // candidate bitmask, mask_words_per_image * batch
  int* blk_counts;      // per scan block
  int* cand_total;      // [1]
  int* img_cand_off;    // [batch+1]
  Cand* cands;
  int cand_cap;
  CandOut* couts;
  int* kp_scan;         // per candidate exclusive scan of npeaks, [cand_cap+1]
  int* kp_total;        // [1]
  int* npeaks;          // orientation peaks per candidate, [cand_cap]
  int* scan_tmp;        // exclusive scan of blk_counts, [blk_cap+1]
  int* scan_tiles;      // per-tile sums of the multi-block scan, [scan_tiles_for(max(blk_cap, cand_cap))]
};
int scan_tiles_for(long long cap);
long long mask_words_per_image(const Layout& L);
int mask_blocks_per_image(const Layout& L);
void launch_extrema(hipStream_t st, const Layout& L, const float* gpyr, float* dog, bool write_dog,
                    float2* grad, const MathConsts* mc, int batch, DetectBufs& D);
void launch_grad(hipStream_t st, const Layout& L, const float* gpyr, float2* grad, int batch, int s_lo,
                 int s_hi, const MathConsts* mc);
void launch_refine_orient(hipStream_t st, const Layout& L, const float* gpyr, const float2* grad,
                          const float* dog, const MathConsts* mc, DetectBufs& D, int batch);
void launch_emit(hipStream_t st, DetectBufs& D, int batch, sift_keypoint* kpts, int kp_cap,
                 int* img_kp_off);
// Device status bits; bit i <-> sticky error word err[i] (DescArgs::err_flag = &err[0],
// status_kernel).
constexpr int kErrAssert = 1;      // keypoint octave/layer outside the pyramid (CV_Assert)
constexpr int kErrWorkspace = 2;   // candidate workspace overflow
constexpr int kErrKpCapacity = 4;  // keypoint total above the output capacity
constexpr int kErrStall = 8;       // a bounded in-kernel wait expired (pyramid_pc.hip); err[3]
void launch_status(hipStream_t st, const int* cand_total, int cand_cap, const int* img_off, int batch, int kp_cap,
                   int* err, int* stat);

// descriptor.hip
void launch_descriptors(hipStream_t st, const Layout& L, const float2* grad, const MathConsts* mc,
                        const sift_keypoint* kpts, const int* img_kp_off, int batch,
                        int kp_cap, float* desc, int first_octave, int* err_flag,
                        bool detected,  // detected: keypoints from this library's detection (radius <= 40)
                        int* perm);     // [kp_cap] scratch: the lane-balance ranking
void launch_math_selftest(hipStream_t st, int op, const float* a, const float* b, float* out, int n,
                          const MathConsts* mc);

}  // namespace sift
