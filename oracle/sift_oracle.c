/*
 * sift_oracle.c -- CPU restatement of the reference SIFT path (test oracle).
 *
 * TEST INFRASTRUCTURE ONLY -- see sift_oracle.h.  PARITY UNPINNED: the
 * reference (canhld94/SIFT-GPU src/sift.cpp) needs OpenCV 4.0, which is not in
 * this image, and it has no tests or golden vectors of its own.
 *
 * Every function cites the reference lines whose arithmetic it restates.
 * Evaluation order, int/float/double promotions and rounding helpers follow
 * the reference expression by expression; no FMA (build: -ffp-contract=off).
 */
#include "sift_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- tuning constants (src/sift.cpp:4-47) ------------------------------ */
enum { N_LAYERS = 2, N_SCALES = 5, IMG_BORDER = 5, MAX_INTERP = 5, ORI_BINS = 36,
       DESC_W = 4, DESC_BINS = 8 };
static const double K_SIGMA = 1.6;
static const double K_PI = 3.14159265359;           /* src/sift.cpp:7, not M_PI */
static const double K_CONTRAST = 0.04;
static const double K_EDGE = 10;
static const float ORI_SIG_FCTR = 1.5f;
static const float ORI_RADIUS = 3 * 1.5f;           /* SIFT_ORI_RADIUS */
static const float ORI_PEAK_RATIO = 0.8f;
static const float DESCR_SCL_FCTR = 3.f;
static const float DESCR_MAG_THR = 0.2f;
static const float INT_DESCR_FCTR = 512.f;
static const float DOG_THRESHOLD = 8;               /* literal at src/sift.cpp:564 */
static const double CV_PI_D = 3.1415926535897932384626433832795;

/* ---- OpenCV scalar helpers ------------------------- */
/* cvRound: SSE2 cvtss2si / cvtsd2si under the default MXCSR = half-to-even. */
static inline int round_f(float v) { return (int)lrintf(v); }
static inline int round_d(double v) { return (int)lrint(v); }
static inline int floor_f(float v) { int i = (int)v; return i - (i > v); }
static inline float sat_u8(float v) {
  int iv = round_f(v);
  return (float)(iv < 0 ? 0 : iv > 255 ? 255 : iv);
}
int so_cv_round(float v) { return round_f(v); }

/* libm calls on the path -- powf (src/sift.cpp:384), cosf/sinf (:583-584).
 * glibc's float versions are not correctly rounded (measured here over every
 * float in [0, 2pi): sinf differs from the correctly rounded value on 0.094%
 * of inputs, cosf on 0.041%; powf(2, y) on 0.0045% of y in [-0.5, 2)) and
 * glibc dispatches SSE2/FMA variants per CPU.  Both the oracle and the GPU
 * therefore evaluate them as (float)f((double)x), which is platform-stable
 * (SURVEY.md Appendix A).  This is a documented, unpinned deviation. */
static inline float pow2f_cr(float y) { return (float)exp2((double)y); }
static inline float cosf_cr(float x) { return (float)cos((double)x); }
static inline float sinf_cr(float x) { return (float)sin((double)x); }

/* ---- hal::exp32f (OpenCV 4.0 mathfuncs_core, EXPTAB_SCALE = 6) --------- */
static const double EXP_A0 = .9670371139572337719125840413672004409288e-2;
static const double EXP_PRESCALE = 1.4426950408889634073599246810019 * 64;
static const double EXP_POSTSCALE = 1. / 64;
static const double EXP_MAXVAL = 3000. * 64;
static float exp_tab[64];
static int exp_tab_ready = 0;

static void exp_tab_init(void) {
  if (exp_tab_ready) return;
  /* expTab[j] = 2^(j/64) * A0 in double (literal table), then (float). */
  for (int j = 0; j < 64; ++j) {
    double p = (double)exp2l((long double)j / 64.0L);
    exp_tab[j] = (float)(p * EXP_A0);
  }
  exp_tab_ready = 1;
}

void so_exp32f(const float* x, float* y, int n) {
  exp_tab_init();
  const float A4 = (float)(1.000000000000002438532970795181890933776 / EXP_A0);
  const float A3 = (float)(.6931471805521448196800669615864773144641 / EXP_A0);
  const float A2 = (float)(.2402265109513301490103372422686535526573 / EXP_A0);
  const float A1 = (float)(.5550339366753125211915322047004666939128e-1 / EXP_A0);
  const float lo = (float)(-EXP_MAXVAL / EXP_PRESCALE);
  const float hi = (float)(EXP_MAXVAL / EXP_PRESCALE);
  const float post = (float)EXP_POSTSCALE;
  for (int i = 0; i < n; ++i) {
    float v = x[i];
    v = v < lo ? lo : v;
    v = hi < v ? hi : v;
    v *= (float)EXP_PRESCALE;
    int vi = round_f(v);
    v = (v - (float)vi) * post;
    int t = (vi >> 6) + 127;
    t = !(t & ~255) ? t : t < 0 ? 0 : 255;
    union { int32_t i; float f; } sc;
    sc.i = t << 23;
    float poly = (((v + A1) * v + A2) * v + A3) * v + A4;
    y[i] = sc.f * exp_tab[vi & 63] * poly;
  }
}

/* ---- hal::fastAtan2, degrees (OpenCV 4.0 mathfuncs_core) --------------- */
void so_fast_atan2(const float* y, const float* x, float* out, int n) {
  const float deg = (float)(180 / CV_PI_D);
  const float p1 = 0.9997878412794807f * deg, p3 = -0.3258083974640975f * deg;
  const float p5 = 0.1555786518463281f * deg, p7 = -0.04432655554792128f * deg;
  const float eps = (float)DBL_EPSILON;
  for (int i = 0; i < n; ++i) {
    float ax = fabsf(x[i]), ay = fabsf(y[i]);
    float mn = ax < ay ? ax : ay, mx = ax < ay ? ay : ax;
    float c = mn / (mx + eps);
    float c2 = c * c;
    float a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x[i] < 0) a = 180.f - a;
    if (y[i] < 0) a = 360.f - a;
    out[i] = a;
  }
}

/* ---- hal::magnitude32f ------------------------------------------------- */
void so_magnitude32f(const float* x, const float* y, float* out, int n) {
  for (int i = 0; i < n; ++i) {
    float a = x[i], b = y[i];
    out[i] = sqrtf(a * a + b * b);
  }
}

/* ---- Matx33f::solve(DECOMP_LU): 3x3 Cramer (OpenCV Matx_FastSolveOp) --- */
int so_solve3(const float* a, const float* b, float* x) {
#define A(i, j) a[(i)*3 + (j)]
  float d = (float)(A(0, 0) * (A(1, 1) * A(2, 2) - A(2, 1) * A(1, 2)) -
                    A(0, 1) * (A(1, 0) * A(2, 2) - A(2, 0) * A(1, 2)) +
                    A(0, 2) * (A(1, 0) * A(2, 1) - A(2, 0) * A(1, 1)));
  if (d == 0) { x[0] = x[1] = x[2] = 0; return 0; }
  d = 1 / d;
  x[0] = d * (b[0] * (A(1, 1) * A(2, 2) - A(1, 2) * A(2, 1)) -
              A(0, 1) * (b[1] * A(2, 2) - A(1, 2) * b[2]) +
              A(0, 2) * (b[1] * A(2, 1) - A(1, 1) * b[2]));
  x[1] = d * (A(0, 0) * (b[1] * A(2, 2) - A(1, 2) * b[2]) -
              b[0] * (A(1, 0) * A(2, 2) - A(1, 2) * A(2, 0)) +
              A(0, 2) * (A(1, 0) * b[2] - b[1] * A(2, 0)));
  x[2] = d * (A(0, 0) * (A(1, 1) * b[2] - b[1] * A(2, 1)) -
              A(0, 1) * (A(1, 0) * b[2] - b[1] * A(2, 0)) +
              b[0] * (A(1, 0) * A(2, 1) - A(1, 1) * A(2, 0)));
#undef A
  return 1;
}

/* ---- layout helpers ---------------------------------------------------- */
void so_octave_shapes(int rows, int cols, int n_octaves, int* orows, int* ocols) {
  int r = rows, c = cols;
  for (int o = 0; o < n_octaves; ++o) {
    orows[o] = r;
    ocols[o] = c;
    r /= 2; /* Size(src.cols/2, src.rows/2), src/sift.cpp:254 */
    c /= 2;
  }
}

size_t so_pyramid_offsets(int rows, int cols, int n_octaves, int per, size_t* off) {
  int orow[32], ocol[32];
  so_octave_shapes(rows, cols, n_octaves, orow, ocol);
  size_t t = 0;
  for (int o = 0; o < n_octaves; ++o)
    for (int s = 0; s < per; ++s) {
      if (off) off[o * per + s] = t;
      t += (size_t)orow[o] * ocol[o];
    }
  return t;
}

/* ---- getGaussianKernel (src/sift.cpp:95-108) --------------------------- */
int so_gaussian_kernel(float sigma, float* coeff) {
  int w = (int)floor(3 * sigma); /* float product, then floor */
  int size = 2 * w + 1;
  double norm = 1. / (2 * K_PI * sigma * sigma);  /* double chain            */
  double den = (double)(2 * sigma * sigma);        /* float chain, then double */
  for (int a = -w; a <= w; ++a)
    for (int b = -w; b <= w; ++b) {
      double g = norm * exp(-(a * a + b * b) * 1. / den);
      g = g * 8192;
      coeff[(a + w) * size + (b + w)] = (float)g;
    }
  return size;
}

/* ---- Gaussian_Blur (src/sift.cpp:110-153) ------------------------------
 * Sequential float dot product in tap raster order; the source's last row
 * and last column read as 0 (getSubMatrix bounds at :116). */
void so_gaussian_blur(const float* src, int rows, int cols, double sigma, float* dst) {
  int w0 = (int)floor(3 * (float)sigma);
  float* k = (float*)malloc(sizeof(float) * (size_t)(2 * w0 + 1) * (2 * w0 + 1));
  int ks = so_gaussian_kernel((float)sigma, k);
  int w = ks / 2;
  for (int y = 0; y < rows; ++y)
    for (int x = 0; x < cols; ++x) {
      float acc = 0;
      const float* kk = k;
      for (int a = -w; a <= w; ++a) {
        int yy = y + a;
        int rok = yy >= 0 && yy < rows - 1;
        for (int b = -w; b <= w; ++b, ++kk) {
          int xx = x + b;
          float e = (rok && xx >= 0 && xx < cols - 1) ? src[(size_t)yy * cols + xx] : 0.f;
          acc += e * *kk;
        }
      }
      dst[(size_t)y * cols + x] = acc / 8192;
    }
  free(k);
}

/* ---- Gaussian_Blur_1D (src/sift.cpp:157-217) ---------------------------
 * Unnormalised 1/sqrt(2 pi s^2) taps; the loop runs k in [-ks/2, ks/2 - 1]
 * (asymmetric, :196 and :207); last row (vertical) / column (horizontal)
 * treated as 0.  Row-partitioning over threads does not change results. */
void so_gaussian_blur_1d(const float* src, int rows, int cols, double sigma, float* dst) {
  int w = (int)floor(3 * sigma);
  int ks = 2 * w + 1;
  float* k = (float*)malloc(sizeof(float) * ks);
  for (int i = -w; i <= w; ++i)
    k[i + w] = (float)(1. / sqrt(2 * K_PI * sigma * sigma) *
                       exp(-((double)i * i) * 1. / (2 * sigma * sigma)));
  float* mid = (float*)malloc(sizeof(float) * (size_t)rows * cols);
  for (int y = 0; y < rows; ++y)
    for (int x = 0; x < cols; ++x) {
      float acc = 0;
      for (int t = -ks / 2; t < ks / 2; ++t)
        acc += (y + t < 0 || y + t >= rows - 1) ? 0 : src[(size_t)(y + t) * cols + x] * k[t + ks / 2];
      mid[(size_t)y * cols + x] = acc;
    }
  for (int y = 0; y < rows; ++y)
    for (int x = 0; x < cols; ++x) {
      float acc = 0;
      for (int t = -ks / 2; t < ks / 2; ++t)
        acc += (x + t < 0 || x + t >= cols - 1) ? 0 : mid[(size_t)y * cols + x + t] * k[t + ks / 2];
      dst[(size_t)y * cols + x] = acc;
    }
  free(mid);
  free(k);
}

/* ---- resize INTER_NEAREST (OpenCV resizeNN; src/sift.cpp:254) ---------- */
void so_resize_nn(const float* src, int srows, int scols, float* dst, int drows, int dcols) {
  double ifx = 1. / ((double)dcols / scols), ify = 1. / ((double)drows / srows);
  for (int y = 0; y < drows; ++y) {
    int sy = (int)floor(y * ify);
    if (sy > srows - 1) sy = srows - 1;
    for (int x = 0; x < dcols; ++x) {
      int sx = (int)floor(x * ifx);
      if (sx > scols - 1) sx = scols - 1;
      dst[(size_t)y * dcols + x] = src[(size_t)sy * scols + sx];
    }
  }
}

/* ---- buildGaussianPyramid (src/sift.cpp:219-263) ----------------------- */
void so_build_gaussian_pyramid(const float* img, int rows, int cols, int n_octaves, float* gpyr) {
  size_t off[32 * 5];
  int orow[32], ocol[32];
  so_pyramid_offsets(rows, cols, n_octaves, N_SCALES, off);
  so_octave_shapes(rows, cols, n_octaves, orow, ocol);
  float sig[N_SCALES];
  double k = pow(2.0, 1.0 / N_LAYERS);
  sig[0] = (float)K_SIGMA;
  for (int i = 1; i < N_SCALES; ++i) {
    double tot = pow(k * 1.0, (double)i) * K_SIGMA;
    sig[i] = (float)sqrt(tot * tot - K_SIGMA * K_SIGMA);
  }
  for (int o = 0; o < n_octaves; ++o)
    for (int s = 0; s < N_SCALES; ++s) {
      float* dst = gpyr + off[o * N_SCALES + s];
      if (o == 0 && s == 0) {
        /* createInitialImage: blur with sqrt(1.6^2 + 0.2^2), :224,:237 */
        so_gaussian_blur(img, rows, cols, sqrt(K_SIGMA * K_SIGMA + 0.2 * 0.2), dst);
      } else if (s == 0) {
        const float* src = gpyr + off[(o - 1) * N_SCALES + N_LAYERS];
        so_resize_nn(src, orow[o - 1], ocol[o - 1], dst, orow[o], ocol[o]);
      } else {
        so_gaussian_blur(gpyr + off[o * N_SCALES], orow[o], ocol[o], sig[s], dst);
      }
    }
}

/* ---- SIFT_FLAG_FAST pyramid (the library's separable form) -------------
 * Not the reference's arithmetic: the separable agreement mode of
 * sift-gpu_amd/csrc/pyramid_pc.hip, restated here so that its planes can be
 * checked bit for bit.  Taps g(a) = (float)(exp(-a^2 / den) / sqrt(2 pi s^2))
 * with den = (double)(2 s s) in float (the square root of getGaussianKernel's
 * normalisation, src/sift.cpp:97-107).  Every blur reads its source with zero
 * padding outside [0, rows-1) x [0, cols-1) (src/sift.cpp:116).
 *   row pass:            h = g0 x[c]; h = fmaf(g_k, x[c-k] + x[c+k], h), k = 1..w
 *   base column pass:    the same folded form down the column
 *   scale column pass:   o = g_w h[r-w]; o = fmaf(g_|d|, h[r+d], o), d = -w+1..w
 * Octave 0's plane 0 is the base blur (w = 4) of the image; plane 0 of octave
 * o > 0 is resize INTER_NEAREST of plane 2 of octave o-1 (src/sift.cpp:252). */
static int fast_taps(float sigma, float* g) {
  const int w = (int)floor(3 * sigma);
  const double den = (double)(2 * sigma * sigma);
  const double nrm = 1. / sqrt(2 * K_PI * sigma * sigma);
  for (int a = -w; a <= w; ++a) g[a + w] = (float)(nrm * exp(-(a * a) * 1. / den));
  return w;
}

static float fast_src(const float* p, int rows, int cols, int r, int c) {
  return (r >= 0 && r < rows - 1 && c >= 0 && c < cols - 1) ? p[(size_t)r * cols + c] : 0.f;
}

static void fast_blur(const float* src, int rows, int cols, float sigma, int folded_cols, float* dst) {
  float gt[64];
  const int w = fast_taps(sigma, gt);
  const float* g = gt + w; /* g[a], a in [-w, w] */
  float* h = (float*)malloc(sizeof(float) * (size_t)(rows + 2 * w) * cols);
  /* row pass for rows [-w, rows + w): zero rows outside give h = +0 */
#pragma omp parallel for schedule(static)
  for (int r = -w; r < rows + w; ++r)
    for (int c = 0; c < cols; ++c) {
      float v = g[0] * fast_src(src, rows, cols, r, c);
      for (int k = 1; k <= w; ++k)
        v = fmaf(g[k], fast_src(src, rows, cols, r, c - k) + fast_src(src, rows, cols, r, c + k), v);
      h[(size_t)(r + w) * cols + c] = v;
    }
#pragma omp parallel for schedule(static)
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) {
#define HH(rr) h[(size_t)((rr) + w) * cols + c]
      float o;
      if (folded_cols) {
        o = g[0] * HH(r);
        for (int k = 1; k <= w; ++k) o = fmaf(g[k], HH(r - k) + HH(r + k), o);
      } else {
        o = g[w] * HH(r - w);
        for (int d = -w + 1; d <= w; ++d) o = fmaf(g[d < 0 ? -d : d], HH(r + d), o);
      }
#undef HH
      dst[(size_t)r * cols + c] = o;
    }
  free(h);
}

void so_fast_pyramid(const float* img, int rows, int cols, int n_octaves, float* gpyr) {
  size_t off[32 * 5];
  int orow[32], ocol[32];
  so_pyramid_offsets(rows, cols, n_octaves, N_SCALES, off);
  so_octave_shapes(rows, cols, n_octaves, orow, ocol);
  float sig[N_SCALES];
  double k = pow(2.0, 1.0 / N_LAYERS);
  sig[0] = (float)sqrt(K_SIGMA * K_SIGMA + 0.2 * 0.2);
  for (int i = 1; i < N_SCALES; ++i) {
    double tot = pow(k * 1.0, (double)i) * K_SIGMA;
    sig[i] = (float)sqrt(tot * tot - K_SIGMA * K_SIGMA);
  }
  for (int o = 0; o < n_octaves; ++o)
    for (int s = 0; s < N_SCALES; ++s) {
      float* dst = gpyr + off[o * N_SCALES + s];
      if (o == 0 && s == 0)
        fast_blur(img, rows, cols, sig[0], 1, dst);
      else if (s == 0)
        so_resize_nn(gpyr + off[(o - 1) * N_SCALES + N_LAYERS], orow[o - 1], ocol[o - 1], dst, orow[o], ocol[o]);
      else
        fast_blur(gpyr + off[o * N_SCALES], orow[o], ocol[o], sig[s], 0, dst);
    }
}

/* ---- buildDoGPyramid (src/sift.cpp:265-283) ---------------------------- */
void so_build_dog_pyramid(const float* gpyr, int rows, int cols, int n_octaves, float* dog) {
  size_t goff[32 * 5], doff[32 * 4];
  int orow[32], ocol[32];
  so_pyramid_offsets(rows, cols, n_octaves, N_SCALES, goff);
  so_pyramid_offsets(rows, cols, n_octaves, 4, doff);
  so_octave_shapes(rows, cols, n_octaves, orow, ocol);
  for (int o = 0; o < n_octaves; ++o)
    for (int s = 0; s < 4; ++s) {
      const float* a = gpyr + goff[o * N_SCALES + s];
      const float* b = gpyr + goff[o * N_SCALES + s + 1];
      float* d = dog + doff[o * 4 + s];
      size_t n = (size_t)orow[o] * ocol[o];
      for (size_t i = 0; i < n; ++i) d[i] = b[i] - a[i];
    }
}

/* ---- adjustLocalExtrema (src/sift.cpp:287-388) ------------------------- */
typedef struct { const float* p[32 * 4]; int rows[32], cols[32]; } plane_set;

#define AT(pl, yy, xx) ((pl)[(size_t)(yy) * ncols + (xx)])

static int adjust_local_extrema(const plane_set* dog, so_keypoint* kp, int oct, int* layer_io,
                                int* r_io, int* c_io) {
  const float img_scale = 1. / 255;
  const float deriv_scale = img_scale * 0.5f;
  const float second_scale = img_scale;
  const float cross_scale = img_scale * 0.25f;
  const int ncols = dog->cols[oct], nrows = dog->rows[oct];
  int layer = *layer_io, r = *r_io, c = *c_io;
  float xi = 0, xr = 0, xc = 0, contr = 0;
  int it = 0;
  for (; it < MAX_INTERP; ++it) {
    const float* cur = dog->p[oct * 4 + layer];
    const float* lo = dog->p[oct * 4 + layer - 1];
    const float* hi = dog->p[oct * 4 + layer + 1];
    float g[3] = {(AT(cur, r, c + 1) - AT(cur, r, c - 1)) * deriv_scale,
                  (AT(cur, r + 1, c) - AT(cur, r - 1, c)) * deriv_scale,
                  (AT(hi, r, c) - AT(lo, r, c)) * deriv_scale};
    float v2 = (float)AT(cur, r, c) * 2;
    float dxx = (AT(cur, r, c + 1) + AT(cur, r, c - 1) - v2) * second_scale;
    float dyy = (AT(cur, r + 1, c) + AT(cur, r - 1, c) - v2) * second_scale;
    float dss = (AT(hi, r, c) + AT(lo, r, c) - v2) * second_scale;
    float dxy = (AT(cur, r + 1, c + 1) - AT(cur, r + 1, c - 1) - AT(cur, r - 1, c + 1) +
                 AT(cur, r - 1, c - 1)) * cross_scale;
    float dxs = (AT(hi, r, c + 1) - AT(hi, r, c - 1) - AT(lo, r, c + 1) + AT(lo, r, c - 1)) *
                cross_scale;
    float dys = (AT(hi, r + 1, c) - AT(hi, r - 1, c) - AT(lo, r + 1, c) + AT(lo, r - 1, c)) *
                cross_scale;
    float H[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss};
    float X[3];
    so_solve3(H, g, X);
    xi = -X[2];
    xr = -X[1];
    xc = -X[0];
    if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
    if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) ||
        fabsf(xc) > (float)(INT_MAX / 3))
      return 0;
    c += round_f(xc);
    r += round_f(xr);
    layer += round_f(xi);
    if (layer < 1 || layer > N_LAYERS || c < IMG_BORDER || c >= ncols - IMG_BORDER ||
        r < IMG_BORDER || r >= nrows - IMG_BORDER)
      return 0;
  }
  if (it >= MAX_INTERP) return 0;
  {
    const float* cur = dog->p[oct * 4 + layer];
    const float* lo = dog->p[oct * 4 + layer - 1];
    const float* hi = dog->p[oct * 4 + layer + 1];
    float g0 = (AT(cur, r, c + 1) - AT(cur, r, c - 1)) * deriv_scale;
    float g1 = (AT(cur, r + 1, c) - AT(cur, r - 1, c)) * deriv_scale;
    float g2 = (AT(hi, r, c) - AT(lo, r, c)) * deriv_scale;
    float t = 0; /* Matx::dot: s = 0; s += a_i*b_i */
    t += g0 * xc;
    t += g1 * xr;
    t += g2 * xi;
    contr = AT(cur, r, c) * img_scale + t * 0.5f;
    if (fabsf(contr) * N_LAYERS < (float)K_CONTRAST) return 0;
    float v2 = AT(cur, r, c) * 2.f;
    float dxx = (AT(cur, r, c + 1) + AT(cur, r, c - 1) - v2) * second_scale;
    float dyy = (AT(cur, r + 1, c) + AT(cur, r - 1, c) - v2) * second_scale;
    float dxy = (AT(cur, r + 1, c + 1) - AT(cur, r + 1, c - 1) - AT(cur, r - 1, c + 1) +
                 AT(cur, r - 1, c - 1)) * cross_scale;
    float tr = dxx + dyy;
    float det = dxx * dyy - dxy * dxy;
    const float et = (float)K_EDGE;
    if (det <= 0 || tr * tr * et >= (et + 1) * (et + 1) * det) return 0;
  }
  kp->x = (c + xc) * (1 << oct);
  kp->y = (r + xr) * (1 << oct);
  kp->octave = oct + (layer << 8) + (round_d((xi + 0.5) * 255) << 16);
  kp->size = (float)K_SIGMA * pow2f_cr((layer + xi) / N_LAYERS) * (1 << oct) * 2;
  kp->response = fabsf(contr);
  *layer_io = layer;
  *r_io = r;
  *c_io = c;
  return 1;
}

/* ---- calcOrientationHist (src/sift.cpp:389-458) ------------------------ */
static float orientation_hist(const float* img, int nrows, int ncols, int py, int px, int radius,
                              float sigma, float* hist) {
  const int n = ORI_BINS;
  int len = (radius * 2 + 1) * (radius * 2 + 1);
  float* X = (float*)malloc(sizeof(float) * (size_t)len * 4);
  float *Y = X + len, *O = Y + len, *W = O + len;
  float tmp[ORI_BINS + 4];
  float* th = tmp + 2;
  float escale = -1.f / (2.f * sigma * sigma);
  for (int i = 0; i < n; ++i) th[i] = 0.f;
  int k = 0;
  for (int i = -radius; i <= radius; ++i) {
    int y = py + i;
    if (y <= 0 || y >= nrows - 1) continue;
    for (int j = -radius; j <= radius; ++j) {
      int x = px + j;
      if (x <= 0 || x >= ncols - 1) continue;
      X[k] = (float)(AT(img, y, x + 1) - AT(img, y, x - 1));
      Y[k] = (float)(AT(img, y - 1, x) - AT(img, y + 1, x));
      W[k] = (i * i + j * j) * escale;
      ++k;
    }
  }
  len = k;
  so_exp32f(W, W, len);
  so_fast_atan2(Y, X, O, len);
  so_magnitude32f(X, Y, X, len);
  for (k = 0; k < len; ++k) {
    int bin = round_f((n / 360.f) * O[k]);
    if (bin >= n) bin -= n;
    if (bin < 0) bin += n;
    th[bin] += W[k] * X[k];
  }
  th[-1] = th[n - 1];
  th[-2] = th[n - 2];
  th[n] = th[0];
  th[n + 1] = th[1];
  for (int i = 0; i < n; ++i)
    hist[i] = (th[i - 2] + th[i + 2]) * (1.f / 16.f) + (th[i - 1] + th[i + 1]) * (4.f / 16.f) +
              th[i] * (6.f / 16.f);
  float mx = hist[0];
  for (int i = 1; i < n; ++i) mx = mx < hist[i] ? hist[i] : mx;
  free(X);
  return mx;
}

/* ---- findScaleSpaceExtremaComputer + driver (src/sift.cpp:462-577) ----- */
static int scan_layer(const plane_set* gp, const plane_set* dog, int o, int layer, so_keypoint* kps,
                      int cap, int count) {
  const int n = ORI_BINS;
  const float* img = dog->p[o * 4 + layer];
  const float* prv = dog->p[o * 4 + layer - 1];
  const float* nxt = dog->p[o * 4 + layer + 1];
  const int nrows = dog->rows[o], ncols = dog->cols[o];
  const int st = ncols;
  so_keypoint kp = {0, 0, 0, -1, 0, 0, -1}; /* cv::KeyPoint() defaults */
  float hist[ORI_BINS];
  for (int r = IMG_BORDER; r < nrows - IMG_BORDER; ++r) {
    const float* cp = img + (size_t)r * st;
    const float* pp = prv + (size_t)r * st;
    const float* np = nxt + (size_t)r * st;
    for (int c = IMG_BORDER; c < ncols - IMG_BORDER; ++c) {
      float v = cp[c];
      if (!(fabsf(v) > DOG_THRESHOLD)) continue;
      int is_ext;
      if (v > 0) {
        is_ext = 1;
        for (int dy = -1; dy <= 1 && is_ext; ++dy)
          for (int dx = -1; dx <= 1; ++dx) {
            int q = c + dy * st + dx;
            if (!(v >= np[q] && v >= pp[q] && ((dy == 0 && dx == 0) || v >= cp[q]))) { is_ext = 0; break; }
          }
      } else if (v < 0) {
        is_ext = 1;
        for (int dy = -1; dy <= 1 && is_ext; ++dy)
          for (int dx = -1; dx <= 1; ++dx) {
            int q = c + dy * st + dx;
            if (!(v <= np[q] && v <= pp[q] && ((dy == 0 && dx == 0) || v <= cp[q]))) { is_ext = 0; break; }
          }
      } else {
        is_ext = 0;
      }
      if (!is_ext) continue;
      int r1 = r, c1 = c, ly = layer;
      if (!adjust_local_extrema(dog, &kp, o, &ly, &r1, &c1)) continue;
      float scl = kp.size * 0.5f / (1 << o);
      const float* g = gp->p[o * N_SCALES + ly];
      float omax = orientation_hist(g, nrows, ncols, r1, c1, round_f(ORI_RADIUS * scl),
                                    ORI_SIG_FCTR * scl, hist);
      float thr = (float)(omax * ORI_PEAK_RATIO);
      for (int j = 0; j < n; ++j) {
        int l = j > 0 ? j - 1 : n - 1;
        int rr = j < n - 1 ? j + 1 : 0;
        if (hist[j] > hist[l] && hist[j] > hist[rr] && hist[j] >= thr) {
          float bin = j + 0.5f * (hist[l] - hist[rr]) / (hist[l] - 2 * hist[j] + hist[rr]);
          bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
          kp.angle = 360.f - (float)((360.f / n) * bin);
          if (fabsf(kp.angle - 360.f) < FLT_EPSILON) kp.angle = 0.f;
          if (count < cap) kps[count] = kp;
          ++count;
        }
      }
    }
  }
  return count;
}

static void make_planes(const float* base, int rows, int cols, int n_octaves, int per, plane_set* ps) {
  size_t off[32 * 5];
  so_pyramid_offsets(rows, cols, n_octaves, per, off);
  so_octave_shapes(rows, cols, n_octaves, ps->rows, ps->cols);
  for (int i = 0; i < n_octaves * per; ++i) ps->p[i] = base + off[i];
}

int so_find_scale_space_extrema(const float* gpyr, const float* dog, int rows, int cols,
                                int n_octaves, so_keypoint* kps, int cap) {
  plane_set gp, dp;
  make_planes(gpyr, rows, cols, n_octaves, N_SCALES, &gp);
  make_planes(dog, rows, cols, n_octaves, 4, &dp);
  int count = 0;
  for (int o = 0; o < n_octaves; ++o)
    for (int i = 1; i <= N_LAYERS; ++i) count = scan_layer(&gp, &dp, o, i, kps, cap, count);
  return count;
}

/* ---- calcSIFTDescriptor (src/sift.cpp:579-722) ------------------------- */
static void sift_descriptor(const float* img, int nrows, int ncols, float ptx, float pty, float ori,
                            float scl, float* dst) {
  const int d = DESC_W, n = DESC_BINS;
  int px = round_f(ptx), py = round_f(pty);
  float cos_t = cosf_cr(ori * (float)(CV_PI_D / 180));
  float sin_t = sinf_cr(ori * (float)(CV_PI_D / 180));
  float bins_per_rad = n / 360.f;
  float exp_scale = -1.f / (d * d * 0.5f);
  float hist_width = DESCR_SCL_FCTR * scl;
  int radius = round_f(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
  int diag = (int)sqrt(((double)ncols) * ncols + ((double)nrows) * nrows);
  if (radius > diag) radius = diag;
  cos_t /= hist_width;
  sin_t /= hist_width;
  int len = (radius * 2 + 1) * (radius * 2 + 1);
  const int hlen = (d + 2) * (d + 2) * (n + 2);
  float* buf = (float*)malloc(sizeof(float) * ((size_t)len * 6 + hlen));
  float *X = buf, *Y = X + len, *O = Y + len, *W = O + len, *RB = W + len, *CB = RB + len;
  float* hist = CB + len;
  for (int i = 0; i < hlen; ++i) hist[i] = 0.;
  int k = 0;
  for (int i = -radius; i <= radius; ++i)
    for (int j = -radius; j <= radius; ++j) {
      float c_rot = j * cos_t - i * sin_t;
      float r_rot = j * sin_t + i * cos_t;
      float rbin = r_rot + d / 2 - 0.5f;
      float cbin = c_rot + d / 2 - 0.5f;
      int r = py + i, c = px + j;
      if (rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < nrows - 1 && c > 0 &&
          c < ncols - 1) {
        X[k] = (float)(AT(img, r, c + 1) - AT(img, r, c - 1));
        Y[k] = (float)(AT(img, r - 1, c) - AT(img, r + 1, c));
        RB[k] = rbin;
        CB[k] = cbin;
        W[k] = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
        ++k;
      }
    }
  len = k;
  so_fast_atan2(Y, X, O, len);
  so_magnitude32f(X, Y, Y, len); /* Mag aliases Y in the reference */
  so_exp32f(W, W, len);
  for (k = 0; k < len; ++k) {
    float rbin = RB[k], cbin = CB[k];
    float obin = (O[k] - ori) * bins_per_rad;
    float mag = Y[k] * W[k];
    int r0 = floor_f(rbin), c0 = floor_f(cbin), o0 = floor_f(obin);
    rbin -= r0;
    cbin -= c0;
    obin -= o0;
    if (o0 < 0) o0 += n;
    if (o0 >= n) o0 -= n;
    float v_r1 = mag * rbin, v_r0 = mag - v_r1;
    float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
    float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
    float v111 = v_rc11 * obin, v110 = v_rc11 - v111;
    float v101 = v_rc10 * obin, v100 = v_rc10 - v101;
    float v011 = v_rc01 * obin, v010 = v_rc01 - v011;
    float v001 = v_rc00 * obin, v000 = v_rc00 - v001;
    int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
    hist[idx] += v000;
    hist[idx + 1] += v001;
    hist[idx + (n + 2)] += v010;
    hist[idx + (n + 3)] += v011;
    hist[idx + (d + 2) * (n + 2)] += v100;
    hist[idx + (d + 2) * (n + 2) + 1] += v101;
    hist[idx + (d + 3) * (n + 2)] += v110;
    hist[idx + (d + 3) * (n + 2) + 1] += v111;
  }
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) {
      int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
      hist[idx] += hist[idx + n];
      hist[idx + 1] += hist[idx + n + 1];
      for (k = 0; k < n; ++k) dst[(i * d + j) * n + k] = hist[idx + k];
    }
  const int dl = d * d * n;
  float nrm2 = 0;
  for (k = 0; k < dl; ++k) nrm2 += dst[k] * dst[k];
  float thr = sqrtf(nrm2) * DESCR_MAG_THR;
  nrm2 = 0;
  for (k = 0; k < dl; ++k) {
    float v = dst[k] < thr ? dst[k] : thr; /* std::min(dst, thr) */
    dst[k] = v;
    nrm2 += v * v;
  }
  float s = sqrtf(nrm2);
  nrm2 = INT_DESCR_FCTR / (s < FLT_EPSILON ? FLT_EPSILON : s);
  for (k = 0; k < dl; ++k) dst[k] = sat_u8(dst[k] * nrm2);
  float nrm1 = 0;
  for (k = 0; k < dl; ++k) {
    dst[k] *= nrm2;
    nrm1 += dst[k];
  }
  nrm1 = 1.f / (nrm1 < FLT_EPSILON ? FLT_EPSILON : nrm1);
  for (k = 0; k < dl; ++k) dst[k] = sqrtf(dst[k] * nrm1);
  free(buf);
}

/* ---- calDescriptor + unpackOctave (src/sift.cpp:724-753) --------------- */
static int g_threads = 1;
void so_set_threads(int n) { g_threads = n < 1 ? 1 : n; }

void so_calc_descriptors(const float* gpyr, int rows, int cols, int n_octaves,
                         const so_keypoint* kps, int n, float* desc, int first_octave) {
  plane_set gp;
  make_planes(gpyr, rows, cols, n_octaves, N_SCALES, &gp);
#ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads) schedule(dynamic, 16)
#endif
  for (int i = 0; i < n; ++i) {
    so_keypoint kp = kps[i];
    int octave = kp.octave & 255;
    int layer = (kp.octave >> 8) & 255;
    octave = octave < 128 ? octave : (-128 | octave);
    float scale = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
    float size = kp.size * scale;
    float ptx = kp.x * scale, pty = kp.y * scale;
    int pi = (octave - first_octave) * N_SCALES + layer;
    float angle = 360.f - kp.angle;
    if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
    int oi = octave - first_octave;
    sift_descriptor(gp.p[pi], gp.rows[oi], gp.cols[oi], ptx, pty, angle, size * 0.5f,
                    desc + (size_t)i * 128);
  }
}

/* ---- SIFT_NCL (src/sift.cpp:59-91) ------------------------------------- */
int so_sift(const float* img, int rows, int cols, int n_octaves, so_keypoint** kps_out,
            float** desc_out) {
  size_t ng = so_pyramid_offsets(rows, cols, n_octaves, N_SCALES, NULL);
  size_t nd = so_pyramid_offsets(rows, cols, n_octaves, 4, NULL);
  float* g = (float*)malloc(sizeof(float) * ng);
  float* d = (float*)malloc(sizeof(float) * nd);
  so_build_gaussian_pyramid(img, rows, cols, n_octaves, g);
  so_build_dog_pyramid(g, rows, cols, n_octaves, d);
  int cap = 4096;
  so_keypoint* kps = (so_keypoint*)malloc(sizeof(so_keypoint) * cap);
  int n = so_find_scale_space_extrema(g, d, rows, cols, n_octaves, kps, cap);
  if (n > cap) {
    free(kps);
    cap = n;
    kps = (so_keypoint*)malloc(sizeof(so_keypoint) * cap);
    n = so_find_scale_space_extrema(g, d, rows, cols, n_octaves, kps, cap);
  }
  float* desc = (float*)malloc(sizeof(float) * 128 * (size_t)(n > 0 ? n : 1));
  so_calc_descriptors(g, rows, cols, n_octaves, kps, n, desc, 0);
  free(g);
  free(d);
  *kps_out = kps;
  *desc_out = desc;
  return n;
}

void so_free(void* p) { free(p); }

/* ---- synthetic image --------------------------- */
static inline uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

void so_synth_image(int b, int rows, int cols, float* out) {
  static const int S[6] = {3, 6, 12, 24, 48, 96};
  static const int A[6] = {48, 56, 56, 48, 40, 32};
  uint32_t s = 0x5EED0000u + (uint32_t)b;
  for (int y = 0; y < rows; ++y)
    for (int x = 0; x < cols; ++x) {
      int acc = 0;
      for (int k = 0; k < 6; ++k) {
        uint32_t salt = s * 0x9E3779B1u + (uint32_t)k * 0x85EBCA6Bu;
        int gx = x / S[k], gy = y / S[k];
        int fx = (x % S[k]) * 256 / S[k], fy = (y % S[k]) * 256 / S[k];
#define LAT(a, bb) ((int)(lowbias32((uint32_t)(a) * 73856093u ^ (uint32_t)(bb) * 19349663u ^ salt) & 255) - 128)
        int l00 = LAT(gx, gy), l10 = LAT(gx + 1, gy), l01 = LAT(gx, gy + 1), l11 = LAT(gx + 1, gy + 1);
#undef LAT
        int v = ((l00 * (256 - fx) + l10 * fx) * (256 - fy) + (l01 * (256 - fx) + l11 * fx) * fy) >> 16;
        acc += A[k] * v;
      }
      int p = 128 + (acc >> 7);
      p = p < 0 ? 0 : p > 255 ? 255 : p;
      out[(size_t)y * cols + x] = (float)p;
    }
}

/* ---- element-wise helper evaluation (test hook) ------------------------- */
void so_helper(int op, const float* a, const float* b, float* out, int n) {
  switch (op) {
    case 0: so_exp32f(a, out, n); return;
    case 1: so_fast_atan2(a, b, out, n); return;
    case 2: so_magnitude32f(a, b, out, n); return;
    default: break;
  }
  for (int i = 0; i < n; ++i) {
    float r;
    switch (op) {
      case 3: r = cosf_cr(a[i]); break;
      case 4: r = sinf_cr(a[i]); break;
      case 5: r = pow2f_cr(a[i]); break;
      case 6: r = (float)round_f(a[i]); break;
      default: r = (float)floor_f(a[i]); break;
    }
    out[i] = r;
  }
}
