// pyramid_fast.hip -- SIFT_FLAG_FAST Gaussian pyramid for gfx950.
//
// The north_star's separable form of buildGaussianPyramid (src/sift.cpp:229-263).
// Every scale is still blurred from its octave base with the reference's
// sigma and kernel width (sig[] at :240-245, w = floor(3 sigma) at :97) and the
// reference's source padding (rows / cols outside [0, rows-1) x [0, cols-1)
// read as 0, getSubMatrix :116), but the 2-D kernel
// K[a][b] = 8192 g(a) g(b) (:103-104) is applied as a row pass and a column
// pass with fused multiply-adds.  That is not bit-exact with the reference's
// 2-D float chain (different rounding order); DESIGN.md §8 and
// tests/test_gpu_fast.py give the measured difference.
//
// One launch per octave writes all five planes of that octave:
//   octave 0:  base = blur9(image): row pass into a 16-row ring, column pass
//   octave o:  base = INTER_NEAREST half of octave o-1, scale 2 (:252-254)
//   scale s:   row pass of the base rows into a per-scale ring of 8 + 2 w_s
//              rows, column pass out of the ring.
// A workgroup owns a 128-column strip and walks a chunk of rows 8 at a time,
// so every row pass is done once per row (the vertical halo is carried in the
// rings, not recomputed) and every source pixel is read from HBM once (plus
// an 18-column halo that hits L2).  Bound: HBM, 24 algorithmic bytes per pixel
// (one read, five plane writes) against ~180 FMA per pixel.
#include "common.hpp"

#include <math.h>

namespace sift {

namespace {

constexpr int kFW = 128;               // output columns per strip
constexpr int kRB = 8;                 // rows per step
constexpr int kH = 18;                 // widest scale half-width (sig[4] = 6.197)
constexpr int kBW = kFW + 2 * kH;      // 164 base columns per strip
constexpr int kBP = 172;               // base / row-pass ring pitch (== 4 mod 8)
constexpr int kIP = 180;               // image staging pitch (176 columns used)
constexpr int kIQ = 44;                // float4 per staged image row
constexpr int kRP = 132;               // scale ring pitch (== 4 mod 8)
constexpr int kHbRows = 16;            // octave-0 row-pass ring: rows [Z-4, Z+12)
constexpr int kStage = kRB * kIP;      // staged image rows / base rows (aliased)
// scale rings: 8 + 2w rows for w = 4, 8, 12, 18
constexpr int kRing4 = 0, kRing8 = 16, kRing12 = 40, kRing18 = 72, kRingRows = 116;
constexpr int kLds0 = kStage + kHbRows * kBP + kRingRows * kRP;   // floats, octave 0
constexpr int kLdsN = kStage + kRingRows * kRP + kBW;             // floats (+ column map), octave > 0
static_assert(kRB * kBP <= kStage, "base rows alias the image staging rows");
static_assert(kBP % 8 == 4 && kRP % 8 == 4 && kIP % 4 == 0, "b128 row pitches");
static_assert(kLds0 % 4 == 0 && kLdsN % 4 == 0, "float4 LDS arrays");

// Row pass of one scale: h[Z + r][8j + p] = sum_b g[b] base[r][8j + p + 18 - W + b].
// The 16-lane groups of a ds_read_b128 hold two whole base rows x 8 column
// groups; with kBP == 4 (mod 8) their 16-byte slots are distinct (conflict free).
template <int W>
__device__ __forceinline__ void row_pass(const float* __restrict__ bs, float* __restrict__ ring,
                                         const float* __restrict__ g, int r, int j, int slot) {
  constexpr int ST = (kH - W) & ~3, E = (kH - W) & 3;
  constexpr int L = (E + kRB + 2 * W + 3) & ~3;
  float win[L];
  const float4* src = reinterpret_cast<const float4*>(bs + r * kBP + 8 * j + ST);
#pragma unroll
  for (int q = 0; q < L / 4; ++q) {
    const float4 t = src[q];
    win[4 * q] = t.x;
    win[4 * q + 1] = t.y;
    win[4 * q + 2] = t.z;
    win[4 * q + 3] = t.w;
  }
  float acc[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) acc[p] = 0.f;
#pragma unroll
  for (int b = 0; b <= 2 * W; ++b) {
    const float k = g[b];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = __builtin_fmaf(win[E + p + b], k, acc[p]);
  }
  float4* dst = reinterpret_cast<float4*>(ring + slot * kRP + 8 * j);
  dst[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  dst[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// Column pass of one scale: rows [Z - W, Z - W + 8) of the plane, column col,
// from ring rows [Z - 2W, Z + 8) (exactly the ring's 8 + 2W slots, from s0).
template <int W>
__device__ __forceinline__ void col_pass(const float* __restrict__ ring, const float* __restrict__ g,
                                         int col, int s0, float* __restrict__ plane,
                                         long long pitch, int Z, int y0, int y1, bool colok) {
  constexpr int M = kRB + 2 * W;
  float win[M];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    int s = s0 + k;
    s = s >= M ? s - M : s;
    win[k] = ring[s * kRP + col];
  }
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
  for (int a = 0; a <= 2 * W; ++a) {
    const float k = g[a];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_fmaf(win[i + a], k, acc[i]);
  }
  if (colok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int y = Z - W + i;
      if (y >= y0 && y < y1) plane[(long long)y * pitch] = acc[i];
    }
  }
}

}  // namespace

struct FastCoefs {  // 1-D taps: K[a][b] / 8192 = g(a) g(b) up to float rounding
  float base[9];
  float s1[9], s2[17], s3[25], s4[37];
};

struct FastArgs {
  float* gpyr;
  long long g_img;
  long long off[kScales];  // plane offsets of this octave in the image block
  const float* src;        // octave 0: the input images; else gpyr
  long long src_off, s_pitch, s_img;
  const FastCoefs* coef;
  double ify, ifx;         // resize NN scale factors (octave > 0)
  int pitch, rows, cols;
  int srows, scols;        // source (previous octave) shape
  int chunk;               // rows per workgroup (multiple of kRB)
  int vec;                 // octave 0: 16-byte source row loads are legal
};

namespace {

// Octave-0 image rows [Y, Y+8) x columns [x0-24, x0+152) -> 2 float4 per lane
// (lanes >= 96 hold one).  Source padding of the base blur: 0 outside
// [0, rows-1) x [0, cols-1).
__device__ __forceinline__ void fetch_image(const FastArgs& A, const float* __restrict__ img, int x0,
                                            int Y, float4 (&v)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < kRB * kIQ) {
      const int r = i / kIQ, q = i - r * kIQ;
      const int y = Y + r, x = x0 - 24 + 4 * q;
      if (y >= 0 && y < A.rows - 1) {
        const float* row = img + (long long)y * A.s_pitch;
        const int lim = A.cols - 1;
        if (A.vec && x >= 0 && x + 3 < lim) {
          v[u] = *reinterpret_cast<const float4*>(row + x);
        } else {
          v[u].x = (x >= 0 && x < lim) ? row[x] : 0.f;
          v[u].y = (x + 1 >= 0 && x + 1 < lim) ? row[x + 1] : 0.f;
          v[u].z = (x + 2 >= 0 && x + 2 < lim) ? row[x + 2] : 0.f;
          v[u].w = (x + 3 >= 0 && x + 3 < lim) ? row[x + 3] : 0.f;
        }
      }
    }
  }
}

__device__ __forceinline__ void put_image(float* __restrict__ stage, const float4 (&v)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < kRB * kIQ) {
      const int r = i / kIQ, q = i - r * kIQ;
      reinterpret_cast<float4*>(stage + r * kIP)[q] = v[u];
    }
  }
}

// Octave-0 row pass of the base blur: ring rows [Y, Y+8), base columns
// [0, 168) (column c <-> image column x0 - 18 + c; 164 are used).
__device__ __forceinline__ void hb_pass(const float* __restrict__ stage, float* __restrict__ hb,
                                        const float* __restrict__ g, int Y) {
  const int t = threadIdx.x;
  if (t >= kRB * 21) return;
  const int r = t / 21, j = t - r * 21;
  float win[20];
  const float4* src = reinterpret_cast<const float4*>(stage + r * kIP + 8 * j);
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const float4 v = src[q];
    win[4 * q] = v.x;
    win[4 * q + 1] = v.y;
    win[4 * q + 2] = v.z;
    win[4 * q + 3] = v.w;
  }
  float acc[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) acc[p] = 0.f;
#pragma unroll
  for (int b = 0; b < 9; ++b) {
    const float k = g[b];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = __builtin_fmaf(win[p + b + 2], k, acc[p]);
  }
  float4* dst = reinterpret_cast<float4*>(hb + ((Y + r) & (kHbRows - 1)) * kBP + 8 * j);
  dst[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  dst[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// Stores one base value: the plane-0 interior (unpadded) to HBM and the
// padded copy (0 outside [0, rows-1) x [0, cols-1)) as the scales' source.
__device__ __forceinline__ void put_base(const FastArgs& A, float* __restrict__ bs, float* __restrict__ plane0,
                                         int r, int c, int y, int x, int y0, int y1, float v) {
  if (c >= kH && c < kH + kFW && x < A.cols && y >= y0 && y < y1) plane0[(long long)y * A.pitch + x] = v;
  const bool src_ok = y >= 0 && y < A.rows - 1 && x >= 0 && x < A.cols - 1;
  bs[r * kBP + c] = src_ok ? v : 0.f;
}

template <bool OCT0>
__global__ __launch_bounds__(256, 2) void pyr_fast_kernel(FastArgs A) {
  __shared__ float4 lds4[(OCT0 ? kLds0 : kLdsN) / 4];
  float* const lds = reinterpret_cast<float*>(lds4);
  float* const stage = lds;
  float* const hb = lds + kStage;  // octave 0 only
  float* const rings = lds + kStage + (OCT0 ? kHbRows * kBP : 0);
  int* const xmap = reinterpret_cast<int*>(rings + kRingRows * kRP);  // octave > 0 only

  const int t = threadIdx.x;
  const int b = blockIdx.z;
  const int x0 = blockIdx.x * kFW;
  const int y0 = blockIdx.y * A.chunk;
  const int y1 = min(y0 + A.chunk, A.rows);
  const int R = A.rows, C = A.cols;
  float* const gimg = A.gpyr + b * A.g_img;
  float* const plane0 = gimg + A.off[0];
  const FastCoefs* __restrict__ K = A.coef;
  const int rbase = y0 - 64;  // ring slot of row y: (y - rbase) mod ring rows (rows used >= y0 - 54)

  const float* img = OCT0 ? A.src + b * A.s_img : nullptr;
  const float* prev = OCT0 ? nullptr : A.src + b * A.s_img + A.src_off;
  float4 pre[2];
  const int Zbeg = y0 - kH, Zend = y1 + kH;
  if (OCT0) {
    // prologue: row-pass rows [Zbeg-4, Zbeg+4)
    fetch_image(A, img, x0, Zbeg - 4, pre);
    put_image(stage, pre);
    __syncthreads();
    hb_pass(stage, hb, K->base, Zbeg - 4);
    fetch_image(A, img, x0, Zbeg + 4, pre);
  } else {
    for (int c = t; c < kBW; c += 256) {
      const int x = x0 - kH + c;
      int sx = -1;
      if (x >= 0 && x < C) {
        sx = (int)floor(x * A.ifx);
        sx = sx < A.scols - 1 ? sx : A.scols - 1;
      }
      xmap[c] = sx;
    }
  }
  __syncthreads();

  const int ht = t & 127;
  const int hr = ht >> 4, hj = ht & 15;  // row-pass item: base row hr, columns [8hj, 8hj+8)
  const int x = x0 + ht;                 // column-pass item
  const bool colok = x < C;
  for (int Z = Zbeg; Z < Zend; Z += kRB) {
    // ---- base rows [Z, Z+8) ----
    if (OCT0) {
      put_image(stage, pre);
      __syncthreads();
      hb_pass(stage, hb, K->base, Z + 4);
      __syncthreads();
      if (t < kBW) {
        float win[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) win[k] = hb[((Z - 4 + k) & (kHbRows - 1)) * kBP + t];
        float acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
        for (int a = 0; a < 9; ++a) {
          const float k = K->base[a];
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] = __builtin_fmaf(win[i + a], k, acc[i]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) put_base(A, stage, plane0, i, t, Z + i, x0 - kH + t, y0, y1, acc[i]);
      }
    } else {
      for (int i = t; i < kRB * kBW; i += 256) {
        const int r = i / kBW, c = i - r * kBW;
        const int y = Z + r;
        const int sx = xmap[c];
        float v = 0.f;
        if (y >= 0 && y < R && sx >= 0) {
          int sy = (int)floor(y * A.ify);
          sy = sy < A.srows - 1 ? sy : A.srows - 1;
          v = prev[(long long)sy * A.s_pitch + sx];
        }
        put_base(A, stage, plane0, r, c, y, x0 - kH + c, y0, y1, v);
      }
    }
    __syncthreads();
    // ---- row passes: h rows [Z, Z+8) of every scale that still needs them ----
    {
      const int y = Z + hr;
      if (t < 128) {
        if (Z + kRB > y0 - 18 && Z < y1 + 18)
          row_pass<18>(stage, rings + kRing18 * kRP, K->s4, hr, hj, (y - rbase) % (kRB + 36));
        if (Z + kRB > y0 - 4 && Z < y1 + 4)
          row_pass<4>(stage, rings + kRing4 * kRP, K->s1, hr, hj, (y - rbase) % (kRB + 8));
      } else {
        if (Z + kRB > y0 - 12 && Z < y1 + 12)
          row_pass<12>(stage, rings + kRing12 * kRP, K->s3, hr, hj, (y - rbase) % (kRB + 24));
        if (Z + kRB > y0 - 8 && Z < y1 + 8)
          row_pass<8>(stage, rings + kRing8 * kRP, K->s2, hr, hj, (y - rbase) % (kRB + 16));
      }
    }
    __syncthreads();
    if (OCT0 && Z + kRB < Zend) fetch_image(A, img, x0, Z + kRB + 4, pre);  // next step's image rows
    // ---- column passes: plane rows [Z - w, Z - w + 8) ----
    if (t < 128) {
      if (Z - 18 + kRB > y0 && Z - 18 < y1)
        col_pass<18>(rings + kRing18 * kRP, K->s4, ht, (Z - 36 - rbase) % (kRB + 36), gimg + A.off[4] + x,
                     A.pitch, Z, y0, y1, colok);
      if (Z - 4 + kRB > y0 && Z - 4 < y1)
        col_pass<4>(rings + kRing4 * kRP, K->s1, ht, (Z - 8 - rbase) % (kRB + 8), gimg + A.off[1] + x,
                    A.pitch, Z, y0, y1, colok);
    } else {
      if (Z - 12 + kRB > y0 && Z - 12 < y1)
        col_pass<12>(rings + kRing12 * kRP, K->s3, ht, (Z - 24 - rbase) % (kRB + 24), gimg + A.off[3] + x,
                     A.pitch, Z, y0, y1, colok);
      if (Z - 8 + kRB > y0 && Z - 8 < y1)
        col_pass<8>(rings + kRing8 * kRP, K->s2, ht, (Z - 16 - rbase) % (kRB + 16), gimg + A.off[2] + x,
                    A.pitch, Z, y0, y1, colok);
    }
  }
}

// 1-D taps of sigma: g(a) = exp(-a^2 / (2 sigma^2)) / sqrt(2 pi sigma^2), the
// square root of the 2-D kernel's normalisation (src/sift.cpp:103, same
// float 2*sigma*sigma chain and PI).
void fast_taps(float sigma, float* g) {
  const int w = (int)floor(3 * sigma);
  const double den = (double)(2 * sigma * sigma);
  const double nrm = 1. / sqrt(2 * kRefPi * sigma * sigma);
  for (int a = -w; a <= w; ++a) g[a + w] = (float)(nrm * exp(-(a * a) * 1. / den));
}

}  // namespace

size_t fast_coefs_size() { return sizeof(FastCoefs); }

int fast_coefs_host(float sigma_base, const float* sig, void* out) {
  FastCoefs& F = *static_cast<FastCoefs*>(out);
  const int wb = (int)floor(3 * sigma_base);
  const int w[4] = {(int)floor(3 * sig[0]), (int)floor(3 * sig[1]), (int)floor(3 * sig[2]),
                    (int)floor(3 * sig[3])};
  if (wb != 4 || w[0] != 4 || w[1] != 8 || w[2] != 12 || w[3] != kH) return -1;
  fast_taps(sigma_base, F.base);
  fast_taps(sig[0], F.s1);
  fast_taps(sig[1], F.s2);
  fast_taps(sig[2], F.s3);
  fast_taps(sig[3], F.s4);
  return 0;
}

void launch_pyramid_fast(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch,
                         const void* coef) {
  const Octave& O = L.oct[o];
  FastArgs A{};
  A.gpyr = gpyr;
  A.g_img = L.g_img;
  for (int s = 0; s < kScales; ++s) A.off[s] = O.g_off[s];
  A.coef = static_cast<const FastCoefs*>(coef);
  A.pitch = O.pitch;
  A.rows = O.rows;
  A.cols = O.cols;
  if (o == 0) {
    A.src = src.p;
    A.src_off = 0;
    A.s_pitch = src.pitch;
    A.s_img = src.img_stride;
    A.vec = (src.pitch % 4 == 0 && src.img_stride % 4 == 0 &&
             (reinterpret_cast<uintptr_t>(src.p) & 15) == 0) ? 1 : 0;
  } else {
    const Octave& P = L.oct[o - 1];
    A.src = gpyr;
    A.src_off = P.g_off[kLayers];
    A.s_pitch = P.pitch;
    A.s_img = L.g_img;
    A.srows = P.rows;
    A.scols = P.cols;
    A.ifx = 1. / ((double)O.cols / P.cols);
    A.ify = 1. / ((double)O.rows / P.rows);
  }
  // Chunk the rows so the launch has ~1.5k workgroups (2 resident per CU),
  // but never below 48 rows (the 36-row halo is recomputed per chunk).
  const int strips = (O.cols + kFW - 1) / kFW;
  const long long per = (long long)strips * batch;
  int chunks = (int)((1536 + per - 1) / per);
  const int max_chunks = (O.rows + 47) / 48;
  chunks = chunks > max_chunks ? max_chunks : chunks;
  if (chunks < 1) chunks = 1;
  int ch = (O.rows + chunks - 1) / chunks;
  ch = (ch + kRB - 1) / kRB * kRB;
  chunks = (O.rows + ch - 1) / ch;
  A.chunk = ch;
  dim3 grid(strips, chunks, batch);
  if (o == 0)
    hipLaunchKernelGGL(pyr_fast_kernel<true>, grid, dim3(256), 0, st, A);
  else
    hipLaunchKernelGGL(pyr_fast_kernel<false>, grid, dim3(256), 0, st, A);
}

}  // namespace sift
