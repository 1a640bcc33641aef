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
//   scale s:   row pass of the base rows into a per-scale ring, column pass
//              out of the ring.
// A workgroup owns a 128-column strip and walks a chunk of rows 8 at a time,
// so every row pass is done once per row (the vertical halo is carried in the
// rings, not recomputed) and every source pixel is read from HBM once (plus
// an 18-column halo that hits L2).  Bound: HBM, 24 algorithmic bytes per pixel
// (one read, five plane writes) against ~180 FMA per pixel.
//
// Latency structure (what the profile showed mattered):
//  * the next step's source rows are loaded into registers while the current
//    step computes, and every load is branch-free (clamped address + select);
//  * plane stores go through a buffer resource: an invalid position gets an
//    out-of-range offset and the hardware drops the store, so each step issues
//    a fixed number of stores.  hipcc can then wait for the prefetch with
//    vmcnt(N) instead of vmcnt(0), and the stores stay in flight across the
//    step boundary (with data-dependent store counts every step waited for
//    all of its stores to reach memory: 40% of the kernel time);
//  * the taps are kernel arguments (scalar cache), not VMEM loads;
//  * steps start on a multiple of 8 and every ring holds a multiple of 8
//    rows, so a column pass starts at one of M/8 ring slots and each start is
//    its own unrolled body with compile-time LDS offsets.
#include "common.hpp"

#include <math.h>
#include <stdlib.h>

namespace sift {

namespace {

constexpr int kFW = 128;               // output columns per strip
constexpr int kRB = 8;                 // rows per step
constexpr int kH = 18;                 // widest scale half-width (sig[4] = 6.197)
constexpr int kLead = 24;              // base rows computed above the chunk (>= kH, multiple of 8)
constexpr int kBW = kFW + 2 * kH;      // 164 base columns per strip
constexpr int kBP = 172;               // base / row-pass ring pitch (== 4 mod 8)
constexpr int kIP = 180;               // image staging pitch (176 columns used)
constexpr int kIQ = 44;                // float4 per staged image row
constexpr int kRP = 132;               // scale ring pitch (== 4 mod 8)
constexpr int kHbRows = 16;            // octave-0 row-pass ring: rows [Z-4, Z+12)
constexpr int kStage = kRB * kIP;      // staged image rows / base rows (aliased)
constexpr int kGather = (kRB * kBW + 255) / 256;  // decimation gathers per lane per step
constexpr int kDrop = 0x7ffffff0;      // buffer offset past every plane: the store is dropped

// Scale ring of half-width W: M = round_up(8 + 2W, 8) rows at row offset off.
template <int W> struct Ring;
template <> struct Ring<4> { static constexpr int off = 0, M = 16; };
template <> struct Ring<8> { static constexpr int off = 16, M = 24; };
template <> struct Ring<12> { static constexpr int off = 40, M = 32; };
template <> struct Ring<18> { static constexpr int off = 72, M = 48; };
constexpr int kRingRows = 120;

constexpr int kLds0 = kStage + kHbRows * kBP + kRingRows * kRP;   // floats, octave 0
constexpr int kLdsN = kStage + kRingRows * kRP + kBW;             // floats (+ column map), octave > 0
static_assert(kRB * kBP <= kStage, "base rows alias the image staging rows");
static_assert(kBP % 8 == 4 && kRP % 8 == 4 && kIP % 4 == 0, "b128 row pitches");
static_assert(kLds0 % 4 == 0 && kLdsN % 4 == 0 && kStage % 4 == 0 && (kHbRows * kBP) % 4 == 0,
              "float4 LDS regions");
static_assert(2 * kLds0 * 4 <= 160 * 1024, "two workgroups per CU");

typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc plane_rsrc(float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void st_plane(Rsrc rs, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, off, 0, 0);
}

// LDS pointers are float4 arrays indexed in float4 units, so every address is
// provably 16-byte aligned and hipcc emits ds_read_b128 / ds_write_b128.
//
// Row pass of one scale: h[Z + r][8j + p] = sum_b g[b] base[r][8j + p + 18 - W + b].
// The 16-lane groups of a ds_read_b128 hold two whole base rows x 8 column
// groups; with kBP == 4 (mod 8) their 16-byte slots are distinct (conflict free).
template <int W>
__device__ __forceinline__ void row_pass(const float4* __restrict__ bs4, float4* __restrict__ rings4,
                                         const float* __restrict__ g, int r, int j, int slot) {
  constexpr int ST = (kH - W) & ~3, E = (kH - W) & 3;
  constexpr int L = (E + kRB + 2 * W + 3) & ~3;
  float win[L];
  const float4* src = bs4 + r * (kBP / 4) + 2 * j + ST / 4;
#pragma unroll
  for (int q = 0; q < L / 4; ++q) {
    const float4 t = src[q];
    win[4 * q] = t.x;
    win[4 * q + 1] = t.y;
    win[4 * q + 2] = t.z;
    win[4 * q + 3] = t.w;
  }
  // Keep the whole 16-byte loads: hipcc trims unused leading / trailing floats
  // and then falls back to 8-byte-aligned ds_read2_b64 (4-way bank conflicts).
#pragma unroll
  for (int k = 0; k < L; ++k)
    if (k < E || k >= E + kRB + 2 * W) asm volatile("" ::"v"(win[k]));
  float acc[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) acc[p] = 0.f;
#pragma unroll
  for (int b = 0; b <= 2 * W; ++b) {
    const float k = g[b];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = __builtin_fmaf(win[E + p + b], k, acc[p]);
  }
  // ds_write_b128 serves 8 lanes (8 x 16 B = 32 banks) per cycle: lanes j and
  // j + 4 would collide at stride 32 B, so the upper half-group writes its two
  // halves in the other order.
  float4* dst = rings4 + (Ring<W>::off + slot) * (kRP / 4) + 2 * j;
  const float4 lo = make_float4(acc[0], acc[1], acc[2], acc[3]);
  const float4 hi = make_float4(acc[4], acc[5], acc[6], acc[7]);
  if (j & 4) {
    dst[1] = hi;
    dst[0] = lo;
  } else {
    dst[0] = lo;
    dst[1] = hi;
  }
}

// Column pass of one scale starting at ring slot S0: rows [Z - W, Z - W + 8)
// of the plane, column x, from ring rows [Z - 2W, Z + 8).  Always stores 8
// values; rows outside [y0, y1) and columns past the image are dropped.
template <int W, int S0>
__device__ __forceinline__ void col_fixed(const float* __restrict__ rings, const float* __restrict__ g,
                                          int col, Rsrc rs, int pitch, int x, int Z, int y0, int y1,
                                          bool colok) {
  constexpr int M = Ring<W>::M, N = kRB + 2 * W;
  const float* ring = rings + Ring<W>::off * kRP + col;
  float win[N];
#pragma unroll
  for (int k = 0; k < N; ++k) win[k] = ring[((S0 + k) % M) * kRP];
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
  for (int a = 0; a <= 2 * W; ++a) {
    const float k = g[a];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_fmaf(win[i + a], k, acc[i]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int y = Z - W + i;
    st_plane(rs, (colok && y >= y0 && y < y1) ? (y * pitch + x) * 4 : kDrop, acc[i]);
  }
}

// Start slot s0 = 8c + R0 (R0 = -2W mod 8): uniform dispatch to the body for c.
template <int W, int C>
__device__ __forceinline__ void col_pass(int c, const float* __restrict__ rings, const float* __restrict__ g,
                                         int col, Rsrc rs, int pitch, int x, int Z, int y0, int y1,
                                         bool colok) {
  constexpr int R0 = (8 - (2 * W) % 8) % 8;
  if constexpr (C + 1 < Ring<W>::M / 8) {
    if (c == C)
      col_fixed<W, 8 * C + R0>(rings, g, col, rs, pitch, x, Z, y0, y1, colok);
    else
      col_pass<W, C + 1>(c, rings, g, col, rs, pitch, x, Z, y0, y1, colok);
  } else {
    col_fixed<W, 8 * C + R0>(rings, g, col, rs, pitch, x, Z, y0, y1, colok);
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
  double ify, ifx;         // resize NN scale factors (octave > 0)
  int pitch, rows, cols;
  int srows, scols;        // source (previous octave) shape
  int chunk;               // rows per workgroup (multiple of kRB)
  int ablate;              // diagnostic only (SIFT_FAST_ABLATE): 4 skips the row passes
  // By value: kernel arguments are constant memory, so the taps come through
  // the scalar cache.  Through a pointer the compiler cannot rule out that the
  // plane stores alias them and reloads every tap with a VMEM load per pass.
  FastCoefs coef;
};

namespace {

// Octave-0 image rows [Y, Y+8) x columns [x0-24, x0+152) -> 2 float4 per lane
// (lanes >= 96 hold one), loaded from clamped addresses with no branch and no
// use: the padding select happens in put_image, a step later, so the loads
// stay in flight.  VEC: rows are 16-byte aligned with a pitch that is a
// multiple of 4 (>= cols), so a float4 at a clamped x never leaves the row.
template <bool VEC>
__device__ __forceinline__ void fetch_image(const FastArgs& A, const float* __restrict__ img, int x0,
                                            int Y, float4 (&v)[2]) {
  const int lim = A.cols - 1;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int r = i / kIQ, q = i - r * kIQ;
    const int y = Y + r, x = x0 - 24 + 4 * q;
    const float* row = img + (long long)min(max(y, 0), A.rows - 1) * A.s_pitch;
    if (VEC) {
      v[u] = *reinterpret_cast<const float4*>(row + min(max(x, 0), (int)A.s_pitch - 4));
    } else {
      v[u].x = row[min(max(x, 0), lim)];
      v[u].y = row[min(max(x + 1, 0), lim)];
      v[u].z = row[min(max(x + 2, 0), lim)];
      v[u].w = row[min(max(x + 3, 0), lim)];
    }
  }
}

// Writes the fetched rows [Y, Y+8) to the staging rows with the source padding
// of the base blur: 0 outside [0, rows-1) x [0, cols-1).
__device__ __forceinline__ void put_image(const FastArgs& A, float4* __restrict__ stage4, const float4 (&v)[2],
                                          int x0, int Y) {
  const int lim = A.cols - 1;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < kRB * kIQ) {
      const int r = i / kIQ, q = i - r * kIQ;
      const int y = Y + r, x = x0 - 24 + 4 * q;
      const bool rowok = y >= 0 && y < A.rows - 1;
      float4 w;
      w.x = (rowok && x >= 0 && x < lim) ? v[u].x : 0.f;
      w.y = (rowok && x + 1 >= 0 && x + 1 < lim) ? v[u].y : 0.f;
      w.z = (rowok && x + 2 >= 0 && x + 2 < lim) ? v[u].z : 0.f;
      w.w = (rowok && x + 3 >= 0 && x + 3 < lim) ? v[u].w : 0.f;
      stage4[r * (kIP / 4) + q] = w;
    }
  }
}

// Octave > 0: the INTER_NEAREST source values of base rows [Z, Z+8) (source
// row min(floor(y * ify), srows-1), column map in LDS), branch-free loads.
__device__ __forceinline__ void fetch_decim(const FastArgs& A, const float* __restrict__ prev,
                                            const int* __restrict__ xmap, int Z, float (&v)[kGather]) {
#pragma unroll
  for (int u = 0; u < kGather; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int r = i / kBW, c = i - r * kBW;
    const int y = Z + r;
    const int sx = xmap[i < kRB * kBW ? c : 0];
    const bool ok = i < kRB * kBW && y >= 0 && y < A.rows && sx >= 0;
    int sy = (int)floor(max(y, 0) * A.ify);
    sy = sy < A.srows - 1 ? sy : A.srows - 1;
    v[u] = prev[ok ? (long long)sy * A.s_pitch + sx : 0];
  }
}

// Octave-0 row pass of the base blur: ring rows [Y, Y+8), base columns
// [0, 168) (column c <-> image column x0 - 18 + c; 164 are used).
__device__ __forceinline__ void hb_pass(const float4* __restrict__ stage4, float4* __restrict__ hb4,
                                        const float* __restrict__ g, int Y) {
  const int t = threadIdx.x;
  if (t >= kRB * 21) return;
  const int r = t / 21, j = t - r * 21;
  float win[20];
  const float4* src = stage4 + r * (kIP / 4) + 2 * j;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const float4 v = src[q];
    win[4 * q] = v.x;
    win[4 * q + 1] = v.y;
    win[4 * q + 2] = v.z;
    win[4 * q + 3] = v.w;
  }
  asm volatile("" ::"v"(win[0]), "v"(win[1]), "v"(win[18]), "v"(win[19]));  // see row_pass
  float acc[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) acc[p] = 0.f;
#pragma unroll
  for (int b = 0; b < 9; ++b) {
    const float k = g[b];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = __builtin_fmaf(win[p + b + 2], k, acc[p]);
  }
  float4* dst = hb4 + ((Y + r) & (kHbRows - 1)) * (kBP / 4) + 2 * j;
  dst[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  dst[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// Stores one base value: the plane-0 interior (unpadded) to HBM and the
// padded copy (0 outside [0, rows-1) x [0, cols-1)) as the scales' source.
__device__ __forceinline__ void put_base(const FastArgs& A, float* __restrict__ bs, Rsrc rs0, int r, int c,
                                         int y, int x, int y0, int y1, float v) {
  const bool out = c >= kH && c < kH + kFW && x < A.cols && y >= y0 && y < y1;
  st_plane(rs0, out ? (y * A.pitch + x) * 4 : kDrop, v);
  const bool src_ok = y >= 0 && y < A.rows - 1 && x >= 0 && x < A.cols - 1;
  bs[r * kBP + c] = src_ok ? v : 0.f;
}

// Octave-0 column pass of the base blur for base rows [Z, Z+8), from row-pass
// ring rows [Z-4, Z+12) starting at slot S0 = (Z - 4) & 15.
template <int S0>
__device__ __forceinline__ void base_col(const FastArgs& A, const float* __restrict__ hb, float* __restrict__ bs,
                                         Rsrc rs0, int t, int Z, int x0, int y0, int y1) {
  float win[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) win[k] = hb[((S0 + k) & (kHbRows - 1)) * kBP + t];
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    const float k = A.coef.base[a];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_fmaf(win[i + a], k, acc[i]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) put_base(A, bs, rs0, i, t, Z + i, x0 - kH + t, y0, y1, acc[i]);
}

template <bool OCT0, bool VEC>
__global__ __launch_bounds__(256, 2) void pyr_fast_kernel(FastArgs A) {
  __shared__ float4 lds4[(OCT0 ? kLds0 : kLdsN) / 4];
  float* const lds = reinterpret_cast<float*>(lds4);
  float* const stage = lds;
  float4* const stage4 = lds4;
  float* const hb = lds + kStage;  // octave 0 only
  float4* const hb4 = lds4 + kStage / 4;
  float4* const rings4 = lds4 + (kStage + (OCT0 ? kHbRows * kBP : 0)) / 4;
  float* const rings = reinterpret_cast<float*>(rings4);
  int* const xmap = reinterpret_cast<int*>(rings + kRingRows * kRP);  // octave > 0 only

  const int t = threadIdx.x;
  const int b = blockIdx.z;
  const int x0 = blockIdx.x * kFW;
  const int y0 = blockIdx.y * A.chunk;
  const int y1 = min(y0 + A.chunk, A.rows);
  const int C = A.cols;
  float* const gimg = A.gpyr + b * A.g_img;
  const long long plane_bytes = (long long)A.rows * A.pitch * 4;
  const Rsrc rs0 = plane_rsrc(gimg + A.off[0], plane_bytes);
  const FastCoefs& K = A.coef;
  const int rbase = y0 - 64;  // ring slot of row y: (y - rbase) mod M; rows used >= y0 - 60

  const float* img = OCT0 ? A.src + b * A.s_img : nullptr;
  const float* prev = OCT0 ? nullptr : A.src + b * A.s_img + A.src_off;
  float4 pre[2];
  float gv[kGather];
  const int Zbeg = y0 - kLead, Zend = y1 + kH;
  if (OCT0) {
    // prologue: row-pass rows [Zbeg-4, Zbeg+4)
    fetch_image<VEC>(A, img, x0, Zbeg - 4, pre);
    put_image(A, stage4, pre, x0, Zbeg - 4);
    __syncthreads();
    hb_pass(stage4, hb4, K.base, Zbeg - 4);
    fetch_image<VEC>(A, img, x0, Zbeg + 4, pre);
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
    __syncthreads();
    fetch_decim(A, prev, xmap, Zbeg, gv);
  }
  // 16 dropped stores: the loop enters with as many VMEM ops behind the
  // prefetch as a step's column passes leave, so hipcc's wait for it at the
  // top of the loop is vmcnt(16+) on every path instead of vmcnt(0).
#pragma unroll
  for (int k = 0; k < 16; ++k) st_plane(rs0, kDrop, 0.f);
  __syncthreads();

  const int ht = t & 127;
  const int hr = ht >> 4, hj = ht & 15;  // row-pass item: base row hr, columns [8hj, 8hj+8)
  const int x = x0 + ht;                 // column-pass item
  const bool colok = x < C;
  for (int Z = Zbeg; Z < Zend; Z += kRB) {
    // ---- base rows [Z, Z+8) ----
    if (OCT0) {
      put_image(A, stage4, pre, x0, Z + 4);
      __syncthreads();
      hb_pass(stage4, hb4, K.base, Z + 4);
      __syncthreads();
      if (t < kBW) {
        if (Z & 8)
          base_col<4>(A, hb, stage, rs0, t, Z, x0, y0, y1);
        else
          base_col<12>(A, hb, stage, rs0, t, Z, x0, y0, y1);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kGather; ++u) {
        const int i = t + 256 * u;
        if (i < kRB * kBW) {
          const int r = i / kBW, c = i - r * kBW;
          const int y = Z + r;
          const bool ok = y >= 0 && y < A.rows && xmap[c] >= 0;
          put_base(A, stage, rs0, r, c, y, x0 - kH + c, y0, y1, ok ? gv[u] : 0.f);
        }
      }
    }
    __syncthreads();
    // next step's source rows, in flight during this step's passes
    if (Z + kRB < Zend) {
      if (OCT0)
        fetch_image<VEC>(A, img, x0, Z + kRB + 4, pre);
      else
        fetch_decim(A, prev, xmap, Z + kRB, gv);
    }
    // ---- row passes: h rows [Z, Z+8) -> ring slots [(Z - rbase) mod M, +8) ----
    if (!(A.ablate & 4)) {
      if (t < 128) {
        if (Z + kRB > y0 - 18 && Z < y1 + 18)
          row_pass<18>(stage4, rings4, K.s4, hr, hj, (Z - rbase) % Ring<18>::M + hr);
        if (Z + kRB > y0 - 4 && Z < y1 + 4)
          row_pass<4>(stage4, rings4, K.s1, hr, hj, (Z - rbase) % Ring<4>::M + hr);
      } else {
        if (Z + kRB > y0 - 12 && Z < y1 + 12)
          row_pass<12>(stage4, rings4, K.s3, hr, hj, (Z - rbase) % Ring<12>::M + hr);
        if (Z + kRB > y0 - 8 && Z < y1 + 8)
          row_pass<8>(stage4, rings4, K.s2, hr, hj, (Z - rbase) % Ring<8>::M + hr);
      }
    }
    __syncthreads();
    // ---- column passes: plane rows [Z - w, Z - w + 8), every step (fixed store count) ----
    if (t < 128) {
      col_pass<18, 0>(((Z - 36 - rbase) % Ring<18>::M) >> 3, rings, K.s4, ht,
                      plane_rsrc(gimg + A.off[4], plane_bytes), A.pitch, x, Z, y0, y1, colok);
      col_pass<4, 0>(((Z - 8 - rbase) % Ring<4>::M) >> 3, rings, K.s1, ht,
                     plane_rsrc(gimg + A.off[1], plane_bytes), A.pitch, x, Z, y0, y1, colok);
    } else {
      col_pass<12, 0>(((Z - 24 - rbase) % Ring<12>::M) >> 3, rings, K.s3, ht,
                      plane_rsrc(gimg + A.off[3], plane_bytes), A.pitch, x, Z, y0, y1, colok);
      col_pass<8, 0>(((Z - 16 - rbase) % Ring<8>::M) >> 3, rings, K.s2, ht,
                     plane_rsrc(gimg + A.off[2], plane_bytes), A.pitch, x, Z, y0, y1, colok);
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

// coef: the host-side FastCoefs block from fast_coefs_host (copied into the
// kernel arguments).
void launch_pyramid_fast(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch,
                         const void* coef) {
  const Octave& O = L.oct[o];
  FastArgs A{};
  A.gpyr = gpyr;
  A.g_img = L.g_img;
  for (int s = 0; s < kScales; ++s) A.off[s] = O.g_off[s];
  A.coef = *static_cast<const FastCoefs*>(coef);
  A.pitch = O.pitch;
  A.rows = O.rows;
  A.cols = O.cols;
  bool vec = false;
  if (o == 0) {
    A.src = src.p;
    A.src_off = 0;
    A.s_pitch = src.pitch;
    A.s_img = src.img_stride;
    vec = src.pitch % 4 == 0 && src.img_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(src.p) & 15) == 0;
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
  // but never below 48 rows (the 42-row lead is recomputed per chunk).
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
  static const int ablate = getenv("SIFT_FAST_ABLATE") ? atoi(getenv("SIFT_FAST_ABLATE")) : 0;
  A.ablate = ablate;
  dim3 grid(strips, chunks, batch);
  if (o > 0)
    hipLaunchKernelGGL((pyr_fast_kernel<false, false>), grid, dim3(256), 0, st, A);
  else if (vec)
    hipLaunchKernelGGL((pyr_fast_kernel<true, true>), grid, dim3(256), 0, st, A);
  else
    hipLaunchKernelGGL((pyr_fast_kernel<true, false>), grid, dim3(256), 0, st, A);
}

}  // namespace sift
