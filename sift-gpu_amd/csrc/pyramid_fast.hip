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
// (one read, five plane writes) against ~194 FMA per pixel.
//
// What the profile showed mattered:
//  * FMA issue.  Every FMA stream is written on pairs (v_pk_fma_f32: twice
//    the rate of v_fma_f32 from one or two waves per SIMD, measured by
//    tools/ubench_fma.hip), with both operands of every pair in aligned
//    registers straight from LDS: row passes pair two rows (the base / image
//    rows are staged row-pair interleaved, so one ds_read_b128 yields two
//    columns of two rows), column passes pair two columns (ds_read_b64);
//  * the taps sit in VGPRs for the whole walk, one per tap (pk_tap);
//  * the next step's source rows are loaded during the column passes with
//    loads hipcc does not track and waited for with an explicit vmcnt (see
//    ld2_async); every load is branch-free (clamped address, the padding
//    select happens when the values are staged);
//  * plane stores go through a buffer resource: an invalid position gets an
//    out-of-range offset and the hardware drops the store, so each wave
//    issues a fixed number of stores per step and the wait for the prefetch
//    can leave them in flight;
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
constexpr int kIW = 176;               // staged image columns [x0-24, x0+152)
constexpr int kSP = 356;               // staged image row-pair pitch (floats; 2 x 176 + 4)
constexpr int kBP2 = 332;              // base row-pair pitch (floats; 2 x 164 + 4, == 4 mod 8)
constexpr int kBP = 172;               // octave-0 row-pass ring pitch (168 columns used)
constexpr int kRP = 132;               // scale ring pitch (== 4 mod 8)
constexpr int kHbRows = 16;            // octave-0 row-pass ring: rows [Z-4, Z+12)
constexpr int kStage = 4 * kSP;        // staged image row pairs / base row pairs (aliased)
constexpr int kImgUnits = 4 * (kIW / 2);          // 2 rows x 2 columns per unit: 352 per step
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
static_assert(4 * kBP2 <= kStage, "base row pairs alias the image staging rows");
static_assert(kSP % 4 == 0 && kBP2 % 8 == 4 && kBP % 4 == 0 && kRP % 8 == 4, "b128 row pitches");
static_assert(kLds0 % 4 == 0 && kLdsN % 4 == 0 && kStage % 4 == 0 && (kHbRows * kBP) % 4 == 0,
              "float4 LDS regions");
static_assert(2 * kLds0 * 4 <= 160 * 1024, "two workgroups per CU");
static_assert(kGather == 6, "SIFT_VM_WAIT operand list");

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ Rsrc plane_rsrc(float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void st_plane(Rsrc rs, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, off, 0, 0);
}

__device__ __forceinline__ void st_plane2(Rsrc rs, int off, f2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rs, off, 0, 0);
}

// Window reads of the column passes.  hipcc pairs two ds_read_b64 off one
// base register that are < 2 KB apart into a ds_read2_b64, which moves half as
// many bytes per LDS cycle (8 cycles for 2 x 8 B per lane against 2 x 2).  The
// window rows are read off four opaque copies of the base, row k off copy
// k & 3: rows on one copy are >= 4 ring rows (> 2 KB) apart, so no pair forms.
typedef const __attribute__((address_space(3))) f2* LdsF2;

template <int NB>
__device__ __forceinline__ void lds_bases(const f2* p, LdsF2 (&b)[NB]) {
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    b[i] = (LdsF2)p;
    asm volatile("" : "+v"(b[i]));
  }
}


__device__ __forceinline__ f2 splat(float k) { return f2{k, k}; }

// acc + a * g_b with the taps held in VGPRs as pairs g[j] = (g_2j, g_2j+1):
// op_sel picks tap b out of its pair for both halves, so a tap costs one VGPR
// and no copy.  (As SGPR operands all 97 taps spilled; loaded per pass from
// the argument segment, the scalar loads made every pass wait lgkmcnt(0) for
// its whole LDS window; as (k, k) pairs in LDS the broadcast reads doubled
// the LDS cycles.)  The FMA loops below issue 4 or 8 independent chains, so
// dependent pk_fma are never adjacent.
__device__ __forceinline__ f2 pk_tap(f2 a, const f2* g, int b, f2 c) {
  f2 d;
  if (b & 1)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(d) : "v"(a), "v"(g[b >> 1]), "v"(c));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "v"(g[b >> 1]), "v"(c));
  return d;
}

// Taps of half-width W as VGPR pairs (see pk_tap).
template <int W>
__device__ __forceinline__ void tap_pairs(const __attribute__((address_space(4))) float* k, f2 (&g)[W + 1]) {
#pragma unroll
  for (int j = 0; j <= W; ++j) {
    g[j] = f2{k[2 * j], 2 * j + 1 <= 2 * W ? k[2 * j + 1] : 0.f};
    asm volatile("" : "+v"(g[j]));
  }
}

// Row pass of one scale for base rows (2s, 2s+1) and output columns
// [4j, 4j+4): h[Z + 2s + e][4j + i] = sum_b g[b] base[2s + e][4j + i + 18 - W + b].
// The base rows are staged row-pair interleaved (bs2[s][c] = (row 2s, row
// 2s+1) at column c), so each pk_fma operand is an aligned register pair of a
// ds_read_b128.  Lane -> (s, j) puts two row pairs x 8 column groups in each
// 16-lane group of a ds_read_b128; with kBP2 == 4 (mod 8) their 16-byte slots
// are distinct (conflict free).  The two output rows are written with
// ds_write_b128 (8 contiguous lanes per group: conflict free).
template <int W>
__device__ __forceinline__ void row_pass(const float4* __restrict__ bs4, float4* __restrict__ rings4, const f2* g,
                                         int s, int j, int slot) {
  constexpr int C0 = kH - W, NW = 4 + 2 * W;
  static_assert(C0 % 2 == 0 && NW % 2 == 0, "windows start on a column pair");
  const float4* src = bs4 + s * (kBP2 / 4) + 2 * j + C0 / 2;
  f2 w[NW];
#pragma unroll
  for (int q = 0; q < NW / 2; ++q) {
    const float4 v = src[q];
    w[2 * q] = f2{v.x, v.y};
    w[2 * q + 1] = f2{v.z, v.w};
  }
  f2 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = splat(0.f);
#pragma unroll
  for (int b = 0; b <= 2 * W; ++b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = pk_tap(w[i + b], g, b, acc[i]);
  }
  // slot + 1 never wraps: slot = (Z - rbase) mod M + 2s with Z - rbase and M
  // multiples of 8.
  float4* dst = rings4 + (Ring<W>::off + slot) * (kRP / 4) + j;
  dst[0] = make_float4(acc[0].x, acc[1].x, acc[2].x, acc[3].x);
  dst[kRP / 4] = make_float4(acc[0].y, acc[1].y, acc[2].y, acc[3].y);
}

// Column pass of one scale, two columns per lane: plane rows [Y, Y + NR),
// columns x, x+1, from ring rows [Y - W, Y + NR + W) starting at ring slot S0
// (ds_read_b64: 32 contiguous lanes per group, conflict free).  Always issues
// NR (8-byte) stores; rows outside [y0, y1) and column pairs past the image
// are dropped (a pair that straddles an odd image width also writes the pitch
// padding column, which nothing reads).
template <int W, int S0, int NR>
__device__ __forceinline__ void col_fixed(const float* __restrict__ rings, const f2* g, int lane, Rsrc rs, int pitch,
                                          int x, int Y, int y0, int y1, bool colok) {
  constexpr int M = Ring<W>::M, N = NR + 2 * W;
  LdsF2 ring[4];
  lds_bases(reinterpret_cast<const f2*>(rings + Ring<W>::off * kRP) + lane, ring);
  f2 win[N];
#pragma unroll
  for (int k = 0; k < N; ++k) win[k] = ring[k & 3][((S0 + k) % M) * (kRP / 2)];
  f2 acc[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) acc[i] = splat(0.f);
#pragma unroll
  for (int a = 0; a <= 2 * W; ++a) {
#pragma unroll
    for (int i = 0; i < NR; ++i) acc[i] = pk_tap(win[i + a], g, a, acc[i]);
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int y = Y + i;
    st_plane2(rs, (colok && y >= y0 && y < y1) ? (y * pitch + x) * 4 : kDrop, acc[i]);
  }
  // A distinct tail per body: otherwise hipcc sinks the (identical) FMA and
  // store code of the M/8 bodies into one and moves every window into it with
  // v_mov -- N extra VALU per pass, and the compile-time offsets lost.
  asm volatile("; col_fixed %0 %1 %2" ::"n"(W), "n"(S0), "n"(NR));
}

// Rows [Z - W + R, +NR) of the plane.  Their window starts at ring slot
// s0 = (Z - 2W + R - rbase) mod M = 8c + R0 with R0 = (R - 2W) mod 8 (steps
// and rbase are multiples of 8): uniform dispatch to the body for c.
template <int W, int NR, int R, int C>
__device__ __forceinline__ void col_pass(int c, const float* __restrict__ rings, const f2* g, int lane, Rsrc rs,
                                         int pitch, int x, int Z, int y0, int y1, bool colok) {
  constexpr int R0 = (((R - 2 * W) % 8) + 8) % 8;
  if constexpr (C + 1 < Ring<W>::M / 8) {
    if (c == C)
      col_fixed<W, 8 * C + R0, NR>(rings, g, lane, rs, pitch, x, Z - W + R, y0, y1, colok);
    else
      col_pass<W, NR, R, C + 1>(c, rings, g, lane, rs, pitch, x, Z, y0, y1, colok);
  } else {
    col_fixed<W, 8 * C + R0, NR>(rings, g, lane, rs, pitch, x, Z - W + R, y0, y1, colok);
  }
}

template <int W, int R>
__device__ __forceinline__ int col_slot(int Z, int rbase) {
  return ((Z - 2 * W + R - rbase) % Ring<W>::M) >> 3;
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
  int ify2;                // octave > 0 and srows == 2 * rows: ify is exactly 2
  FastCoefs coef;          // by value: scalar loads from the argument segment
};

namespace {

typedef const __attribute__((address_space(4))) FastArgs* KArgs;  // A in the argument segment

// Source prefetch with loads the compiler does not track (inline asm).  With
// ordinary loads hipcc counted VMEM operations conservatively across the
// column passes' branches and waited for most of a step's plane stores to
// reach memory before it let a prefetched value be used.  Here the loads are
// issued right before the column passes and waited for right after them with
// vmcnt(n) -- n = the stores this wave's column passes issue (fixed per wave)
// and VMEM operations retire in order -- so the stores stay in flight into the
// next step.  The destination registers are operands of the wait, so nothing
// reads them before it.
__device__ __forceinline__ f2 ld2_async(const float* p) {
  f2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}

__device__ __forceinline__ float ld1_async(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}

struct Pre {         // one step's prefetched source values
  f2 v[4];           // octave 0, 8-byte rows: units (t, t+256) x rows (2s, 2s+1)
  float s[8];        // octave 0, unaligned rows: the same, element by element
  float g[kGather];  // octave > 0
};

#define SIFT_VM_WAIT(CNT)                                                                                  \
  do {                                                                                                     \
    if constexpr (OCT0 && VEC) {                                                                           \
      asm volatile("s_waitcnt vmcnt(" #CNT ")"                                                             \
                   : "+v"(P.v[0]), "+v"(P.v[1]), "+v"(P.v[2]), "+v"(P.v[3])::"memory");                    \
    } else if constexpr (OCT0) {                                                                           \
      asm volatile("s_waitcnt vmcnt(" #CNT ")"                                                             \
                   : "+v"(P.s[0]), "+v"(P.s[1]), "+v"(P.s[2]), "+v"(P.s[3]), "+v"(P.s[4]), "+v"(P.s[5]),   \
                     "+v"(P.s[6]), "+v"(P.s[7])::"memory");                                                \
    } else {                                                                                               \
      asm volatile("s_waitcnt vmcnt(" #CNT ")"                                                             \
                   : "+v"(P.g[0]), "+v"(P.g[1]), "+v"(P.g[2]), "+v"(P.g[3]), "+v"(P.g[4]),                 \
                     "+v"(P.g[5])::"memory");                                                              \
    }                                                                                                      \
  } while (0)

// Octave-0 image rows [Y, Y+8) x columns [x0-24, x0+152) in units of 2 rows x
// 2 columns (unit i: row pair s = i / 88, column pair q = i % 88); lanes hold
// units t and t + 256 (< 352), from clamped addresses.  VEC: rows are 16-byte
// aligned with a pitch that is a multiple of 4 (>= cols), so a float2 at a
// clamped even x never leaves the row.
template <bool VEC>
__device__ __forceinline__ void fetch_image(const FastArgs& A, const float* __restrict__ img, int x0, int Y,
                                            Pre& P) {
  const int lim = A.cols - 1;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int s = i / (kIW / 2), q = i - s * (kIW / 2);
    const int y = Y + 2 * s, x = x0 - 24 + 2 * q;
    const float* r0 = img + (long long)min(max(y, 0), A.rows - 1) * A.s_pitch;
    const float* r1 = img + (long long)min(max(y + 1, 0), A.rows - 1) * A.s_pitch;
    if (VEC) {
      const int xv = min(max(x, 0), (int)A.s_pitch - 2);
      P.v[2 * u] = ld2_async(r0 + xv);
      P.v[2 * u + 1] = ld2_async(r1 + xv);
    } else {
      const int xa = min(max(x, 0), lim), xb = min(max(x + 1, 0), lim);
      P.s[4 * u] = ld1_async(r0 + xa);
      P.s[4 * u + 1] = ld1_async(r0 + xb);
      P.s[4 * u + 2] = ld1_async(r1 + xa);
      P.s[4 * u + 3] = ld1_async(r1 + xb);
    }
  }
}

// Stages the fetched units row-pair interleaved, (r0 c, r1 c, r0 c+1, r1 c+1),
// with the source padding of the base blur: 0 outside [0, rows-1) x [0, cols-1).
template <bool VEC>
__device__ __forceinline__ void put_image(const FastArgs& A, float4* __restrict__ stage4, const Pre& P, int x0,
                                          int Y) {
  const int lim = A.cols - 1;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < kImgUnits) {
      const int s = i / (kIW / 2), q = i - s * (kIW / 2);
      const int y = Y + 2 * s, x = x0 - 24 + 2 * q;
      const bool ok0 = y >= 0 && y < A.rows - 1, ok1 = y + 1 >= 0 && y + 1 < A.rows - 1;
      const bool oka = x >= 0 && x < lim, okb = x + 1 >= 0 && x + 1 < lim;
      const float a0 = VEC ? P.v[2 * u].x : P.s[4 * u], b0 = VEC ? P.v[2 * u].y : P.s[4 * u + 1];
      const float a1 = VEC ? P.v[2 * u + 1].x : P.s[4 * u + 2], b1 = VEC ? P.v[2 * u + 1].y : P.s[4 * u + 3];
      stage4[s * (kSP / 4) + q] = make_float4((ok0 && oka) ? a0 : 0.f, (ok1 && oka) ? a1 : 0.f,
                                              (ok0 && okb) ? b0 : 0.f, (ok1 && okb) ? b1 : 0.f);
    }
  }
}

// Octave > 0: the INTER_NEAREST source values of base rows [Z, Z+8) (source
// row min(floor(y * ify), srows-1), column map in LDS), clamped addresses.
__device__ __forceinline__ void fetch_decim(const FastArgs& A, const float* __restrict__ prev,
                                            const int* __restrict__ xmap, int Z, Pre& P) {
#pragma unroll
  for (int u = 0; u < kGather; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int r = i / kBW, c = i - r * kBW;
    const int y = Z + r;
    const int sx = xmap[i < kRB * kBW ? c : 0];
    const bool ok = i < kRB * kBW && y >= 0 && y < A.rows && sx >= 0;
    // resize NN row map; exactly 2y when the source has twice the rows
    // (ify == 2.0 then, and floor(2y) needs no double arithmetic)
    int sy = A.ify2 ? 2 * max(y, 0) : (int)floor(max(y, 0) * A.ify);
    sy = sy < A.srows - 1 ? sy : A.srows - 1;
    P.g[u] = ld1_async(prev + (ok ? (long long)sy * A.s_pitch + sx : 0));
  }
}

// Octave > 0: base rows [Z, Z+8) from the prefetched decimation values: the
// plane-0 interior (unpadded) to HBM and the padded copy (0 outside
// [0, rows-1) x [0, cols-1)) into the row-pair interleaved base rows.
__device__ __forceinline__ void put_decim(const FastArgs& A, float* __restrict__ bs, Rsrc rs0,
                                          const int* __restrict__ xmap, const Pre& P, int Z, int x0, int y0,
                                          int y1) {
#pragma unroll
  for (int u = 0; u < kGather; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < kRB * kBW) {
      const int r = i / kBW, c = i - r * kBW;
      const int y = Z + r, x = x0 - kH + c;
      const float v = (y >= 0 && y < A.rows && xmap[c] >= 0) ? P.g[u] : 0.f;
      const bool out = c >= kH && c < kH + kFW && x < A.cols && y >= y0 && y < y1;
      st_plane(rs0, out ? (y * A.pitch + x) * 4 : kDrop, v);
      const bool src_ok = y >= 0 && y < A.rows - 1 && x >= 0 && x < A.cols - 1;
      bs[(r >> 1) * kBP2 + 2 * c + (r & 1)] = src_ok ? v : 0.f;
    }
  }
}

// Octave-0 row pass of the base blur: ring rows [Y, Y+8), base columns
// [0, 164) (column c <-> image column x0 - 18 + c); lane t < 164 does row pair
// s = t / 41, columns [4j, 4j+4), j = t % 41, from staged columns
// [4j+2, 4j+14).
__device__ __forceinline__ void hb_pass(const float4* __restrict__ stage4, float4* __restrict__ hb4, const f2* g,
                                        int Y) {
  const int t = threadIdx.x;
  if (t >= 4 * 41) return;
  const int s = t / 41, j = t - s * 41;
  const float4* src = stage4 + s * (kSP / 4) + 2 * j + 1;
  f2 w[12];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const float4 v = src[q];
    w[2 * q] = f2{v.x, v.y};
    w[2 * q + 1] = f2{v.z, v.w};
  }
  f2 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = splat(0.f);
#pragma unroll
  for (int b = 0; b < 9; ++b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = pk_tap(w[i + b], g, b, acc[i]);
  }
  hb4[((Y + 2 * s) & (kHbRows - 1)) * (kBP / 4) + j] = make_float4(acc[0].x, acc[1].x, acc[2].x, acc[3].x);
  hb4[((Y + 2 * s + 1) & (kHbRows - 1)) * (kBP / 4) + j] = make_float4(acc[0].y, acc[1].y, acc[2].y, acc[3].y);
}

// Octave-0 column pass of the base blur for base rows [Z+H, Z+H+4) and base
// columns (2p, 2p+1), from row-pass ring rows [Z+H-4, Z+H+8) starting at slot
// S0 = (Z + H - 4) & 15.  Both wave roles take a half (H = 0: waves 0-1,
// H = 4: waves 2-3), so the phase is 36 packed FMAs deep, not 72.  Writes the plane-0 interior to HBM and the padded copy
// (0 outside [0, rows-1) x [0, cols-1)) into the row-pair interleaved base
// rows.  c = 2p is even, so a pair is entirely inside or outside the strip's
// output columns.
template <int S0, int H>
__device__ __forceinline__ void base_col(const FastArgs& A, const f2* g, const float* __restrict__ hb,
                                         float4* __restrict__ bs4, Rsrc rs0, int p, int Z, int x0, int y0,
                                         int y1) {
  LdsF2 h2[4];  // see lds_bases (hb rows are 688 B apart)
  lds_bases(reinterpret_cast<const f2*>(hb) + p, h2);
  f2 win[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) win[k] = h2[k & 3][((S0 + k) & (kHbRows - 1)) * (kBP / 2)];
  f2 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = splat(0.f);
#pragma unroll
  for (int a = 0; a < 9; ++a) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = pk_tap(win[i + a], g, a, acc[i]);
  }
  const int c = 2 * p, x = x0 - kH + c;
  const bool colout = c >= kH && c < kH + kFW && x < A.cols;
  const bool oka = x >= 0 && x < A.cols - 1, okb = x + 1 >= 0 && x + 1 < A.cols - 1;
#pragma unroll
  for (int s = H / 2; s < H / 2 + 2; ++s) {
    const int y = Z + 2 * s;
    const f2 e0 = acc[2 * s - H], e1 = acc[2 * s + 1 - H];
    st_plane2(rs0, (colout && y >= y0 && y < y1) ? (y * A.pitch + x) * 4 : kDrop, e0);
    st_plane2(rs0, (colout && y + 1 >= y0 && y + 1 < y1) ? ((y + 1) * A.pitch + x) * 4 : kDrop, e1);
    const bool ok0 = y >= 0 && y < A.rows - 1, ok1 = y + 1 >= 0 && y + 1 < A.rows - 1;
    bs4[s * (kBP2 / 4) + p] = make_float4((ok0 && oka) ? e0.x : 0.f, (ok1 && oka) ? e1.x : 0.f,
                                          (ok0 && okb) ? e0.y : 0.f, (ok1 && okb) ? e1.y : 0.f);
  }
  asm volatile("; base_col %0 %1" ::"n"(S0), "n"(H));  // see col_fixed
}

// LDS carve-up and per-workgroup constants of the step walk.
struct Walk {
  float4* stage4;  // staged image row pairs (octave 0) / base row pairs
  float4* hb4;     // octave-0 row-pass ring
  float4* rings4;  // scale rings
  int* xmap;       // octave > 0: decimation column map
  float* gimg;     // this image's pyramid block
  const float* img;   // octave 0: this image
  const float* prev;  // octave > 0: the previous octave's scale-3 plane
  long long plane_bytes;
  Rsrc rs0;
  int x0, y0, y1, rbase, Zbeg, Zend;
};

// The step walk of one wave role.  The waves of a workgroup split into two
// roles that run their own copy of the loop (same barriers, so the
// workgroup stays in step):
//   role 0 (waves 0, 1): row and column passes of sigma 4 (W = 18) and sigma 1 (4)
//   role 1 (waves 2, 3): row passes of sigma 3 (12) and sigma 2 (8), column
//                        pass of sigma 3 (wave 2) / sigma 2 (wave 3)
// so each wave's loop is about half the code.  Row passes: the lanes of a role's two waves cover row
// pair hs x 4-column group hj; column passes: lane -> columns (xc, xc + 1).
// Every wave issues exactly 8 plane stores in the column passes.
template <bool OCT0, bool VEC, int WA, int WB>
__device__ __forceinline__ void walk(const FastArgs& A, const Walk& K, int wv) {
  const KArgs KA = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
  f2 kb[5], ka[WA + 1], kc[WB + 1];
  tap_pairs<4>(KA->coef.base, kb);
  tap_pairs<WA>(WA == 18 ? KA->coef.s4 : KA->coef.s3, ka);
  tap_pairs<WB>(WB == 4 ? KA->coef.s1 : KA->coef.s2, kc);
  const int t = threadIdx.x;
  const int L = t & 127;
  const int hs = ((L >> 4) & 1) | ((L >> 6) << 1);
  const int hj = (L & 15) | (((L >> 5) & 1) << 4);
  const int lane = t & 63;
  const int xc = K.x0 + 2 * lane;
  const bool colok = xc < A.cols;
  const int x0 = K.x0, y0 = K.y0, y1 = K.y1, rbase = K.rbase;
  const float* rings = reinterpret_cast<const float*>(K.rings4);
  float* stage = reinterpret_cast<float*>(K.stage4);
  Pre P;
  for (int Z = K.Zbeg; Z < K.Zend; Z += kRB) {
    __syncthreads();  // this step's staged image rows (octave 0) / base rows are published
    // ---- octave 0: base rows [Z, Z+8) from the staged image rows ----
    if (OCT0) {
      hb_pass(K.stage4, K.hb4, kb, Z + 4);
      __syncthreads();
      constexpr int H = WA == 18 ? 0 : 4;  // this role's half of the base rows
      if ((t & 127) < kBW / 2) {
        const float* hb = reinterpret_cast<const float*>(K.hb4);
        if (Z & 8)
          base_col<(4 + H) & 15, H>(A, kb, hb, K.stage4, K.rs0, t & 127, Z, x0, y0, y1);
        else
          base_col<(12 + H) & 15, H>(A, kb, hb, K.stage4, K.rs0, t & 127, Z, x0, y0, y1);
      }
      __syncthreads();
    }
    // next step's source values, in flight during the row and column passes
    // (after the base stores, so exactly the 8 column-pass stores follow them)
    const bool more = Z + kRB < K.Zend;
    if (more) {
      if (OCT0)
        fetch_image<VEC>(A, K.img, x0, Z + kRB + 4, P);
      else
        fetch_decim(A, K.prev, K.xmap, Z + kRB, P);
    }
    // ---- row passes: h rows [Z, Z+8) -> ring slots [(Z - rbase) mod M, +8) ----
    if (Z + kRB > y0 - WA && Z < y1 + WA)
      row_pass<WA>(K.stage4, K.rings4, ka, hs, hj, (Z - rbase) % Ring<WA>::M + 2 * hs);
    if (Z + kRB > y0 - WB && Z < y1 + WB)
      row_pass<WB>(K.stage4, K.rings4, kc, hs, hj, (Z - rbase) % Ring<WB>::M + 2 * hs);
    __syncthreads();
    // ---- column passes: plane rows [Z - w, Z - w + 8) ----
    if (WA == 18) {
      const Rsrc rs4 = plane_rsrc(K.gimg + A.off[4], K.plane_bytes);
      const Rsrc rs1 = plane_rsrc(K.gimg + A.off[1], K.plane_bytes);
      if (wv == 0) {
        col_pass<18, 4, 0, 0>(col_slot<18, 0>(Z, rbase), rings, ka, lane, rs4, A.pitch, xc, Z, y0, y1, colok);
        col_pass<4, 4, 0, 0>(col_slot<4, 0>(Z, rbase), rings, kc, lane, rs1, A.pitch, xc, Z, y0, y1, colok);
      } else {
        col_pass<18, 4, 4, 0>(col_slot<18, 4>(Z, rbase), rings, ka, lane, rs4, A.pitch, xc, Z, y0, y1, colok);
        col_pass<4, 4, 4, 0>(col_slot<4, 4>(Z, rbase), rings, kc, lane, rs1, A.pitch, xc, Z, y0, y1, colok);
      }
    } else {
      if (wv == 2)
        col_pass<12, 8, 0, 0>(col_slot<12, 0>(Z, rbase), rings, ka, lane, plane_rsrc(K.gimg + A.off[3], K.plane_bytes),
                              A.pitch, xc, Z, y0, y1, colok);
      else
        col_pass<8, 8, 0, 0>(col_slot<8, 0>(Z, rbase), rings, kc, lane, plane_rsrc(K.gimg + A.off[2], K.plane_bytes),
                             A.pitch, xc, Z, y0, y1, colok);
    }
    // stage the next step's source (the row passes are done with this step's base rows)
    if (more) {
      SIFT_VM_WAIT(8);
      if (OCT0)
        put_image<VEC>(A, K.stage4, P, x0, Z + kRB + 4);
      else
        put_decim(A, stage, K.rs0, K.xmap, P, Z + kRB, x0, y0, y1);
    }
  }
}

template <bool OCT0, bool VEC>
__global__ __launch_bounds__(256, 2) void pyr_fast_kernel(FastArgs A) {
  __shared__ float4 lds4[(OCT0 ? kLds0 : kLdsN) / 4];
  float* const lds = reinterpret_cast<float*>(lds4);
  Walk K;
  K.stage4 = lds4;
  K.hb4 = lds4 + kStage / 4;
  K.rings4 = lds4 + (kStage + (OCT0 ? kHbRows * kBP : 0)) / 4;
  K.xmap = reinterpret_cast<int*>(lds + kStage + kRingRows * kRP);

  const int t = threadIdx.x;
  const int b = blockIdx.z;
  K.x0 = blockIdx.x * kFW;
  K.y0 = blockIdx.y * A.chunk;
  K.y1 = min(K.y0 + A.chunk, A.rows);
  K.gimg = A.gpyr + b * A.g_img;
  K.plane_bytes = (long long)A.rows * A.pitch * 4;
  K.rs0 = plane_rsrc(K.gimg + A.off[0], K.plane_bytes);
  K.rbase = K.y0 - 64;  // ring slot of row y: (y - rbase) mod M; rows used >= y0 - 60
  K.img = OCT0 ? A.src + b * A.s_img : nullptr;
  K.prev = OCT0 ? nullptr : A.src + b * A.s_img + A.src_off;
  K.Zbeg = K.y0 - kLead;
  K.Zend = K.y1 + kH;
  const int x0 = K.x0;

  Pre P;
  if (OCT0) {
    // prologue: row-pass rows [Zbeg-4, Zbeg+4), then stage step 0's image rows
    f2 kb[5];
    tap_pairs<4>(((KArgs)__builtin_amdgcn_kernarg_segment_ptr())->coef.base, kb);
    fetch_image<VEC>(A, K.img, x0, K.Zbeg - 4, P);
    SIFT_VM_WAIT(0);
    put_image<VEC>(A, K.stage4, P, x0, K.Zbeg - 4);
    __syncthreads();
    hb_pass(K.stage4, K.hb4, kb, K.Zbeg - 4);
    __syncthreads();
    fetch_image<VEC>(A, K.img, x0, K.Zbeg + 4, P);
    SIFT_VM_WAIT(0);
    put_image<VEC>(A, K.stage4, P, x0, K.Zbeg + 4);
  } else {
    for (int c = t; c < kBW; c += 256) {
      const int x = x0 - kH + c;
      int sx = -1;
      if (x >= 0 && x < A.cols) {
        sx = (int)floor(x * A.ifx);
        sx = sx < A.scols - 1 ? sx : A.scols - 1;
      }
      K.xmap[c] = sx;
    }
    __syncthreads();
    fetch_decim(A, K.prev, K.xmap, K.Zbeg, P);
    SIFT_VM_WAIT(0);
    put_decim(A, lds, K.rs0, K.xmap, P, K.Zbeg, x0, K.y0, K.y1);
  }
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  if (wv < 2)
    walk<OCT0, VEC, 18, 4>(A, K, wv);
  else
    walk<OCT0, VEC, 12, 8>(A, K, wv);
}

#undef SIFT_VM_WAIT

void fast_taps(float sigma, float* g) { fast_taps_host(sigma, g); }

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
    A.ify2 = P.rows == 2 * O.rows && A.ify == 2.0;
  }
  // Row chunks per strip: every chunk walks kLead + kH = 42 rows it does not
  // output, and the grid runs in rounds of `resident` workgroups (2 per CU),
  // so pick the chunk count that minimises rounds x rows walked per chunk
  // (octave 1 of a 64 x 1080p batch: 1 chunk, not 3; octave 2: 2, not 6).
  const int strips = (O.cols + kFW - 1) / kFW;
  const long long per = (long long)strips * batch;
  const int resident = resident_grid(
      o > 0 ? (const void*)pyr_fast_kernel<false, false> : (const void*)pyr_fast_kernel<true, true>, 256, 0, 512);
  int ch = 0;
  double best = 0;
  for (int c = 1; c <= (O.rows + kRB - 1) / kRB; ++c) {
    const int h = ((O.rows + c - 1) / c + kRB - 1) / kRB * kRB;
    const int cc = (O.rows + h - 1) / h;
    const double rounds = (double)((per * cc + resident - 1) / resident);
    const double cost = rounds * (h + kLead + kH);
    if (ch == 0 || cost < best) {
      best = cost;
      ch = h;
    }
  }
  const int chunks = (O.rows + ch - 1) / ch;
  A.chunk = ch;
  dim3 grid(strips, chunks, batch);
  if (o > 0)
    hipLaunchKernelGGL((pyr_fast_kernel<false, false>), grid, dim3(256), 0, st, A);
  else if (vec)
    hipLaunchKernelGGL((pyr_fast_kernel<true, true>), grid, dim3(256), 0, st, A);
  else
    hipLaunchKernelGGL((pyr_fast_kernel<true, false>), grid, dim3(256), 0, st, A);
}

}  // namespace sift
