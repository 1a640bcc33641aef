// pyramid_tri.hip -- SIFT_FLAG_FAST Gaussian pyramid for gfx950: three wave
// roles per workgroup, octave-0 base blur pipelined one step ahead (round 4).
//
// The separable form of src/sift.cpp:229-263: every scale blurred from its
// octave base with the reference's sigma, width floor(3 sigma) (:97) and zero
// padding outside [0, rows-1) x [0, cols-1) (:116); K[a][b] = 8192 g(a) g(b)
// applied as a row pass and a column pass of fused multiply-adds -- agreement,
// not parity (tests/test_gpu_fast.py; oracle/sift_oracle.c's
// oracle_fast_pyramid restates the exact operation order, and the GPU planes
// equal it bit for bit).
//
//  * One workgroup = three waves over a 64-column strip of one image and a
//    chunk of rows, walking down 8 rows per step, ONE workgroup barrier per
//    step:
//      wave 0: plane 4 (w = 18);
//      wave 1: plane 3 (w = 12) + half of the octave-0 base blur;
//      wave 2: planes 2 (w = 8) and 1 (w = 4) + the other half + the next
//              octave's decimated plane 0.
//    Per step the three waves issue about the same VALU work (~590 / 400 +
//    200 / 390 + 200 wave-instructions at octave 0).
//  * Octave 0's base blur (createInitialImage, w = 4) runs one step ahead of
//    the scales: at step t waves 1 and 2 turn image rows into the base rows
//    the scales read at step t + 1 (double-buffered), each over its own half
//    of the strip's base columns, so the row pass -> column pass hand-off of
//    the base needs only a wave-level sync.  Round 3 ran the base passes and
//    the scales of a step one after the other behind three barriers; the
//    s_memtime stamps of that kernel (profiles/r4_tri_stamps.txt) showed
//    wave 0 parked at barriers 48 % of its time and waves 1-2 12-15 %.
//  * Column pass = scatter into P >= 2w + 1 register accumulators indexed by
//    output row mod P (P = 40, 32, 24 | 12); the slot pattern repeats every
//    NC = P / 8 steps and each role's step body is unrolled over its NC phases
//    (no phase switch, no accumulator copies); in-place v_fmac with the tap as
//    a literal.
//  * Source rows (image rows for octave 0, plane-0 rows above) arrive by
//    LDS-DMA (buffer_load ... lds) one step ahead, issued by waves 1 and 2;
//    out-of-range offsets give the zero padding.  Planes leave through buffer
//    stores whose offset is pushed past the plane for rows / columns outside
//    the output range (pyramid_tri_fits keeps every plane below that offset).
// Algorithmic HBM traffic: 24 B per pyramid pixel -- one read
// (image / plane 0) and five plane writes.
#include "common.hpp"

#include <algorithm>
#include <array>
#include <functional>
#include <map>
#include <mutex>
#include <queue>
#include <utility>
#include <vector>

namespace sift {

#include "../build/sym_coefs.inc"

namespace {

constexpr int kTW = 64;              // output columns per strip
constexpr int kTH = 18;              // widest half-width
constexpr int kTB = 8;               // rows per step
constexpr int kTLead = 24;           // rows walked above the chunk (>= kTH + 2, multiple of kTB)
constexpr int kTPit = 128;           // base row pitch (floats; = 0 mod 64: pt_rows' ds_read_b128 conflict free)
constexpr int kTBC = kTW + 2 * kTH;  // 100 base columns per strip: [x0 - 18, x0 + 82)
constexpr int kTIW = 112;            // octave-0 image ring row: columns [x0 - 24, x0 + 88)
constexpr int kTHbPit = 104;         // octave-0 base row-pass ring row: columns [x0 - 20, x0 + 84)
constexpr int kTHbRows = 16;
constexpr int kTHalf = kTHbPit / 2;  // base row-pass columns per io role (13 groups of 4)
constexpr int kTHr = 4;              // rows per row-pass transpose round
constexpr int kTDropP = 0x7ffffff0;  // a buffer offset past every plane
constexpr unsigned kTDropV = 0x7f000000u;  // one store-offset part past every plane (pyramid_tri_fits)

struct TriLds0 {  // octave 0: 26,112 B (6 workgroups per CU)
  float base[2][kTB][kTPit];      // base rows of step t in [t & 1], columns [x0 - 18, x0 + 82)
  float h[4][kTHr][kTW];          // row-pass output [scale: w18, w12, w8, w4][row][column]
  float img[2][kTB][kTIW];        // image rows, LDS-DMA ring
  float hb[kTHbRows][kTHbPit];    // base row-pass ring
};
struct TriLdsN {  // octave > 0
  float base[2][kTB][kTPit];      // plane-0 rows, LDS-DMA ring
  float h[4][kTHr][kTW];
};

typedef __amdgpu_buffer_rsrc_t TRsrc;

__device__ __forceinline__ TRsrc pt_rsrc(float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}
typedef unsigned tu32x4 __attribute__((ext_vector_type(4)));
typedef unsigned tu32x2 __attribute__((ext_vector_type(2)));
// 16 / 8 bytes per lane; voff carries the lane's whole offset (row and column)
__device__ __forceinline__ void pt_store4(TRsrc rs, unsigned voff, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(tu32x4, v), rs, (int)voff, 0, 0);
}
__device__ __forceinline__ void pt_store2(TRsrc rs, unsigned voff, float a, float b) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(tu32x2, make_float2(a, b)), rs, (int)voff, 0, 0);
}
// lane l's dword lands at M0 + 4l
__device__ __forceinline__ void pt_dma(unsigned lds_byte, unsigned voff, TRsrc rs, unsigned soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, %3 offen lds"
               ::"s"(lds_byte), "v"(voff), "s"(rs), "s"(soff) : "memory", "m0");
}
__device__ __forceinline__ unsigned pt_lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(const __attribute__((address_space(3))) float*)p);
}
__device__ __forceinline__ void pt_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// LDS hand-off between the lanes of one wave: the wave's LDS operations run
// in program order, so only the compiler needs fencing (nothing moves across)
__device__ __forceinline__ void pt_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  asm volatile("" ::: "memory");
}
// dropped stores at distinct, non-adjacent offsets (no merging)
template <int N>
__device__ __forceinline__ void pt_pad(TRsrc rs) {
#pragma unroll
  for (int i = 0; i < N; ++i) __builtin_amdgcn_raw_buffer_store_b32(0u, rs, kTDropP - 64 * i, 0, 0);
}
#define PT_WAIT(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")

template <int W>
__host__ __device__ constexpr float ttap(int k) {
  return W == 18 ? kFastT4[k] : W == 12 ? kFastT3[k] : W == 8 ? kFastT2[k] : W == 4 ? kFastT1[k] : kFastT0[k];
}

// Wave roles: scales (W1, W2 = 0 for one), accumulator slots, steps per slot
// cycle, planes, h-buffer slots; io = loads the source rows and runs half of
// the octave-0 base blur.
template <int ROLE> struct TRole;
// P: the smallest multiple of kTB that is >= 2w + 1 (role 2's two scales
// share the cycle of the larger); NC = P / kTB steps per slot cycle.
template <> struct TRole<0> {
  static constexpr int W1 = 18, W2 = 0, P1 = 40, P2 = 1, NC = P1 / kTB, pl1 = 4, pl2 = 0, h1 = 0;
  static constexpr bool io = false;
};
template <> struct TRole<1> {
  static constexpr int W1 = 12, W2 = 0, P1 = 32, P2 = 1, NC = P1 / kTB, pl1 = 3, pl2 = 0, h1 = 1;
  static constexpr bool io = true;
};
template <> struct TRole<2> {
  static constexpr int W1 = 8, W2 = 4, P1 = 24, P2 = 12, NC = P1 / kTB, pl1 = 2, pl2 = 1, h1 = 2, h2 = 3;
  static constexpr bool io = true;
};
static_assert(kTB * TRole<0>::NC % TRole<0>::P1 == 0 && TRole<0>::P1 >= 37, "role 0 cycle");
static_assert(kTB * TRole<1>::NC % TRole<1>::P1 == 0 && TRole<1>::P1 >= 25, "role 1 cycle");
static_assert(kTB * TRole<2>::NC % TRole<2>::P1 == 0 && kTB * TRole<2>::NC % TRole<2>::P2 == 0 &&
                  TRole<2>::P1 >= 17 && TRole<2>::P2 >= 9,
              "role 2 cycle");
static_assert(TRole<2>::pl1 == kLayers, "the decimated plane (nOctaveLayers) is role 2's first scale");
static_assert(sizeof(TriLds0) * 6 <= 163840, "six octave-0 workgroups per CU");

// Column pass of one source row at cycle row R: output R - d gets g_|d| h,
// d = -W..W, slot (R - d) mod P; d = -W is that output's first term (assigns).
// In-place v_fmac / v_mul with the tap as a literal.
template <int W, int P, int R, int D>
__device__ __forceinline__ void pt_fma_one(float (&acc)[P], float h) {
  constexpr int slot = ((R - D) % P + P) % P;
  constexpr unsigned bits = __builtin_bit_cast(unsigned, ttap<W>(D < 0 ? -D : D));
  if constexpr (D == -W)
    asm("v_mul_f32 %0, %2, %1" : "=v"(acc[slot]) : "v"(h), "n"(bits));
  else
    asm("v_fmac_f32 %0, %2, %1" : "+v"(acc[slot]) : "v"(h), "n"(bits));
}
template <int W, int P, int R, int... I>
__device__ __forceinline__ void pt_scatter(float (&acc)[P], float h, std::integer_sequence<int, I...>) {
  (pt_fma_one<W, P, R, I - W>(acc, h), ...);
}

// Column pass of a step at cycle phase M: rows J = 0..7 scatter in order, and
// output row 8M + J - W (slot mod P) is complete after row J.
template <int W, int P, int M, int... J>
__device__ __forceinline__ void pt_col(float (&acc)[P], const float (&c)[kTB], float (&o)[kTB],
                                       std::integer_sequence<int, J...>) {
  ((pt_scatter<W, P, kTB * M + J>(acc, c[J], std::make_integer_sequence<int, 2 * W + 1>{}),
    o[J] = acc[((kTB * M + J - W) % P + P) % P]),
   ...);
}

// Runs f(integral_constant<M>) for M = 0, 1, ... while it returns true.
template <class F, int... M>
__device__ __forceinline__ bool pt_cycle(F&& f, std::integer_sequence<int, M...>) {
  return (f(std::integral_constant<int, M>{}) && ...);
}

}  // namespace

struct TriArgs {
  float* gpyr;
  long long g_img;
  long long off[kScales];  // plane offsets of this octave in the image block
  const float* src;        // octave 0: the input images; else this octave's plane 0
  long long s_pitch, s_img;
  long long nxt_off;       // next octave's plane 0 (fused decimation), or -1
  int n_pitch, n_rows, n_cols;
  int pitch, rows, cols;
  // work items (tri_plan): n_full strip columns (image, strip) walked whole,
  // dispatched first (blocks [0, grid_full)); the other columns in `chunks`
  // row chunks of `chunk` rows (multiple of kTB), chunk-major
  int strips, columns;
  int n_full, grid_full;
  int chunk, chunks;
};

namespace {

// Row pass of the role's scales for base row j (= lane >> 4), columns
// 4i .. 4i + 3 (i = lane & 15), from the staged row `brow` (column kTH + u is
// output column 4i + u): pair sums p_k shared by the role's two scales.
template <int W1, int W2>
__device__ __forceinline__ void pt_rows(const float* brow, float (&h1)[4], float (&h2)[4]) {
  const float4* p = reinterpret_cast<const float4*>(brow);
  constexpr int qlo = (kTH - W1) / 4, qhi = (kTH + 3 + W1) / 4;
  float v[40];
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    if (q < qlo || q > qhi) {
      v[4 * q] = v[4 * q + 1] = v[4 * q + 2] = v[4 * q + 3] = 0.f;
      continue;
    }
    float4 f = p[q];
    asm("" : "+v"(f.x), "+v"(f.y), "+v"(f.z), "+v"(f.w));  // whole b128 reads (no misaligned b64 pairs)
    v[4 * q] = f.x;
    v[4 * q + 1] = f.y;
    v[4 * q + 2] = f.z;
    v[4 * q + 3] = f.w;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    h1[u] = ttap<W1>(0) * v[kTH + u];
    if (W2) h2[u] = ttap<W2>(0) * v[kTH + u];
  }
#pragma unroll
  for (int k = 1; k <= W1; ++k) {
    float pk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) pk[u] = v[kTH + u - k] + v[kTH + u + k];
    asm volatile("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      h1[u] = fmaf(ttap<W1>(k), pk[u], h1[u]);
      if (k <= W2) h2[u] = fmaf(ttap<W2>(k), pk[u], h2[u]);
    }
  }
}

// Octave-0 base blur (createInitialImage, w = 4) of io role ROLE at step t:
// row pass of image rows [Ys + 12, Ys + 20) over the role's half of the
// base row-pass columns, then the column pass of base rows [Ys + 8, Ys + 16)
// (the rows the scales read at step t + 1) over the same half -> plane 0
// (columns inside the strip) and the LDS base rows with their zero padding.
template <int ROLE>
__device__ __forceinline__ void tri_base(TriLds0& L, int t, int Ystart, int Ys, int x0, int y0, int y1, int rows,
                                         int cols, TRsrc r0, unsigned pitch4, float (*tr)[kTW]) {
  const int lane = threadIdx.x & 63;
  constexpr int g0 = (ROLE - 1) * (kTHalf / 4);  // first column group of the role
  auto hb_row = [&](int Y) { return (Y - Ystart + 4 * kTHbRows) & (kTHbRows - 1); };  // Y >= Ystart - 48
  const int sl = t & 1;
  // ---- row pass: 8 rows x 13 column groups of 4, lane = task ----
#pragma unroll
  for (int it0 = 0; it0 < kTB * (kTHalf / 4); it0 += 64) {
    const int it = it0 + lane;
    if (it < kTB * (kTHalf / 4)) {
      const int j = it / (kTHalf / 4), g = g0 + it - j * (kTHalf / 4);
      // row-pass column 4g + u is image column x0 - 20 + 4g + u = ring column 4g + 4 + u
      const float4* p = reinterpret_cast<const float4*>(&L.img[sl][j][4 * g]);
      float v[12];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const float4 f = p[q];
        v[4 * q] = f.x;
        v[4 * q + 1] = f.y;
        v[4 * q + 2] = f.z;
        v[4 * q + 3] = f.w;
      }
      float hv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) hv[u] = kFastT0[0] * v[4 + u];
#pragma unroll
      for (int k = 1; k <= 4; ++k) {
        float pk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pk[u] = v[4 + u - k] + v[4 + u + k];
        asm volatile("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
        for (int u = 0; u < 4; ++u) hv[u] = fmaf(kFastT0[k], pk[u], hv[u]);
      }
      *reinterpret_cast<float4*>(&L.hb[hb_row(Ys + 12 + j)][4 * g]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
    }
  }
  pt_wave_sync();
  // ---- column pass: lane = row-pass column hc of the role's half, in two
  // halves of 4 base rows (12-row windows: fewer live registers) ----
  const int hc = (ROLE - 1) * kTHalf + min(lane, kTHalf - 1);
  const int xb = x0 - 20 + hc;  // image column of this lane
  const bool own = lane < kTHalf;
  const bool out0 = own && xb >= x0 && xb < x0 + kTW;  // a plane-0 output column of this role
  // plane-0 stores: 4 rows x the role's 32 output columns per dwordx4 store
  // (lane = row lane >> 4, columns 4 (lane & 15) .. + 3 of the strip)
  const int sg = lane & 15, sr = lane >> 4, sx = x0 + 4 * sg;
  const bool sown = (sg >> 3) == ROLE - 1 && sx < cols;
  const int bc = hc - 2;  // base column: image column x0 - 18 + bc
  const bool wr = own && bc >= 0 && bc < kTBC;
  const bool cpad = xb >= 0 && xb < cols - 1;
  float* brow = &L.base[sl ^ 1][0][max(bc, 0)];
#pragma unroll
  for (int j0 = 0; j0 < kTB; j0 += 4) {
    float hv[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) hv[q] = L.hb[hb_row(Ys + 4 + j0 + q)][hc];
    float bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = kFastT0[0] * hv[4 + j];
#pragma unroll
    for (int k = 1; k <= 4; ++k) {
      float pk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) pk[j] = hv[4 + j - k] + hv[4 + j + k];
      asm volatile("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = fmaf(kFastT0[k], pk[j], bv[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int y = Ys + 8 + j0 + j;
      if (wr) brow[(j0 + j) * kTPit] = (cpad && y >= 0 && y < rows - 1) ? bv[j] : 0.f;
      if (out0) tr[j][xb - x0] = bv[j];
    }
    pt_wave_sync();
    const float4 v = *reinterpret_cast<const float4*>(&tr[sr][4 * sg]);
    pt_wave_sync();
    const int y = Ys + 8 + j0 + sr;
    pt_store4(r0, (sown && y >= y0 && y < y1) ? (unsigned)y * pitch4 + (unsigned)sx * 4u : kTDropV, v);
  }
}

// One wave's walk over its workgroup's strip in role ROLE; the three roles run
// the same barrier sequence (one barrier per step).
template <bool OCT0, int ROLE>
__device__ __forceinline__ void tri_walk(const TriArgs& A, void* ldsv, int b, int x0, int y0, int y1) {
  using R_ = TRole<ROLE>;
  constexpr int W1 = R_::W1, W2 = R_::W2, P1 = R_::P1, P2 = R_::P2, NC = R_::NC;
  constexpr bool kIO = R_::io, kDec = ROLE == 2;
  // VMEM stores per step (after the step's LDS-DMA loads), each 4 rows of
  // the strip: octave-0 plane 0 (io roles), the role's scales, the
  // decimated plane
  constexpr int kStores = (kTB / 4) * ((OCT0 && kIO ? 1 : 0) + (W2 ? 2 : 1) + (kDec ? 1 : 0));
  static_assert(kStores <= 63, "vmcnt is 6 bits");
  const int lane = threadIdx.x & 63;
  float* const gimg = A.gpyr + b * A.g_img;
  const long long plane_bytes = (long long)A.rows * A.pitch * 4;
  const TRsrc ra = pt_rsrc(gimg + A.off[R_::pl1], plane_bytes);
  const TRsrc rb = pt_rsrc(gimg + A.off[R_::pl2], W2 ? plane_bytes : 0);
  const bool nxt = kDec && A.nxt_off >= 0;
  const TRsrc rn = pt_rsrc(gimg + (nxt ? A.nxt_off : 0), nxt ? (long long)A.n_rows * A.n_pitch * 4 : 0);
  const TRsrc r0 = pt_rsrc(gimg + A.off[0], plane_bytes);
  const unsigned pitch4 = A.pitch * 4, n_pitch4 = A.n_pitch * 4;
  // wide stores: lane = (row lane >> 4 of a 4-row round, columns xg .. xg + 3);
  // a group that runs past cols writes the row's padding (pitch >= cols
  // rounded up to 32), which no kernel reads
  const int sr = lane >> 4, xg = x0 + 4 * (lane & 15);
  const bool xok = xg < A.cols;
  const float* src = A.src + b * A.s_img;
  const int rows = A.rows, cols = A.cols;
  const int Ystart = y0 - kTLead;
  const int nsteps = (y1 + kTH - Ystart + kTB - 1) / kTB;
  float a1[P1], a2[P2];
#pragma unroll
  for (int k = 0; k < P1; ++k) a1[k] = 0.f;
#pragma unroll
  for (int k = 0; k < P2; ++k) a2[k] = 0.f;

  // Source staging (io roles): role 1 loads rows 0-3 of a step's 8, role 2
  // rows 4-7, each row as two LDS-DMA loads (lanes 0-63, then the rest of the
  // ring row: 48 lanes of the 112-column image row, 36 of the 100-column base
  // row).  Columns start at x0 - 24 (image) / x0 - 18 (plane 0).
  constexpr int kRowW = OCT0 ? kTIW : kTBC;
  constexpr int kRowP = OCT0 ? kTIW : kTPit;
  const int c0 = OCT0 ? x0 - 24 : x0 - kTH;
  unsigned voff[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int c = c0 + lane + 64 * hh;
    voff[hh] = (c >= 0 && c < cols - 1) ? (unsigned)c * 4u : kTDropV;
  }
  const TRsrc rsrc = pt_rsrc(const_cast<float*>(src), (long long)rows * A.s_pitch * 4);
  constexpr int kHalfRows = kTB / 2;
  const int rw = kHalfRows * (ROLE - 1);
  float* const ring = OCT0 ? &static_cast<TriLds0*>(ldsv)->img[0][0][0] : &static_cast<TriLdsN*>(ldsv)->base[0][0][0];
  // octave 0: the image rows step s's base row pass reads; else the step's base rows
  auto src_row = [&](int s) { return Ystart + kTB * s + (OCT0 ? 12 : 0); };
  auto issue = [&](int s) {
    const int r0_ = src_row(s);
    float* slot = ring + (s & 1) * kTB * kRowP;
#pragma unroll
    for (int i = 0; i < kHalfRows; ++i) {
      const int r = r0_ + rw + i;
      const unsigned soff = (r >= 0 && r < rows - 1) ? (unsigned)(r * A.s_pitch * 4) : kTDropV;
      float* dst = slot + (rw + i) * kRowP;
      pt_dma(pt_lds_addr(dst), voff[0], rsrc, soff);
      if (lane < kRowW - 64) pt_dma(pt_lds_addr(dst + 64), voff[1], rsrc, soff);
    }
  };
  // octave 0: steps -2 and -1 fill the base row-pass ring and the first base rows
  const int s0 = OCT0 ? -2 : 0;
  if constexpr (kIO) {
    issue(s0);
    pt_pad<kStores>(r0);
  }
  int s = s0;
  // A step's scale passes touch only outputs above the chunk before step 0
  // (stores drop) and every stored output's accumulator starts with an
  // assignment at row y - w >= Ystart + 6 (step 0), so dead steps skip them.
  auto step = [&](auto Mc) -> bool {
    constexpr int M = decltype(Mc)::value;
    if (s >= nsteps) return false;
    const int Ys = Ystart + kTB * s;
    if constexpr (kIO) PT_WAIT(kStores);  // own loads of step s; the other role's: the barrier
    pt_barrier();
    if constexpr (kIO) {
      issue(s + 1);
      if constexpr (OCT0)
        tri_base<ROLE>(*static_cast<TriLds0*>(ldsv), s, Ystart, Ys, x0, y0, y1, rows, cols, r0, pitch4,
                       static_cast<TriLds0*>(ldsv)->h[R_::h1]);
    }
    float (*hbuf)[kTHr][kTW];
    const float* brow;  // row lane >> 4 of the step's base rows, columns from 4 (lane & 15)
    if constexpr (OCT0) {
      TriLds0& L = *static_cast<TriLds0*>(ldsv);
      hbuf = L.h;
      brow = &L.base[s & 1][lane >> 4][4 * (lane & 15)];
    } else {
      TriLdsN& L = *static_cast<TriLdsN*>(ldsv);
      hbuf = L.h;
      brow = &L.base[s & 1][lane >> 4][4 * (lane & 15)];
    }
    // The step's source rows [Ys, Ys + 8) reach outputs [Ys - W1, Ys + 7 + W1] only
    const bool live = Ys + kTB - 1 + W1 >= y0 && Ys - W1 < y1;
    float o1[kTB], o2[kTB];
    if (live) {
      // ---- row pass of the role's scales (lane = row, 4 columns) into the
      // wave's own h rows, read back as lane = column, 4 rows per round ----
      float c1[kTB], c2[kTB];
#pragma unroll
      for (int r4 = 0; r4 < kTB; r4 += kTHr) {
        float h1[4], h2[4];
        pt_rows<W1, W2>(brow + r4 * kTPit, h1, h2);
        *reinterpret_cast<float4*>(&hbuf[R_::h1][sr][xg - x0]) = make_float4(h1[0], h1[1], h1[2], h1[3]);
        if constexpr (W2 != 0)
          *reinterpret_cast<float4*>(&hbuf[R_::h2][sr][xg - x0]) = make_float4(h2[0], h2[1], h2[2], h2[3]);
        pt_wave_sync();
#pragma unroll
        for (int jj = 0; jj < kTHr; ++jj) {
          c1[r4 + jj] = hbuf[R_::h1][jj][lane];
          if constexpr (W2 != 0) c2[r4 + jj] = hbuf[R_::h2][jj][lane];
        }
        pt_wave_sync();
      }
      // ---- column pass: lane = column; phase M of the role's slot cycle ----
      pt_col<W1, P1, M>(a1, c1, o1, std::make_integer_sequence<int, kTB>{});
      if constexpr (W2 != 0) pt_col<W2, P2, M>(a2, c2, o2, std::make_integer_sequence<int, kTB>{});
    }
    // ---- stores: the step's completed outputs, turned through the role's h
    // rows so that every lane stores 4 consecutive columns of one row
    // (dwordx4; the decimated plane dwordx2): a quarter of the store
    // instructions of lane = column stores (round 4: -0.11 ms per 64 x 1080p
    // step, profiles/r4_tri_ablation.txt) ----
#pragma unroll
    for (int r4 = 0; r4 < kTB; r4 += 4) {
      float4 v1 = make_float4(0.f, 0.f, 0.f, 0.f), v2 = v1;
      if (live) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          hbuf[R_::h1][jj][lane] = o1[r4 + jj];
          if constexpr (W2 != 0) hbuf[R_::h2][jj][lane] = o2[r4 + jj];
        }
        pt_wave_sync();
        v1 = *reinterpret_cast<const float4*>(&hbuf[R_::h1][sr][xg - x0]);
        if constexpr (W2 != 0) v2 = *reinterpret_cast<const float4*>(&hbuf[R_::h2][sr][xg - x0]);
        pt_wave_sync();
      }
      const int ya = Ys + r4 + sr - W1;  // this lane's output row
      pt_store4(ra, (live && xok && ya >= y0 && ya < y1) ? (unsigned)ya * pitch4 + (unsigned)xg * 4u : kTDropV, v1);
      if constexpr (W2 != 0) {
        const int yb = Ys + r4 + sr - W2;
        pt_store4(rb, (live && xok && yb >= y0 && yb < y1) ? (unsigned)yb * pitch4 + (unsigned)xg * 4u : kTDropV, v2);
      }
      if constexpr (kDec) {  // plane nOctaveLayers (src/sift.cpp:252) -> next octave's plane 0 at (y/2, x/2)
        const bool dn = live && xok && (ya & 1) == 0 && ya >= y0 && ya < y1;
        pt_store2(rn, dn ? (unsigned)(ya >> 1) * n_pitch4 + (unsigned)(xg >> 1) * 4u : kTDropV, v1.x, v1.z);
      }
    }
    asm volatile("; pt_step %0 %1" ::"n"(ROLE), "n"(M));
    ++s;
    return true;
  };
  while (pt_cycle(step, std::make_integer_sequence<int, NC>{})) {
  }
  if constexpr (kIO) PT_WAIT(0);  // the last (unused) loads land before the wave ends
}

#undef PT_WAIT

template <bool OCT0>
__global__ __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(4))) void pyr_tri_kernel(TriArgs A) {
  __shared__ __attribute__((aligned(16))) char lds[OCT0 ? sizeof(TriLds0) : sizeof(TriLdsN)];
  // XCD-aware order within each phase (speed only): blocks b and b + 8 share
  // an XCD, so XCD x takes a contiguous run of the phase's items and
  // neighbouring strips, which read each other's halo columns, meet in one L2.
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int col, y0, y1;
  if ((int)blockIdx.x < A.grid_full) {
    const int vk = (int)(blockIdx.x & 7) * (A.grid_full >> 3) + (int)(blockIdx.x >> 3);
    if (vk >= A.n_full) return;
    col = vk;
    y0 = 0;
    y1 = A.rows;
  } else {
    const int bb = (int)blockIdx.x - A.grid_full, gb = (int)gridDim.x - A.grid_full;
    const int vk = (bb & 7) * (gb >> 3) + (bb >> 3);
    const int rest = A.columns - A.n_full;
    if (vk >= rest * A.chunks) return;
    col = A.n_full + vk % rest;
    y0 = (vk / rest) * A.chunk;
    y1 = min(y0 + A.chunk, A.rows);
  }
  const int b = col / A.strips, x0 = (col - b * A.strips) * kTW;
  if (wv == 0)
    tri_walk<OCT0, 0>(A, lds, b, x0, y0, y1);
  else if (wv == 1)
    tri_walk<OCT0, 1>(A, lds, b, x0, y0, y1);
  else
    tri_walk<OCT0, 2>(A, lds, b, x0, y0, y1);
}

}  // namespace

bool pyramid_fuses_decimation(const Layout& L, int o) {
  return o > 0 && L.oct[o - 1].rows == 2 * L.oct[o].rows && L.oct[o - 1].cols == 2 * L.oct[o].cols;
}

bool pyramid_tri_fits(const Layout& L, long long src_row_stride) {
  // every plane and the input rows below the dropped-offset part (octave 0 is
  // the largest plane), and the input's row offsets in 32 bits
  const long long plane = (long long)L.oct[0].rows * L.oct[0].pitch * 4;
  const long long srcb = (long long)L.oct[0].rows * src_row_stride * 4;
  return plane < (long long)kTDropV && srcb < (long long)kTDropV;
}

bool fast_taps_match(float sigma_base, const float* sig) {
  const float sg[5] = {sigma_base, sig[0], sig[1], sig[2], sig[3]};
  const int ws[5] = {4, 4, 8, 12, 18};
  const float* tabs[5] = {kFastT0, kFastT1, kFastT2, kFastT3, kFastT4};
  for (int t = 0; t < 5; ++t) {
    float g[64];
    if (fast_taps_host(sg[t], nullptr) != 2 * ws[t] + 1) return false;
    fast_taps_host(sg[t], g);
    for (int a = 0; a <= ws[t]; ++a)
      if (__builtin_memcmp(&tabs[t][a], &g[ws[t] + a], 4) != 0 || __builtin_memcmp(&g[ws[t] - a], &g[ws[t] + a], 4) != 0)
        return false;
  }
  return true;
}

// Work items of one launch: every strip column walks its rows plus `halo`
// rows it does not output (the lead above, the tail below, octave 0's base
// prologue), so short chunks cost halo, and the grid runs in rounds of
// `slots` resident workgroups, so a ragged last round idles the chip.  The
// plan: n_full columns walked whole, dispatched first, then the other
// columns in `chunks` chunks each.  Candidates (n_full a multiple of slots, or
// every column; 1-32 chunks) are scored by list-scheduling the items in
// dispatch order on `slots` identical slots (cost = rows walked); round 3
// cut every column into equal chunks (64 x 1080p octave 0: 5 rounds of 272 +
// 60 rows = 1,660 rows per slot; the mixed plan: 1,080 + 60, then 270 + 60 =
// 1,470).
TriPlan tri_plan(int columns, int rows, int slots, int halo) {
  static std::mutex mu;
  static std::map<std::array<int, 4>, TriPlan> cache;
  const std::array<int, 4> key{columns, rows, slots, halo};
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  TriPlan best{columns, rows, 1};
  long long best_cost = -1, best_items = 0;
  std::vector<int> fulls;
  for (long long f = 0; f < columns; f += slots) fulls.push_back((int)f);
  fulls.push_back(columns);
  for (int nf : fulls)
    for (int c = 1; c <= (nf == columns ? 1 : 32); ++c) {
      const int ch = nf == columns ? rows : ((rows + c - 1) / c + kTB - 1) / kTB * kTB;
      const int cc = nf == columns ? 1 : (rows + ch - 1) / ch;
      if (cc != c) continue;  // the same chunking as a smaller c
      // list scheduling in dispatch order: each item to the earliest free slot
      std::priority_queue<long long, std::vector<long long>, std::greater<long long>> q;
      for (int i = 0; i < std::min<long long>(slots, (long long)nf + (long long)(columns - nf) * cc); ++i) q.push(0);
      auto put = [&](long long len) {
        const long long t = q.top();
        q.pop();
        q.push(t + len + halo);
      };
      for (int i = 0; i < nf; ++i) put(rows);
      for (int k = 0; k < cc; ++k)
        for (int i = nf; i < columns; ++i) put(std::min(ch, rows - k * ch));
      long long cost = 0;
      while (!q.empty()) {
        cost = std::max(cost, q.top());
        q.pop();
      }
      const long long items = nf + (long long)(columns - nf) * cc;
      if (best_cost < 0 || cost < best_cost || (cost == best_cost && items < best_items)) {
        best_cost = cost;
        best_items = items;
        best = TriPlan{nf, ch, cc};
      }
    }
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = best;
  return best;
}

// Octave o of the pyramid, all five planes, and the next octave's plane 0 when
// it is an exact half (pyramid_fuses_decimation).  src: octave 0's input
// images (ignored for o > 0: the source is plane 0 of octave o).
void launch_pyramid_tri(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch) {
  const Octave& O = L.oct[o];
  TriArgs A{};
  A.gpyr = gpyr;
  A.g_img = L.g_img;
  for (int s = 0; s < kScales; ++s) A.off[s] = O.g_off[s];
  A.pitch = O.pitch;
  A.rows = O.rows;
  A.cols = O.cols;
  if (o == 0) {
    A.src = src.p;
    A.s_pitch = src.pitch;
    A.s_img = src.img_stride;
  } else {
    A.src = gpyr + O.g_off[0];
    A.s_pitch = O.pitch;
    A.s_img = L.g_img;
  }
  A.nxt_off = -1;
  if (o + 1 < L.n_oct && pyramid_fuses_decimation(L, o + 1)) {
    const Octave& N = L.oct[o + 1];
    A.nxt_off = N.g_off[0];
    A.n_pitch = N.pitch;
    A.n_rows = N.rows;
    A.n_cols = N.cols;
  }
  A.strips = (O.cols + kTW - 1) / kTW;
  A.columns = A.strips * batch;
  const int resident = resident_grid(o > 0 ? (const void*)pyr_tri_kernel<false> : (const void*)pyr_tri_kernel<true>,
                                     192, 0, 2048);
  const TriPlan P = tri_plan(A.columns, O.rows, resident, kTLead + kTH + 2 + (o == 0 ? 16 : 0));
  A.n_full = P.n_full;
  A.grid_full = (P.n_full + 7) / 8 * 8;
  A.chunk = P.chunk;
  A.chunks = P.chunks;
  const long long rest = (long long)(A.columns - P.n_full) * P.chunks;
  const int grid = A.grid_full + (int)((rest + 7) / 8 * 8);
  if (o > 0)
    hipLaunchKernelGGL((pyr_tri_kernel<false>), dim3(grid), dim3(192), 0, st, A);
  else
    hipLaunchKernelGGL((pyr_tri_kernel<true>), dim3(grid), dim3(192), 0, st, A);
}

}  // namespace sift
