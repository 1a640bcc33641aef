// pyramid_tri.hip -- SIFT_FLAG_FAST Gaussian pyramid for gfx950, three wave
// roles per workgroup (round 3).
//
// The same separable form as pyramid_pair.hip (src/sift.cpp:229-263: every
// scale blurred from its octave base with the reference's sigma, width
// floor(3 sigma) :97 and zero padding outside [0, rows-1) x [0, cols-1)
// :116; K[a][b] = 8192 g(a) g(b) applied as a row pass and a column pass of
// fused multiply-adds -- agreement, not parity, tests/test_gpu_fast.py), with
// the work split so that the VALU issue stays busy:
//
//  * One workgroup = three waves over a 64-column strip of one image and a
//    chunk of rows, walking down 4 rows per step:
//      wave 0: plane 4 (w = 18);  wave 1: plane 3 (w = 12) + octave-0 base;
//      wave 2: planes 2 (w = 8) and 1 (w = 4) + octave-0 base + the next
//      octave's decimated plane 0.
//    Per pixel and step the three waves issue about the same VALU work
//    (74 / 50 + 18 / 48 + 18 lane-ops), and the heaviest one (wave 0) issues
//    no loads, so it never waits on vmcnt (which on gfx9 also waits for every
//    older store).
//  * Column pass = scatter into P >= 2w + 1 register accumulators indexed by
//    output row mod P (P = 40, 28, 20 | 10); the slot pattern repeats every
//    4 * NC rows (NC = 10, 7, 5 steps) and each role's step body is unrolled
//    for its NC phases -- no phase switch, so no accumulator copies at a merge
//    (pyramid_pair.hip's switch costs a copy per accumulator and doubles its
//    live registers), and the accumulators are updated by in-place v_fmac with
//    the tap as a literal.  Few VGPRs -> 5 waves per SIMD.
//  * Source rows (image rows for octave 0, plane-0 rows above) arrive by
//    LDS-DMA (buffer_load ... lds) two steps ahead, issued by waves 1 and 2;
//    out-of-range offsets give the zero padding.  Planes leave through buffer
//    stores whose offset is pushed past the plane for rows / columns outside
//    the output range.
// Algorithmic HBM traffic: 24 B per pyramid pixel -- one read
// (image / plane 0) and five plane writes.
#include "common.hpp"

#include <algorithm>
#include <utility>

#ifndef PT_WPE
#define PT_WPE 5
#endif
// rows per step (4 or 8); 8 halves the barriers and LDS round trips per row
#ifndef PT_ROWS
#define PT_ROWS 8
#endif
// 1: each workgroup walks an equal share of the batch's (column strip, row)
// work, split into pieces at strip ends (about 2.5 pieces of ~1350 rows per
// workgroup for octave 0 of 64 x 1080p); 0: one fixed row chunk per workgroup
// Phase ablation (timing experiments only; results are garbage when set):
// 1 = no plane-store instructions, 2 = no column-pass FMAs, 4 = plane stores
// issued but dropped, 8 = no row-pass FMAs, 16 = no workgroup barriers.
#ifndef PT_ABL
#define PT_ABL 0
#endif
#ifndef PT_PART
#define PT_PART 0
#endif

namespace sift {

#include "../build/sym_coefs.inc"

namespace {

constexpr int kTW = 64;               // output columns per strip
constexpr int kTH = 18;               // widest half-width
constexpr int kTB = PT_ROWS;          // rows per step
static_assert(kTB == 4 || kTB == 8, "rows per step");
constexpr int kTLead = kTB == 4 ? 20 : 24;  // rows walked above the chunk (>= kTH + 2, multiple of kTB)
constexpr int kTBC = kTW + 2 * kTH;   // 100 base columns per strip: [x0 - 18, x0 + 82)
constexpr int kTPit = 128;            // staged row pitch (floats)
constexpr int kTHbRows = kTB + 8;     // octave-0 base row-pass ring: rows [Y - 4, Y + kTB + 4)
constexpr int kTHbPit = 100;
constexpr int kTLd = kTB == 4 ? 2 : 1;  // source-row prefetch lead (steps): 8 rows either way
constexpr int kTRing = kTLd + 1;      // source-row ring slots: the step being read + the steps in flight
constexpr int kTDropP = 0x7ffffff0;   // a buffer offset past every plane
constexpr unsigned kTDropV = 0x7f000000u;  // one store-offset part past every plane (caller checks)

struct TriLds0 {  // octave 0
  float base[kTB][kTPit];          // base rows [Ys, Ys + kTB), columns [x0 - 18, x0 + 110)
  float h[4][kTB][kTW];            // row-pass output [scale: w18, w12, w8, w4][row][column]
  float img[kTRing][kTB][kTPit];   // image rows, LDS-DMA ring (columns [x0 - 22, x0 + 106))
  float hb[kTHbRows][kTHbPit];     // base row-pass ring
};
struct TriLdsN {  // octave > 0
  float base[kTRing][kTB][kTPit];  // plane-0 rows, LDS-DMA ring (columns [x0 - 18, x0 + 110))
  float h[4][kTB][kTW];
};

typedef __amdgpu_buffer_rsrc_t TRsrc;

__device__ __forceinline__ TRsrc pt_rsrc(float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void pt_store(TRsrc rs, unsigned voff, unsigned soff, float v) {
  if constexpr (PT_ABL & 1) return;
  if constexpr (PT_ABL & 4) soff = kTDropV;
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)voff, (int)soff, 0);
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
__device__ __forceinline__ void pt_barrier() {
  if constexpr (PT_ABL & 16)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void pt_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
// cycle, planes, h-buffer slots; io = loads the source rows and runs the
// octave-0 base passes.
template <int ROLE> struct TRole;
// P: the smallest multiple of kTB that is >= 2w + 1 (role 2's two scales
// share the cycle of the larger); NC = P / kTB steps per slot cycle.
template <> struct TRole<0> {
  static constexpr int W1 = 18, W2 = 0, P1 = 40, P2 = 1, NC = P1 / kTB, pl1 = 4, pl2 = 0, h1 = 0, h2 = 0;
  static constexpr bool io = false;
};
template <> struct TRole<1> {
  static constexpr int W1 = 12, W2 = 0, P1 = kTB == 4 ? 28 : 32, P2 = 1, NC = P1 / kTB, pl1 = 3, pl2 = 0, h1 = 1,
                       h2 = 0;
  static constexpr bool io = true;
};
template <> struct TRole<2> {
  static constexpr int W1 = 8, W2 = 4, P1 = kTB == 4 ? 20 : 24, P2 = kTB == 4 ? 10 : 12, NC = P1 / kTB, pl1 = 2,
                       pl2 = 1, h1 = 2, h2 = 3;
  static constexpr bool io = true;
};
static_assert(kTB * TRole<0>::NC % TRole<0>::P1 == 0 && TRole<0>::P1 >= 37, "role 0 cycle");
static_assert(kTB * TRole<1>::NC % TRole<1>::P1 == 0 && TRole<1>::P1 >= 25, "role 1 cycle");
static_assert(kTB * TRole<2>::NC % TRole<2>::P1 == 0 && kTB * TRole<2>::NC % TRole<2>::P2 == 0 &&
                  TRole<2>::P1 >= 17 && TRole<2>::P2 >= 9,
              "role 2 cycle");
static_assert(TRole<2>::pl1 == kLayers, "the decimated plane (nOctaveLayers) is role 2's first scale");

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
  if constexpr (PT_ABL & 2) {
    acc[((R - W) % P + P) % P] = h;
    return;
  }
  (pt_fma_one<W, P, R, I - W>(acc, h), ...);
}

// Column pass of a step at cycle phase M: rows J = 0..3 scatter in order, and
// output row 4M + J - W (slot mod P) is complete after row J.
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
  int chunk;               // output rows per workgroup (multiple of kTB)
  int strips, chunks, items;
  int R4;                  // PT_PART: output steps per strip column
  long long T;             // PT_PART: output steps over the batch (columns x R4)
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
  for (int k = 1; k <= ((PT_ABL & 8) ? 0 : W1); ++k) {
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

// One wave's walk over its workgroup's strip in role ROLE; the three roles run
// the same barrier sequence.
template <bool OCT0, int ROLE>
__device__ __forceinline__ void tri_walk(const TriArgs& A, void* ldsv, int b, int x0, int y0, int y1) {
  using R_ = TRole<ROLE>;
  constexpr int W1 = R_::W1, W2 = R_::W2, P1 = R_::P1, P2 = R_::P2, NC = R_::NC;
  constexpr bool kIO = R_::io, kDec = ROLE == 2;
  // VMEM stores per step: octave-0 base column pass (4, io roles), 1 per row
  // and scale, + 1 per row for the decimated plane
  constexpr int kStores = (PT_ABL & 1) ? 0 : (OCT0 && kIO ? kTB : 0) + kTB * ((W2 ? 2 : 1) + (kDec ? 1 : 0));
  constexpr int kLoads = kIO ? kTB : 0;  // LDS-DMA loads per step (half the step's rows, two per row)
  constexpr int kWaitN = kTLd * kStores + (kTLd - 1) * kLoads;
  static_assert(kWaitN <= 63, "vmcnt is 6 bits");
  const int t = threadIdx.x, lane = t & 63;
  float* const gimg = A.gpyr + b * A.g_img;
  const long long plane_bytes = (long long)A.rows * A.pitch * 4;
  const TRsrc ra = pt_rsrc(gimg + A.off[R_::pl1], plane_bytes);
  const TRsrc rb = pt_rsrc(gimg + A.off[R_::pl2], W2 ? plane_bytes : 0);
  const bool nxt = kDec && A.nxt_off >= 0;
  const TRsrc rn = pt_rsrc(gimg + (nxt ? A.nxt_off : 0), nxt ? (long long)A.n_rows * A.n_pitch * 4 : 0);
  const TRsrc r0 = pt_rsrc(gimg + A.off[0], plane_bytes);
  const unsigned pitch4 = A.pitch * 4, n_pitch4 = A.n_pitch * 4;
  const int x = x0 + lane;
  const unsigned vx = x < A.cols ? (unsigned)x * 4u : kTDropV;
  const unsigned vxn = ((x & 1) == 0 && x < A.cols) ? (unsigned)(x >> 1) * 4u : kTDropV;
  const float* src = A.src + b * A.s_img;
  const int rows = A.rows, cols = A.cols;
  const int Ystart = y0 - kTLead;
  const int nsteps = (y1 + kTH - Ystart + kTB - 1) / kTB;
  float a1[P1], a2[P2];
#pragma unroll
  for (int k = 0; k < P1; ++k) a1[k] = 0.f;
#pragma unroll
  for (int k = 0; k < P2; ++k) a2[k] = 0.f;

  // Source staging (io roles): role 1 loads the first half of a step's rows,
  // role 2 the second, each row as two 64-lane LDS-DMA loads (columns c0 + lane,
  // c0 + 64 + lane; c0 = x0 - 22 for the image, x0 - 18 for plane 0).
  const int c0 = OCT0 ? x0 - 22 : x0 - kTH;
  unsigned voff[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int c = c0 + lane + 64 * hh;
    voff[hh] = (c >= 0 && c < cols - 1) ? (unsigned)c * 4u : kTDropV;
  }
  const TRsrc rsrc = pt_rsrc(const_cast<float*>(src), (long long)rows * A.s_pitch * 4);
  constexpr int kHalf = kTB / 2;
  const int rw = kHalf * (ROLE - 1);
  float* const ring = OCT0 ? &static_cast<TriLds0*>(ldsv)->img[0][0][0] : &static_cast<TriLdsN*>(ldsv)->base[0][0][0];
  auto issue = [&](int r0_, int sl) {
#pragma unroll
    for (int i = 0; i < kHalf; ++i) {
      const int r = r0_ + rw + i;
      const unsigned soff = (r >= 0 && r < rows - 1) ? (unsigned)(r * A.s_pitch * 4) : kTDropV;
      float* dst = ring + (sl * kTB + rw + i) * kTPit;
      pt_dma(pt_lds_addr(dst), voff[0], rsrc, soff);
      pt_dma(pt_lds_addr(dst + 64), voff[1], rsrc, soff);
    }
  };
  // octave 0: step s's base row pass makes base row-pass rows [Ys + 4,
  // Ys + 4 + kTB) from these image rows; octave > 0: the step's base rows
  auto src_row = [&](int s) { return Ystart + kTB * s + (OCT0 ? 4 : 0); };
  auto ring_slot = [](int s) { return (s + 4 * kTRing) % kTRing; };  // s >= s0
  const int s0 = OCT0 ? -(8 / kTB) : 0;  // octave 0: the steps that fill the base ring
  // ring position of base row-pass row Ystart + r (r >= -16)
  auto hb_pos = [](int r) { return (r + 8 * kTHbRows) % kTHbRows; };
  if constexpr (kIO) {
#pragma unroll
    for (int i = 0; i < kTLd; ++i) {
      issue(src_row(s0 + i), ring_slot(s0 + i));
      pt_pad<kStores>(r0);
    }
  }
  const int bt = t - 64;  // io roles: thread index over waves 1 and 2
  int s = s0;
  // The prologue steps s < 0 (octave 0) run the scale passes too, on garbage
  // base rows: every output row they touch lies above the chunk (its store
  // drops), and a stored output's accumulator starts with an assignment at
  // row y - w >= Ystart + 2 (step >= 0).  So every step issues the same stores.
  auto step = [&](auto Mc) -> bool {
    constexpr int M = decltype(Mc)::value;
    if (s >= nsteps) return false;
    const int Ys = Ystart + kTB * s;
    const int slot = ring_slot(s);
    if constexpr (kIO) PT_WAIT(kWaitN);  // own loads of step s; the other role's: the barrier
    pt_barrier();
    if constexpr (kIO) issue(src_row(s + kTLd), ring_slot(s + kTLd));
    if constexpr (OCT0) {
      TriLds0& L = *static_cast<TriLds0*>(ldsv);
      // ---- base row pass (createInitialImage, w = 4): ring rows [Ys + 4, Ys + 4 + kTB) ----
      if constexpr (kIO) {
#pragma unroll
        for (int it0 = 0; it0 < kTB * (kTBC / 4); it0 += 128) {
          const int it = it0 + bt;
          if (it < kTB * (kTBC / 4)) {
            const int j = it / (kTBC / 4), i = it - j * (kTBC / 4);
            const float4* p = reinterpret_cast<const float4*>(&L.img[slot][j][4 * i]);
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
            const int hs = hb_pos(kTB * s + 4 + j);
            *reinterpret_cast<float4*>(&L.hb[hs][4 * i]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
          }
        }
      }
      pt_barrier();
      // ---- base column pass: base rows [Ys, Ys + 4) -> plane 0 + the LDS base rows ----
      // Every io thread runs it (threads past the 100 base columns on a clamped
      // column), so each io wave issues exactly 4 stores here.
      if constexpr (kIO) {
        const int tc = min(bt, kTBC - 1);
        const int q0 = hb_pos(kTB * s - 4);  // ring row Ys - 4
        float hv[kTB + 8];
#pragma unroll
        for (int q = 0; q < kTB + 8; ++q) {
          const int sl = q0 + q;
          hv[q] = L.hb[sl >= kTHbRows ? sl - kTHbRows : sl][tc];
        }
        const int xb = x0 - kTH + bt;
        const unsigned v0 = (bt >= kTH && bt < kTH + kTW && xb < cols) ? (unsigned)xb * 4u : kTDropV;
        const bool cpad = bt < kTBC && xb >= 0 && xb < cols - 1;
        float bv[kTB];
#pragma unroll
        for (int j = 0; j < kTB; ++j) bv[j] = kFastT0[0] * hv[4 + j];
#pragma unroll
        for (int k = 1; k <= 4; ++k) {
          float pk[kTB];
#pragma unroll
          for (int j = 0; j < kTB; ++j) pk[j] = hv[4 + j - k] + hv[4 + j + k];
          asm volatile("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
          for (int j = 0; j < kTB; ++j) bv[j] = fmaf(kFastT0[k], pk[j], bv[j]);
        }
#pragma unroll
        for (int j = 0; j < kTB; ++j) {
          const int y = Ys + j;
          pt_store(r0, v0, (y >= y0 && y < y1) ? (unsigned)y * pitch4 : kTDropV, bv[j]);
          if (bt < kTPit) L.base[j][bt] = (cpad && y >= 0 && y < rows - 1) ? bv[j] : 0.f;
        }
      }
      pt_barrier();
    }
    // ---- row pass of the role's scales: h rows [Ys, Ys + 4) ----
    float (*hbuf)[kTB][kTW];
    const float* brow;  // row lane >> 4 of the step's base rows, columns from 4 (lane & 15)
    if constexpr (OCT0) {
      TriLds0& L = *static_cast<TriLds0*>(ldsv);
      hbuf = L.h;
      brow = &L.base[lane >> 4][4 * (lane & 15)];
    } else {
      TriLdsN& L = *static_cast<TriLdsN*>(ldsv);
      hbuf = L.h;
      brow = &L.base[slot][lane >> 4][4 * (lane & 15)];
    }
    // The step's source rows [Ys, Ys + kTB) reach outputs [Ys - W1, Ys + kTB - 1 + W1]
    // only; a step whose rows reach no output of [y0, y1) (the lead and tail
    // rows beyond this role's width, and octave 0's prologue) skips both
    // passes: its stores drop anyway and the accumulators it would touch are
    // assigned afresh before any stored output uses them.
    const bool live = Ys + kTB - 1 + W1 >= y0 && Ys - W1 < y1;
    float o1[kTB], o2[kTB];
    if (live) {
      // ---- row pass of the role's scales (lane = row, 4 columns; rows
      // lane >> 4 + r4) into the wave's own h rows, read back as lane = column ----
#pragma unroll
      for (int r4 = 0; r4 < kTB; r4 += 4) {
        float h1[4], h2[4];
        pt_rows<W1, W2>(brow + r4 * kTPit, h1, h2);
        const int j = (lane >> 4) + r4, i = lane & 15;
        *reinterpret_cast<float4*>(&hbuf[R_::h1][j][4 * i]) = make_float4(h1[0], h1[1], h1[2], h1[3]);
        if constexpr (W2 != 0)
          *reinterpret_cast<float4*>(&hbuf[R_::h2][j][4 * i]) = make_float4(h2[0], h2[1], h2[2], h2[3]);
      }
      pt_wave_sync();
      float c1[kTB], c2[kTB];
#pragma unroll
      for (int j = 0; j < kTB; ++j) {
        c1[j] = hbuf[R_::h1][j][lane];
        if constexpr (W2 != 0) c2[j] = hbuf[R_::h2][j][lane];
      }
      pt_wave_sync();
      // ---- column pass: lane = column; phase M of the role's slot cycle ----
      pt_col<W1, P1, M>(a1, c1, o1, std::make_integer_sequence<int, kTB>{});
      if constexpr (W2 != 0) pt_col<W2, P2, M>(a2, c2, o2, std::make_integer_sequence<int, kTB>{});
    } else {
#pragma unroll
      for (int j = 0; j < kTB; ++j) o1[j] = o2[j] = 0.f;
    }
    // ---- stores: the step's completed outputs ----
#pragma unroll
    for (int j = 0; j < kTB; ++j) {
      const int ya = Ys + j - W1;  // wave-uniform rows: scalar offsets
      pt_store(ra, vx, (ya >= y0 && ya < y1) ? (unsigned)ya * pitch4 : kTDropV, o1[j]);
      if constexpr (W2 != 0) {
        const int yb = Ys + j - W2;
        pt_store(rb, vx, (yb >= y0 && yb < y1) ? (unsigned)yb * pitch4 : kTDropV, o2[j]);
      }
      if constexpr (kDec) {  // plane nOctaveLayers (src/sift.cpp:252) -> next octave's plane 0 at (y/2, x/2)
        const bool dn = (ya & 1) == 0 && ya >= y0 && ya < y1;
        pt_store(rn, vxn, dn ? (unsigned)(ya >> 1) * n_pitch4 : kTDropV, o1[j]);
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
__global__ __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(PT_WPE))) void pyr_tri_kernel(TriArgs A) {
  __shared__ __attribute__((aligned(16))) char lds[OCT0 ? sizeof(TriLds0) : sizeof(TriLdsN)];
  // XCD-aware order (speed only): blocks b and b + 8 share an XCD, so XCD x
  // takes the contiguous run [x G/8, (x+1) G/8) of (image, chunk, strip) items
  // and neighbouring strips, which read each other's halo columns, meet in one L2.
  const int per = (int)(gridDim.x >> 3);
  const int vk = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto walk = [&](int b, int x0, int y0, int y1) {
    if (wv == 0)
      tri_walk<OCT0, 0>(A, lds, b, x0, y0, y1);
    else if (wv == 1)
      tri_walk<OCT0, 1>(A, lds, b, x0, y0, y1);
    else
      tri_walk<OCT0, 2>(A, lds, b, x0, y0, y1);
  };
  if constexpr (PT_PART) {
    // steps [vk T / G, (vk + 1) T / G) of the (image, strip)-major order
    long long a = (long long)vk * A.T / gridDim.x;
    const long long e = (long long)(vk + 1) * A.T / gridDim.x;
    while (a < e) {
      const int col = (int)(a / A.R4), st = (int)(a - (long long)col * A.R4);
      const int stop = (int)min(e - (long long)col * A.R4, (long long)A.R4);
      walk(col / A.strips, (col % A.strips) * kTW, kTB * st, min(kTB * stop, A.rows));
      a = (long long)col * A.R4 + stop;
      if (a < e) pt_barrier();  // the next piece's prologue refills the rings the last steps read
    }
  } else {
    if (vk >= A.items) return;
    const int strip = vk % A.strips, rest = vk / A.strips;
    const int ck = rest % A.chunks, b = rest / A.chunks;
    const int x0 = strip * kTW, y0 = ck * A.chunk, y1 = min(y0 + A.chunk, A.rows);
    walk(b, x0, y0, y1);
  }
}

}  // namespace

// Octave o of the pyramid, all five planes, and the next octave's plane 0 when
// it is an exact half (pyramid_pair_fuses).  src: octave 0's input images
// (ignored for o > 0: the source is plane 0 of octave o).
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
  if (o + 1 < L.n_oct && pyramid_pair_fuses(L, o + 1)) {
    const Octave& N = L.oct[o + 1];
    A.nxt_off = N.g_off[0];
    A.n_pitch = N.pitch;
    A.n_rows = N.rows;
    A.n_cols = N.cols;
  }
  A.strips = (O.cols + kTW - 1) / kTW;
  const int resident = resident_grid(o > 0 ? (const void*)pyr_tri_kernel<false> : (const void*)pyr_tri_kernel<true>,
                                     192, 0, 2048);
  // chunk count: every chunk walks kTLead + kTH + 2 rows it does not output
  // (+ 8 for octave 0's base lead) and the grid runs in rounds of `resident`
  // workgroups: minimise rounds x rows walked per chunk
  const long long per = (long long)A.strips * batch;
  int grid;
  if (PT_PART) {
    // equal shares of the batch's output steps; at least kMinSteps steps per
    // workgroup (each piece walks kTLead + kTH + 2 rows it does not output)
    constexpr int kMinSteps = 24;
    A.R4 = (O.rows + kTB - 1) / kTB;
    A.T = per * A.R4;
    const long long g = std::min<long long>(resident, std::max<long long>(8, A.T / kMinSteps));
    grid = (int)(g / 8 * 8);
  } else {
    // chunk count: every chunk walks kTLead + kTH + 2 rows it does not output
    // (+ 8 for octave 0's base lead) and the grid runs in rounds of `resident`
    // workgroups: minimise rounds x rows walked per chunk
    int ch = 0;
    double best = 0;
    for (int c = 1; c <= (O.rows + kTB - 1) / kTB; ++c) {
      const int h = ((O.rows + c - 1) / c + kTB - 1) / kTB * kTB;
      const int cc = (O.rows + h - 1) / h;
      const double rounds = (double)((per * cc + resident - 1) / resident);
      const double cost = rounds * (h + kTLead + kTH + 2 + (o == 0 ? 8 : 0));
      if (ch == 0 || cost < best - 1e-9) {
        best = cost;
        ch = h;
      }
    }
    A.chunk = ch;
    A.chunks = (O.rows + ch - 1) / ch;
    A.items = (int)(per * A.chunks);
    grid = (A.items + 7) / 8 * 8;
  }
  if (o > 0)
    hipLaunchKernelGGL((pyr_tri_kernel<false>), dim3(grid), dim3(192), 0, st, A);
  else
    hipLaunchKernelGGL((pyr_tri_kernel<true>), dim3(grid), dim3(192), 0, st, A);
}

}  // namespace sift
