// pyramid_pair.hip -- SIFT_FLAG_FAST Gaussian pyramid for gfx950, wave-pair
// form (round 3).
//
// The north_star's separable form of buildGaussianPyramid (src/sift.cpp:
// 229-263): every scale is still blurred from its octave base with the
// reference's sigma and width (sig[] :240-245, w = floor(3 sigma) :97) and the
// reference's source padding (rows / columns outside [0, rows-1) x
// [0, cols-1) read as 0, getSubMatrix :116), but K[a][b] = 8192 g(a) g(b)
// (:103-104) is applied as a row pass and a column pass with fused
// multiply-adds -- agreement, not parity (tests/test_gpu_fast.py).
//
// Why a new form.  pyr_fast_kernel (pyramid_fast.hip) keeps the column passes'
// windows in LDS rings (80 KB per 4-wave workgroup, 2 per CU), and its FMA
// stream and plane stores serialise.  Here the column pass is a
// scatter into register accumulators: no rings, 11 KB of LDS per 2-wave
// workgroup (octave 0; 6 KB above), so a CU holds many independent
// workgroups whose phases drift apart -- one workgroup's stores and loads run
// beside another's FMA stream.
//
// One workgroup = two waves over a 64-column strip of one image and a chunk
// of rows, walking down 4 rows per step:
//   wave A: planes 4 (w = 18) and 1 (w = 4); wave B: planes 3 (w = 12), 2 (8).
//   octave 0: the image rows are staged in LDS; the base blur (createInitial
//     Image, sigma sqrt(1.6^2 + 0.2^2), w = 4) runs as a row pass into a
//     12-row LDS ring and a column pass (both waves, one thread per column of
//     the strip's 100 base columns) that stores plane 0 and the padded base
//     rows;  octave o > 0: plane 0 (written by octave o-1's launch, the fused
//     INTER_NEAREST decimation below) is staged as the base rows.
//   row pass: a lane takes one row and 4 adjacent columns; its 40-float window
//     (10 conflict-free ds_read_b128) is folded into pair sums
//     p_k = x(c-k) + x(c+k) shared by the wave's two scales, then
//     h = g0 x(c), h = fma(g_k, p_k, h) for k = 1..w; rows go to the wave's
//     own LDS buffer [scale][row][column];
//   column pass: lane = column.  Source row r adds g_|r-y| h(r) to the
//     accumulator of each output row y in [r - w, r + w] (the first term
//     assigns), held in P >= 2w + 1 registers indexed by y mod P; output r - w
//     is complete after row r and stored at once, so every output receives its
//     terms in ascending row order.  The slot pattern repeats every 40 rows
//     (P = 40, 10, 40, 20 divide 40): the step body is instantiated for the 10
//     step phases and picked by a uniform switch.
//   planes leave through buffer stores whose offset is pushed past the plane
//     for rows / columns outside the output range (no branches);
//   plane 2 (w = 8; gpyr[(o-1)*nScales + nOctaveLayers], nOctaveLayers = 2)
//     also writes the next octave's plane 0, its INTER_NEAREST half
//     (src/sift.cpp:252-254) = (2y, 2x) when the next octave has exactly half
//     the rows and columns (the caller decimates otherwise).
//   the next step's source rows are loaded with instructions the compiler does
//   not track and waited for with an explicit vmcnt that leaves this step's
//   plane stores in flight (pp_ld, PP_WAIT).
// Algorithmic HBM traffic: 24 B per pyramid pixel -- one
// read (image / plane 0) and five plane writes.  Taps are literal operands
// (build/sym_coefs.inc kFastT*, printed from gauss_host.hpp's fast_taps_host).
#include "common.hpp"

#include <math.h>
#include <stdlib.h>

#include <utility>

#ifndef PP_WPE
#define PP_WPE 3
#endif
// Phase ablation (timing experiments only; results are garbage when set):
// 1 = no row-pass window reads, 2 = no column-pass FMAs, 4 = every plane store
// dropped, 8 = no workgroup barriers, 16 = no source loads, 32 = one column-pass
// phase body instead of ten (code size).
#ifndef PP_ABL
#define PP_ABL 0
#endif
// Row-pass window reads issued just ahead of their first tap (fewer live
// VGPRs) instead of all at the top of the pass.
#ifndef PP_ROLE_ONLY  // register-count experiments only: compile one wave role
#define PP_ROLE_ONLY 0
#endif
#ifndef PP_ASM_FMA
#define PP_ASM_FMA 0
#endif
#ifndef PP_LAZY
#define PP_LAZY 0
#endif
#ifndef PP_LAZY_D
#define PP_LAZY_D 3
#endif

namespace sift {

#include "../build/sym_coefs.inc"

namespace {

constexpr int kLazyD = PP_LAZY_D;  // taps between a lazy window read and its first use
constexpr int kPW = 64;         // output columns per strip
constexpr int kPH = 18;         // widest scale half-width
constexpr int kPB = 4;          // rows per step
constexpr int kPer = 10;        // steps per slot cycle (40 rows)
constexpr int kLead = 20;       // rows walked above the chunk (>= kPH, multiple of kPB)
constexpr int kBC = kPW + 2 * kPH;   // 100 base columns per strip: [x0 - 18, x0 + 82)
constexpr int kBPit = 128;      // base row pitch (floats): the row pass's b128 reads are conflict free
constexpr int kIC = kBC + 8;    // 108 staged image columns: [x0 - 22, x0 + 86)
constexpr int kHbRows = 12;     // base row-pass ring: rows [Y - 4, Y + 8)
constexpr int kHbPit = 100;
constexpr int kDropP = 0x7ffffff0;  // buffer offset past every plane: the store is dropped
static_assert(kIC <= 128 && kBC <= 128 && kBPit == 128, "a staged row is two 64-lane DMA loads");
// Store offsets: voffset (per lane, fixed) + soffset (per row, wave-uniform).
// Either part alone pushes the sum past every plane (planes stay below
// kDropV bytes: launch_pyramid_pair's caller checks), and two drop parts
// still fit 32 bits.
constexpr unsigned kDropV = 0x7f000000u;

// Source-row prefetch lead: step s + kLeadSteps's rows are issued in step s.
// vmcnt also counts stores (gfx9), so waiting for a step's loads waits for
// every store issued before them: a longer lead gives those stores more time.
#ifndef PP_LEAD
#define PP_LEAD 2
#endif
constexpr int kLeadSteps = PP_LEAD;
constexpr int kRing = kLeadSteps + 1;  // ring slots: the step being read + the steps in flight
struct PairLds0 {  // octave 0
  float base[2][kPB][kBPit];
  float h[2][2][kPB][kPW];  // [wave][scale][row][column]
  float img[kRing][kPB][kBPit];  // image rows, LDS-DMA ring (columns [x0 - 22, x0 + 106))
  float hb[kHbRows][kHbPit];
};
struct PairLdsN {  // octave > 0
  float base[kRing][kPB][kBPit];  // plane-0 rows, LDS-DMA ring (columns [x0 - 18, x0 + 110))
  float h[2][2][kPB][kPW];
};

typedef __amdgpu_buffer_rsrc_t PRsrc;

__device__ __forceinline__ PRsrc pp_rsrc(float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void pp_store(PRsrc rs, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, off, 0, 0);
}
__device__ __forceinline__ void pp_store_s(PRsrc rs, unsigned voff, unsigned soff, float v) {
  if constexpr (PP_ABL & 4) soff = kDropV;
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)voff, (int)soff, 0);
}

// Source rows go straight to LDS (buffer_load_dword ... lds: lane l's dword
// lands at M0 + 4l).  Out-of-range offsets read 0, which is how the padding
// rows and columns (outside [0, rows-1) x [0, cols-1), getSubMatrix :116)
// arrive as zeros with no select.  The wave waits for its own loads with an
// explicit vmcnt and the workgroup barrier then covers the other wave's.
__device__ __forceinline__ void pp_dma(unsigned lds_byte, unsigned voff, PRsrc rs, unsigned soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, %3 offen lds"
               ::"s"(lds_byte), "v"(voff), "s"(rs), "s"(soff) : "memory", "m0");
}
__device__ __forceinline__ unsigned pp_lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(const __attribute__((address_space(3))) float*)p);
}

__device__ __forceinline__ void pp_barrier() {
  if constexpr (PP_ABL & 8)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void pp_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Scale of a wave role: slot count, plane index, taps (centre first).
template <int W> struct PScale;
template <> struct PScale<18> { static constexpr int P = 40, plane = 4; };
template <> struct PScale<4> { static constexpr int P = 10, plane = 1; };
template <> struct PScale<12> { static constexpr int P = 40, plane = 3; };
template <> struct PScale<8> { static constexpr int P = 20, plane = 2; };
static_assert(kPer * kPB == 40 && 40 % PScale<18>::P == 0 && 40 % PScale<4>::P == 0 &&
                  40 % PScale<12>::P == 0 && 40 % PScale<8>::P == 0,
              "slot counts divide the 40-row cycle");
static_assert(PScale<18>::P >= 37 && PScale<4>::P >= 9 && PScale<12>::P >= 25 && PScale<8>::P >= 17,
              "P >= 2w + 1");

template <int W>
__host__ __device__ constexpr float ptap(int k) {
  return W == 18 ? kFastT4[k] : W == 12 ? kFastT3[k] : W == 8 ? kFastT2[k] : kFastT1[k];
}

}  // namespace

struct PairArgs {
  float* gpyr;
  long long g_img;
  long long off[kScales];  // plane offsets of this octave in the image block
  const float* src;        // octave 0: the input images; else this octave's plane 0
  long long s_pitch, s_img;
  long long nxt_off;       // next octave's plane 0 (fused decimation), or -1
  int n_pitch, n_rows, n_cols;
  int pitch, rows, cols;
  int chunk;               // output rows per workgroup (multiple of kPB)
  int strips, chunks, items;
};

namespace {

// In-place v_fmac with the tap as a literal (PP_ASM_FMA): hipcc otherwise
// renames accumulators through v_fmamk (dst != acc) and copies them back at
// the phase merge, which doubles their live registers.
template <int W, int R, int D>
__device__ __forceinline__ void pp_fma_one(float (&acc)[PScale<W>::P], float h) {
  constexpr int P = PScale<W>::P;
  constexpr int slot = ((R - D) % P + P) % P;
  constexpr unsigned bits = __builtin_bit_cast(unsigned, ptap<W>(D < 0 ? -D : D));
  if constexpr (D == -W)
    asm("v_mul_f32 %0, %2, %1" : "=v"(acc[slot]) : "v"(h), "n"(bits));
  else
    asm("v_fmac_f32 %0, %2, %1" : "+v"(acc[slot]) : "v"(h), "n"(bits));
}
template <int W, int R, int... I>
__device__ __forceinline__ void pp_scatter_asm(float (&acc)[PScale<W>::P], float h, std::integer_sequence<int, I...>) {
  (pp_fma_one<W, R, I - W>(acc, h), ...);
}

// Column pass of one source row at cycle row R: output R - d gets g_|d| h,
// d = -W..W (slot (R - d) mod P); d = -W is that output's first term.
template <int W, int R>
__device__ __forceinline__ void pp_scatter(float (&acc)[PScale<W>::P], float h) {
  constexpr int P = PScale<W>::P;
  if constexpr (PP_ABL & 2) {
    acc[((R - W) % P + P) % P] = h;
    return;
  }
#pragma unroll
  for (int d = -W; d <= W; ++d) {
    const int slot = ((R - d) % P + P) % P;
    if constexpr (PP_ASM_FMA) {
      (void)slot;  // pp_scatter_asm below
    } else {
      const float c = ptap<W>(d < 0 ? -d : d);
      if (d == -W)
        acc[slot] = c * h;
      else
        acc[slot] = fmaf(c, h, acc[slot]);
    }
  }
  if constexpr (PP_ASM_FMA) pp_scatter_asm<W, R>(acc, h, std::make_integer_sequence<int, 2 * W + 1>{});
}

struct PPOut {
  PRsrc ra, rb, rn;
  int Ys, y0, y1, pitch4, n_pitch4;
  unsigned vx, vxn;  // per-lane voffsets: plane column, decimated column (or kDropV)
};

static_assert(kLayers == 2 && PScale<8>::plane == kLayers, "the decimated plane is wave B's w = 8 scale");

// Source row J of a step at cycle phase M, both scales; oa / ob get the two
// outputs it completes (rows Ys + J - WA and Ys + J - WB).
template <int WA, int WB, int M, int J>
__device__ __forceinline__ void pp_row(float (&aa)[PScale<WA>::P], float (&ab)[PScale<WB>::P], float ha, float hb,
                                       float& oa, float& ob) {
  constexpr int R = (kPB * M + J) % 40;
  constexpr int PA = PScale<WA>::P, PB = PScale<WB>::P;
  pp_scatter<WA, R>(aa, ha);
  pp_scatter<WB, R>(ab, hb);
  constexpr int sa = ((R - WA) % PA + PA) % PA, sb = ((R - WB) % PB + PB) % PB;
  oa = aa[sa];
  ob = ab[sb];
}

template <int WA, int WB, int M>
__device__ __forceinline__ void pp_step(float (&aa)[PScale<WA>::P], float (&ab)[PScale<WB>::P],
                                        const float (&ha)[kPB], const float (&hb)[kPB], float (&oa)[kPB],
                                        float (&ob)[kPB]) {
  pp_row<WA, WB, M, 0>(aa, ab, ha[0], hb[0], oa[0], ob[0]);
  pp_row<WA, WB, M, 1>(aa, ab, ha[1], hb[1], oa[1], ob[1]);
  pp_row<WA, WB, M, 2>(aa, ab, ha[2], hb[2], oa[2], ob[2]);
  pp_row<WA, WB, M, 3>(aa, ab, ha[3], hb[3], oa[3], ob[3]);
  // a distinct tail per phase: keeps hipcc from merging the bodies
  asm volatile("; pp_step %0 %1 %2" ::"n"(WA), "n"(WB), "n"(M));
}

// Exactly one body runs for every m (the last phase is the default).
template <int WA, int WB>
__device__ __forceinline__ void pp_dispatch(int m, float (&aa)[PScale<WA>::P], float (&ab)[PScale<WB>::P],
                                            const float (&ha)[kPB], const float (&hb)[kPB], float (&oa)[kPB],
                                            float (&ob)[kPB]) {
  static_assert(kPer == 10, "cases");
  if constexpr ((PP_ABL & 32) != 0) {  // ablation: one phase body only (code size)
    pp_step<WA, WB, 0>(aa, ab, ha, hb, oa, ob);
    return;
  }
  switch (m) {
    case 0: pp_step<WA, WB, 0>(aa, ab, ha, hb, oa, ob); break;
    case 1: pp_step<WA, WB, 1>(aa, ab, ha, hb, oa, ob); break;
    case 2: pp_step<WA, WB, 2>(aa, ab, ha, hb, oa, ob); break;
    case 3: pp_step<WA, WB, 3>(aa, ab, ha, hb, oa, ob); break;
    case 4: pp_step<WA, WB, 4>(aa, ab, ha, hb, oa, ob); break;
    case 5: pp_step<WA, WB, 5>(aa, ab, ha, hb, oa, ob); break;
    case 6: pp_step<WA, WB, 6>(aa, ab, ha, hb, oa, ob); break;
    case 7: pp_step<WA, WB, 7>(aa, ab, ha, hb, oa, ob); break;
    case 8: pp_step<WA, WB, 8>(aa, ab, ha, hb, oa, ob); break;
    default: pp_step<WA, WB, 9>(aa, ab, ha, hb, oa, ob); break;
  }
}

// The step's completed outputs (after the phase switch, so every path issues
// the same stores), and plane 2's decimated copy for the next octave.
template <int WA, int WB>
__device__ __forceinline__ void pp_stores(const float (&oa)[kPB], const float (&ob)[kPB], const PPOut& o) {
#pragma unroll
  for (int j = 0; j < kPB; ++j) {
    const int ya = o.Ys + j - WA, yb = o.Ys + j - WB;  // wave-uniform rows: scalar offsets
    pp_store_s(o.ra, o.vx, (ya >= o.y0 && ya < o.y1) ? (unsigned)(ya * o.pitch4) : kDropV, oa[j]);
    pp_store_s(o.rb, o.vx, (yb >= o.y0 && yb < o.y1) ? (unsigned)(yb * o.pitch4) : kDropV, ob[j]);
    // plane nOctaveLayers (= 2, src/sift.cpp:252) -> next octave's plane 0 at (y / 2, x / 2)
    if constexpr (PScale<WA>::plane == kLayers || PScale<WB>::plane == kLayers) {
      constexpr bool A_ = PScale<WA>::plane == kLayers;
      const int yd = A_ ? ya : yb;
      const bool dn = (yd & 1) == 0 && yd >= o.y0 && yd < o.y1;
      pp_store_s(o.rn, o.vxn, dn ? (unsigned)((yd >> 1) * o.n_pitch4) : kDropV, A_ ? oa[j] : ob[j]);
    }
  }
}

// Distinct, non-adjacent offsets: identical stores to one address would be
// merged, adjacent ones combined into one wide store.
template <int N>
__device__ __forceinline__ void pp_pad(PRsrc rs) {
#pragma unroll
  for (int i = 0; i < N; ++i) pp_store(rs, kDropP - 64 * i, 0.f);
}

// Wait for the step's source loads; N = VMEM operations issued after them.
#define PP_WAIT(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")

// One wave's walk over the workgroup's strip; wave A (WA, WB) = (18, 4),
// wave B = (12, 8).  Both waves run the same barrier sequence.
template <bool OCT0, int WA, int WB>
__device__ __forceinline__ void pp_walk(const PairArgs& A, void* ldsv, int wv, int b, int x0, int y0, int y1) {
  constexpr int PA = PScale<WA>::P, PB = PScale<WB>::P;
  // VMEM stores per step after the prefetch: base column pass (4, octave 0),
  // 2 per row (+1 decimation store per row on wave B)
  constexpr bool kDec = PScale<WA>::plane == kLayers || PScale<WB>::plane == kLayers;
  constexpr int kStores = (OCT0 ? 4 : 0) + kPB * (kDec ? 3 : 2);
  const int t = threadIdx.x, lane = t & 63;
  float* const gimg = A.gpyr + b * A.g_img;
  const long long plane_bytes = (long long)A.rows * A.pitch * 4;
  PPOut o;
  o.ra = pp_rsrc(gimg + A.off[PScale<WA>::plane], plane_bytes);
  o.rb = pp_rsrc(gimg + A.off[PScale<WB>::plane], plane_bytes);
  const bool nxt = A.nxt_off >= 0;
  o.rn = pp_rsrc(gimg + (nxt ? A.nxt_off : 0), nxt ? (long long)A.n_rows * A.n_pitch * 4 : 0);
  const PRsrc r0 = pp_rsrc(gimg + A.off[0], plane_bytes);
  o.y0 = y0;
  o.y1 = y1;
  o.pitch4 = A.pitch * 4;
  o.n_pitch4 = A.n_pitch * 4;
  {
    const int x = x0 + lane;
    o.vx = x < A.cols ? (unsigned)x * 4u : kDropV;
    o.vxn = ((x & 1) == 0 && x < A.cols) ? (unsigned)(x >> 1) * 4u : kDropV;
  }
  const float* src = A.src + b * A.s_img;
  const int rows = A.rows, cols = A.cols;
  const int Ystart = y0 - kLead;
  const int nsteps = (y1 + kPH - Ystart + kPB - 1) / kPB;
  float aa[PA], ab[PB];
#pragma unroll
  for (int k = 0; k < PA; ++k) aa[k] = 0.f;
#pragma unroll
  for (int k = 0; k < PB; ++k) ab[k] = 0.f;

  // Source staging: wave wv loads rows 2wv, 2wv + 1 of a step's four, each as
  // two 64-lane LDS-DMA loads (columns c0 + lane, c0 + 64 + lane; c0 = x0 - 22
  // for the image, x0 - 18 for plane 0); per-lane column offsets are fixed for
  // the walk, the row offset is a scalar; invalid positions are out of range
  // and land as 0.
  const int c0 = OCT0 ? x0 - 22 : x0 - kPH;
  unsigned voff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = c0 + lane + 64 * h;
    voff[h] = (c >= 0 && c < cols - 1) ? (unsigned)c * 4u : kDropV;
  }
  const PRsrc rsrc = pp_rsrc(const_cast<float*>(src), (long long)rows * A.s_pitch * 4);
  const int rw = 2 * wv;  // this wave's first row of the four
  float* const ring = OCT0 ? &static_cast<PairLds0*>(ldsv)->img[0][0][0] : &static_cast<PairLdsN*>(ldsv)->base[0][0][0];
  // rows [r0, r0 + 4) of a step into ring slot sl
  auto issue = [&](int r0, int sl) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = r0 + rw + i;
      const unsigned soff = (r >= 0 && r < rows - 1) ? (unsigned)(r * A.s_pitch * 4) : kDropV;
      float* dst = ring + (sl * kPB + rw + i) * kBPit;
      pp_dma(pp_lds_addr(dst), voff[0], rsrc, soff);
      pp_dma(pp_lds_addr(dst + 64), voff[1], rsrc, soff);
    }
  };
  constexpr int kLoads = 4;  // DMA loads per wave per step
  // VMEM operations younger than a step's loads at its wait: the stores of
  // kLeadSteps steps and the loads of kLeadSteps - 1
  constexpr int kWaitN = kLeadSteps * kStores + (kLeadSteps - 1) * kLoads;
  static_assert(kWaitN <= 63, "vmcnt is 6 bits");
  // source rows of step t: the image rows its base row pass needs (octave 0)
  // or its base rows (octave > 0)
  auto src_row = [&](int t) { return Ystart + kPB * t + (OCT0 ? kPB : 0); };

  const int s0 = OCT0 ? -2 : 0;
  auto ring_slot = [](int t) { return (t + 4 * kRing) % kRing; };  // t >= -2
  // steps s0 .. s0 + kLeadSteps - 1 in flight, each followed by kStores
  // dropped stores so every wait below sees exactly kWaitN younger operations
#pragma unroll
  for (int i = 0; i < kLeadSteps; ++i) {
    issue(src_row(s0 + i), ring_slot(s0 + i));
    pp_pad<kStores>(r0);
  }
  for (int s = s0; s < nsteps; ++s) {
    const int Ys = Ystart + kPB * s;
    const int buf = s & 1;
    const int slot = ring_slot(s);
    // ---- this step's source rows have landed (own loads: vmcnt; the other
    // wave's: the barrier); slot (s + kLeadSteps) % kRing was read in step s - 1 ----
    PP_WAIT(kWaitN);
    pp_barrier();
    issue(src_row(s + kLeadSteps), ring_slot(s + kLeadSteps));
    if constexpr (OCT0) {
      PairLds0& L = *static_cast<PairLds0*>(ldsv);
      // ---- base row pass: ring rows [Ys + 4, Ys + 8) ----
      if (t < kPB * (kBC / 4)) {
        const int j = t / (kBC / 4), i = t - j * (kBC / 4);
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
        float hv[4];  // k outer, columns inner (see the scale row pass)
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
        const int slot = (kPB * (s + 3) + j) % kHbRows;  // ring slot of row Ys + 4 + j (s >= -2)
        *reinterpret_cast<float4*>(&L.hb[slot][4 * i]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
      }
      pp_barrier();
      // ---- base column pass: base rows [Ys, Ys + 4), plane 0 ----
      // Every thread runs it in every step (threads past the 100 base columns
      // on a clamped column, writing the row padding; the prologue steps s < 0
      // on ring rows not yet written, into a base buffer step s + 2 rewrites,
      // with rows above the chunk, so their stores drop), so every wave issues
      // exactly 4 stores here -- the count PP_WAIT relies on.
      {
        const int tc = min(t, kBC - 1);
        const int q0 = (kPB * s + 4) % kHbRows;  // slot of ring row Ys - 4
        float hv[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) {
          const int sl = q0 + q;
          hv[q] = L.hb[sl >= kHbRows ? sl - kHbRows : sl][tc];
        }
        const int xb = x0 - kPH + t;
        const unsigned v0 = (t >= kPH && t < kPH + kPW && xb < cols) ? (unsigned)xb * 4u : kDropV;
        const bool cpad = t < kBC && xb >= 0 && xb < cols - 1;
        float bv[kPB];  // k outer, rows inner (see the scale row pass)
#pragma unroll
        for (int j = 0; j < kPB; ++j) bv[j] = kFastT0[0] * hv[4 + j];
#pragma unroll
        for (int k = 1; k <= 4; ++k) {
          float pk[kPB];
#pragma unroll
          for (int j = 0; j < kPB; ++j) pk[j] = hv[4 + j - k] + hv[4 + j + k];
          asm volatile("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
          for (int j = 0; j < kPB; ++j) bv[j] = fmaf(kFastT0[k], pk[j], bv[j]);
        }
#pragma unroll
        for (int j = 0; j < kPB; ++j) {
          const float v = bv[j];
          const int y = Ys + j;
          pp_store_s(r0, v0, (y >= y0 && y < y1) ? (unsigned)(y * A.pitch * 4) : kDropV, v);
          L.base[buf][j][t] = (cpad && y >= 0 && y < rows - 1) ? v : 0.f;
        }
      }
      pp_barrier();
    }
    // The prologue steps s < 0 (octave 0) run the scale passes too, on
    // garbage base rows: every output row they touch lies above the chunk (its
    // store drops), and a stored output's accumulator starts with an
    // assignment at row y - w >= Ystart + 2 (step >= 0).  So every step issues
    // the same stores, with no branch for the PP_WAIT count to depend on.
    // ---- row passes of this wave's two scales: h rows [Ys, Ys + 4) ----
    float (*hbuf)[kPB][kPW];
    const float* brow;
    if constexpr (OCT0) {
      PairLds0& L = *static_cast<PairLds0*>(ldsv);
      hbuf = L.h[wv];
      brow = &L.base[buf][lane >> 4][4 * (lane & 15)];
    } else {
      PairLdsN& L = *static_cast<PairLdsN*>(ldsv);
      hbuf = L.h[wv];
      brow = &L.base[slot][lane >> 4][4 * (lane & 15)];
    }
    {
      const float4* p = reinterpret_cast<const float4*>(brow);
      // The role's window [kPH - WA, kPH + 3 + WA] in whole 16-B reads (every
      // component kept live, so hipcc cannot narrow a read to a misaligned
      // ds_read2_b64: 2-way bank conflicts).  PP_LAZY: each read is issued
      // kLazyD taps before the tap that first needs it and a chunk dies with
      // its last tap, so ~16 window registers are live instead of 40.
      float4 ch[10];
      constexpr int qlo = (kPH - WA) / 4, qhi = (kPH + 3 + WA) / 4;
      auto first_tap = [](int q) {  // first tap k whose pair sums read chunk q
        int m = 1 << 20;
        for (int e = 4 * q; e < 4 * q + 4; ++e) m = min(m, e < kPH ? kPH - e : max(e - kPH - 3, 0));
        return m;
      };
      auto load = [&](int q) {
        float4 f = (PP_ABL & 1) ? make_float4(lane + q, lane - q, lane * q, q) : p[q];
        asm("" : "+v"(f.x), "+v"(f.y), "+v"(f.z), "+v"(f.w));
        ch[q] = f;
      };
      auto loads_at = [&](int k) {  // the reads due at tap k
#pragma unroll
        for (int q = qlo; q <= qhi; ++q)
          if (PP_LAZY ? max(first_tap(q) - kLazyD, 0) == k : k == 0) load(q);
        if (PP_LAZY) asm volatile("" ::: "memory");  // no hoisting across taps
      };
      auto v = [&](int e) -> float {
        const float4& c = ch[e >> 2];
        return (e & 3) == 0 ? c.x : (e & 3) == 1 ? c.y : (e & 3) == 2 ? c.z : c.w;
      };
      // k outer, the 4 columns inner: the 4 pair sums of a tap, then the 8
      // fma of the 8 chains -- every instruction's operands were produced >= 4
      // instructions earlier (column-outer order made hipcc issue each fma
      // right behind the add or fma it depends on: 0.44 of the VALU issue rate)
      loads_at(0);
      float ha[4], hb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ha[u] = ptap<WA>(0) * v(kPH + u);
        hb[u] = ptap<WB>(0) * v(kPH + u);
      }
#pragma unroll
      for (int k = 1; k <= WA; ++k) {
        loads_at(k);
        float pk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pk[u] = v(kPH + u - k) + v(kPH + u + k);
        asm volatile("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          ha[u] = fmaf(ptap<WA>(k), pk[u], ha[u]);
          if (k <= WB) hb[u] = fmaf(ptap<WB>(k), pk[u], hb[u]);
        }
      }
      const int j = lane >> 4, i = lane & 15;
      *reinterpret_cast<float4*>(&hbuf[0][j][4 * i]) = make_float4(ha[0], ha[1], ha[2], ha[3]);
      *reinterpret_cast<float4*>(&hbuf[1][j][4 * i]) = make_float4(hb[0], hb[1], hb[2], hb[3]);
    }
    pp_wave_sync();
    // ---- column passes: lane = column ----
    float ha[kPB], hb[kPB];
#pragma unroll
    for (int j = 0; j < kPB; ++j) {
      ha[j] = hbuf[0][j][lane];
      hb[j] = hbuf[1][j][lane];
    }
    pp_wave_sync();
    o.Ys = Ys;
    float oa[kPB], ob[kPB];
    pp_dispatch<WA, WB>((s + kPer) % kPer, aa, ab, ha, hb, oa, ob);  // s >= -2
    pp_stores<WA, WB>(oa, ob, o);
  }
  PP_WAIT(0);  // the last (unused) loads land before the wave ends
}

#undef PP_WAIT

template <bool OCT0>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(PP_WPE))) void pyr_pair_kernel(PairArgs A) {
  __shared__ __attribute__((aligned(16))) char lds[OCT0 ? sizeof(PairLds0) : sizeof(PairLdsN)];
  // XCD-aware order (speed only): blocks b and b + 8 share an XCD, so XCD x
  // takes the contiguous run [x G/8, (x+1) G/8) of (image, chunk, strip) items
  // and neighbouring strips, which read each other's halo columns, meet in
  // one L2.
  const int per = (int)(gridDim.x >> 3);
  const int item = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (item >= A.items) return;
  const int strip = item % A.strips, rest = item / A.strips;
  const int ck = rest % A.chunks, b = rest / A.chunks;
  const int x0 = strip * kPW, y0 = ck * A.chunk, y1 = min(y0 + A.chunk, A.rows);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if PP_ROLE_ONLY == 1
  pp_walk<OCT0, 18, 4>(A, lds, wv, b, x0, y0, y1);
#elif PP_ROLE_ONLY == 2
  pp_walk<OCT0, 12, 8>(A, lds, wv, b, x0, y0, y1);
#else
  if (wv == 0)
    pp_walk<OCT0, 18, 4>(A, lds, 0, b, x0, y0, y1);
  else
    pp_walk<OCT0, 12, 8>(A, lds, 1, b, x0, y0, y1);
#endif
}

}  // namespace

bool pair_taps_match(const void* coef) {
  // the FastCoefs block of pyramid_fast.hip: base[9], s1[9], s2[17], s3[25], s4[37]
  const float* f = static_cast<const float*>(coef);
  const int ws[5] = {4, 4, 8, 12, 18};
  const float* tabs[5] = {kFastT0, kFastT1, kFastT2, kFastT3, kFastT4};
  size_t at = 0;
  for (int t = 0; t < 5; ++t) {
    const int w = ws[t];
    for (int a = -w; a <= w; ++a) {
      const float k = tabs[t][a < 0 ? -a : a];
      if (__builtin_memcmp(&k, &f[at + a + w], 4) != 0) return false;
    }
    at += 2 * w + 1;
  }
  return true;
}

// Octave o of the pyramid, all five planes (and the next octave's plane 0
// when it is an exact half, see pyramid_pair_fuses).  src: octave 0's input
// images (ignored for o > 0: the source is plane 0 of octave o).
void launch_pyramid_pair(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch) {
  const Octave& O = L.oct[o];
  PairArgs A{};
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
  A.strips = (O.cols + kPW - 1) / kPW;
  const int resident = resident_grid(o > 0 ? (const void*)pyr_pair_kernel<false> : (const void*)pyr_pair_kernel<true>,
                                     128, 0, 2048);
  // chunk count: every chunk walks kLead + kPH + 2 rows it does not output
  // (plus 8 for octave 0's base lead), and the grid runs in rounds of
  // `resident` workgroups: minimise rounds x rows walked per chunk
  const long long per = (long long)A.strips * batch;
  int ch = 0;
  double best = 0;
  for (int c = 1; c <= (O.rows + kPB - 1) / kPB; ++c) {
    const int h = ((O.rows + c - 1) / c + kPB - 1) / kPB * kPB;
    const int cc = (O.rows + h - 1) / h;
    const double rounds = (double)((per * cc + resident - 1) / resident);
    const double cost = rounds * (h + kLead + kPH + 2 + (o == 0 ? 8 : 0));
    if (ch == 0 || cost < best - 1e-9) {
      best = cost;
      ch = h;
    }
  }
  A.chunk = ch;
  A.chunks = (O.rows + ch - 1) / ch;
  A.items = (int)(per * A.chunks);
  const int grid = (A.items + 7) / 8 * 8;
  if (o > 0)
    hipLaunchKernelGGL((pyr_pair_kernel<false>), dim3(grid), dim3(128), 0, st, A);
  else
    hipLaunchKernelGGL((pyr_pair_kernel<true>), dim3(grid), dim3(128), 0, st, A);
}

// Octave o's plane 0 comes out of octave o-1's launch when it is exactly the
// (2y, 2x) half (resize INTER_NEAREST with both scale factors exactly 2).
bool pyramid_pair_fuses(const Layout& L, int o) {
  return o > 0 && L.oct[o - 1].rows == 2 * L.oct[o].rows && L.oct[o - 1].cols == 2 * L.oct[o].cols;
}

}  // namespace sift
