// pyramid_pc.hip -- SIFT_FLAG_FAST Gaussian pyramid for gfx950: one producer
// wave and three consumer waves per workgroup, synchronised by LDS counters
// instead of workgroup barriers (round 5).
//
// The separable form of src/sift.cpp:229-263 (every scale blurred from its
// octave base with the reference's sigma, width floor(3 sigma) (:97) and zero
// padding outside [0, rows-1) x [0, cols-1) (:116)) in exactly the operation
// order of oracle/sift_oracle.c's so_fast_pyramid, so the planes are its bits
// (tests/test_gpu_fast.py).
//
// Why this structure (profiles/r5_tri_stamps.txt, r5_tri_ablation.txt): the
// previous kernel's three roles (rounds 3-4, removed; git history at commit
// 319d385) met at one s_barrier per step; role 0 (w = 18) waited there 37 %
// of its time while the io roles ran the octave-0 base blur, and the io roles'
// vmcnt wait for their own source rows also waited for every older plane
// store.
//
//  * Workgroup = 4 waves over a 64-column strip and a chunk of rows, 8 rows
//    per step:
//      wave 0 (producer): brings the octave base rows into a ring of kPD
//        steps in LDS -- octave 0: LDS-DMA of image rows, the base blur
//        (createInitialImage, w = 4) row and column passes over the strip's
//        100 base columns, plane 0 stored; octaves > 0: LDS-DMA of plane-0
//        rows straight into the ring, two steps ahead, and the w = 18 scale's
//        row pass into the h18 ring (hpub / hdone counters) -- above octave 0
//        that wave would otherwise idle while the w = 18 consumer is the pole;
//      waves 1-3 (consumers): plane 4 (w = 18), plane 3 (w = 12), planes 2
//        and 1 (w = 8, 4, pair sums shared) + the next octave's decimated
//        plane 0: row pass from the ring (w = 18 above octave 0: from h18),
//        column pass scattered into register accumulators, dwordx4 plane
//        stores.
//  * LDS counters: the producer publishes `pub` = steps whose base rows are
//    in the ring; consumer c publishes done[c] = steps it has read.  A
//    consumer waits only for pub, the producer only for the slowest consumer
//    kPD - 1 steps back: waves drift against each other by up to kPD steps,
//    nobody waits at a workgroup barrier, and consumers never wait on vmcnt
//    (their stores are fire and forget).  Every wait is bounded (kPollMax):
//    on expiry the wave sets the sticky error word and goes on (garbage
//    planes, no hang).
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

constexpr int kPW = 64;              // output columns per strip
constexpr int kPH = 18;              // widest half-width
constexpr int kPB = 8;               // rows per step
constexpr int kPD = 4;               // base ring depth (steps)
constexpr int kPLead = 24;           // rows walked above the chunk (>= kPH + 2, multiple of kPB)
constexpr int kPPit = 128;           // base ring row pitch (floats; = 0 mod 64: conflict-free ds_read_b128)
constexpr int kPBC = kPW + 2 * kPH;  // 100 base columns per strip: [x0 - 18, x0 + 82)
constexpr int kPIW = 112;            // octave-0 image ring row: columns [x0 - 24, x0 + 88)
constexpr int kPHb = 104;            // octave-0 base row-pass ring row: columns [x0 - 20, x0 + 84)
constexpr int kPHbRows = 16;
constexpr int kPImg = 2;             // image ring slots (steps)
constexpr int kPollMax = 1 << 20;    // bound of every wait (~70 M cycles at s_sleep 1)
constexpr unsigned kPDropV = 0x7f000000u;  // one offset part past every plane (pyramid_fast_fits)

struct PcFlags {
  int pub;      // steps published by the producer (relative to the walk's first step)
  int done[3];  // steps consumed by each consumer
  int hpub;     // octaves > 0: steps whose w = 18 row pass the producer has written to h18
  int hdone;    // octaves > 0: steps whose h18 rows consumer 0 has read
};
constexpr int kPH18 = 3;  // octaves > 0: h18 ring depth (steps)
struct PcLds0 {  // octave 0: 32,272 B -> 5 workgroups per CU (96 VGPRs: 5 waves per SIMD)
  float base[kPD][kPB][kPPit];
  float img[kPImg][kPB][kPIW];
  float hb[kPHbRows][kPHb];
  float tr0[kPB][kPW];   // producer's plane-0 store transpose
  PcFlags f;
};
struct PcLdsN {  // octave > 0: 22,552 B
  float base[kPD][kPB][kPPit];
  float h18[kPH18][kPB][kPW];  // w = 18 row-pass output, lane = column 4i + R (pc_xpose4 layout)
  PcFlags f;
};
static_assert(sizeof(PcLds0) * 5 <= 163840, "five octave-0 workgroups per CU");

typedef __amdgpu_buffer_rsrc_t PRsrc;
typedef unsigned pu32x4 __attribute__((ext_vector_type(4)));
typedef unsigned pu32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ PRsrc pc_rsrc(const float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void pc_store4(PRsrc rs, unsigned voff, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pu32x4, v), rs, (int)voff, 0, 0);
}
__device__ __forceinline__ void pc_store2(PRsrc rs, unsigned voff, float a, float b) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(pu32x2, make_float2(a, b)), rs, (int)voff, 0, 0);
}
// LDS-DMA: lane l's dword lands at M0 + 4l
__device__ __forceinline__ void pc_dma(unsigned lds_byte, unsigned voff, PRsrc rs, unsigned soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, %3 offen lds"
               ::"s"(lds_byte), "v"(voff), "s"(rs), "s"(soff) : "memory", "m0");
}
__device__ __forceinline__ unsigned pc_lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) float*)p);
}
// Lanes of one wave hand data through LDS: the wave's LDS operations run in
// program order, so only the compiler needs fencing.
__device__ __forceinline__ void pc_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  asm volatile("" ::: "memory");
}
#define PC_WAIT_VM(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")

// 4 x 4 transpose across the wave's four 16-lane rows, in registers: lane
// (R = lane >> 4, i = lane & 15) holding a[u] = X[R][u] ends with a[k] =
// X[k][R] (v_permlane32_swap swaps rows 2-3 of its first operand with rows
// 0-1 of its second, v_permlane16_swap odd rows of the first with even rows
// of the second; checked by tools/permlane_check.hip).  It turns the row
// pass's (row, 4 columns) lanes into (column 4i + R, 4 rows) lanes and the
// column pass's outputs back into 4 consecutive columns of one row for a
// dwordx4 store: 4 VALU instead of an LDS write, a wait and reads.
__device__ __forceinline__ void pc_xpose4(float (&a)[4]) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[0]), __float_as_uint(a[2]), false, false);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[1]), __float_as_uint(a[3]), false, false);
  const auto r = __builtin_amdgcn_permlane16_swap(p[0], q[0], false, false);
  const auto t = __builtin_amdgcn_permlane16_swap(p[1], q[1], false, false);
  a[0] = __uint_as_float(r[0]);
  a[1] = __uint_as_float(r[1]);
  a[2] = __uint_as_float(t[0]);
  a[3] = __uint_as_float(t[1]);
}

// Counters: a plain LDS word written by one wave, polled by others.  The
// writer drains its earlier LDS operations first (s_waitcnt lgkmcnt(0)), so a
// reader that sees the new value sees the data written before it.
__device__ __forceinline__ void pc_publish(int* w, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int pc_peek(const int* w) {
  return __hip_atomic_load(const_cast<int*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Wait until *w >= v (bounded); then the caller's later LDS reads see what was
// written before the matching publish.
__device__ __forceinline__ void pc_wait_ge(const int* w, int v, int* err, int poll_max) {
  int it = 0;
  while (pc_peek(w) < v) {
    if (++it > poll_max) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void pc_wait_done(const PcFlags& f, int v, int* err, int poll_max) {
  int it = 0;
  while (min(min(pc_peek(&f.done[0]), pc_peek(&f.done[1])), pc_peek(&f.done[2])) < v) {
    if (++it > poll_max) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int W>
__host__ __device__ constexpr float ptap(int k) {
  return W == 18 ? kFastT4[k] : W == 12 ? kFastT3[k] : W == 8 ? kFastT2[k] : W == 4 ? kFastT1[k] : kFastT0[k];
}

// Consumer roles: scales (W2 = 0 for one), accumulator slots P (the smallest
// multiple of kPB >= 2w + 1; role 2's two scales share the larger cycle), NC
// = P / kPB steps per slot cycle, planes.
template <int C> struct PcRole;
template <> struct PcRole<0> {
  static constexpr int W1 = 18, W2 = 0, P1 = 40, P2 = 1, NC = 5, pl1 = 4, pl2 = 0;
};
template <> struct PcRole<1> {
  static constexpr int W1 = 12, W2 = 0, P1 = 32, P2 = 1, NC = 4, pl1 = 3, pl2 = 0;
};
template <> struct PcRole<2> {
  static constexpr int W1 = 8, W2 = 4, P1 = 24, P2 = 12, NC = 3, pl1 = 2, pl2 = 1;
};
static_assert(PcRole<2>::pl1 == kLayers, "the decimated plane (nOctaveLayers) is role 2's first scale");

// Column pass of one source row at cycle row R: output R - d gets g_|d| h,
// d = -W..W, slot (R - d) mod P; d = -W is that output's first term.
template <int W, int P, int R, int D>
__device__ __forceinline__ void pc_fma_one(float (&acc)[P], float h) {
  constexpr int slot = ((R - D) % P + P) % P;
  constexpr unsigned bits = __builtin_bit_cast(unsigned, ptap<W>(D < 0 ? -D : D));
  if constexpr (D == -W)
    asm("v_mul_f32 %0, %2, %1" : "=v"(acc[slot]) : "v"(h), "n"(bits));
  else
    asm("v_fmac_f32 %0, %2, %1" : "+v"(acc[slot]) : "v"(h), "n"(bits));
}
template <int W, int P, int R, int... I>
__device__ __forceinline__ void pc_scatter(float (&acc)[P], float h, std::integer_sequence<int, I...>) {
  (pc_fma_one<W, P, R, I - W>(acc, h), ...);
}
// Column pass of a step at cycle phase M: rows J = 0..7 scatter in order;
// output row 8M + J - W (slot mod P) is complete after row J.
template <int W, int P, int M, int... J>
__device__ __forceinline__ void pc_col(float (&acc)[P], const float (&c)[kPB], float (&o)[kPB],
                                       std::integer_sequence<int, J...>) {
  ((pc_scatter<W, P, kPB * M + J>(acc, c[J], std::make_integer_sequence<int, 2 * W + 1>{}),
    o[J] = acc[((kPB * M + J - W) % P + P) % P]),
   ...);
}
template <class F, int... M>
__device__ __forceinline__ bool pc_cycle(F&& f, std::integer_sequence<int, M...>) {
  return (f(std::integral_constant<int, M>{}) && ...);
}

// Row pass of scales W1 (and W2) for ring row `brow` (column kPH + u is output
// column 4i + u of the lane's group), pair sums shared by the two scales.
template <int W1, int W2>
__device__ __forceinline__ void pc_rows(const float* brow, float (&h1)[4], float (&h2)[4]) {
  const float4* p = reinterpret_cast<const float4*>(brow);
  constexpr int qlo = (kPH - W1) / 4, qhi = (kPH + 3 + W1) / 4;
  float v[40];
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    if (q < qlo || q > qhi) {
      v[4 * q] = v[4 * q + 1] = v[4 * q + 2] = v[4 * q + 3] = 0.f;
      continue;
    }
    float4 f = p[q];
    asm("" : "+v"(f.x), "+v"(f.y), "+v"(f.z), "+v"(f.w));  // whole b128 reads
    v[4 * q] = f.x;
    v[4 * q + 1] = f.y;
    v[4 * q + 2] = f.z;
    v[4 * q + 3] = f.w;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    h1[u] = ptap<W1>(0) * v[kPH + u];
    if (W2) h2[u] = ptap<W2>(0) * v[kPH + u];
  }
#pragma unroll
  for (int k = 1; k <= W1; ++k) {
    float pk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) pk[u] = v[kPH + u - k] + v[kPH + u + k];
    asm volatile("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      h1[u] = fmaf(ptap<W1>(k), pk[u], h1[u]);
      if (k <= W2) h2[u] = fmaf(ptap<W2>(k), pk[u], h2[u]);
    }
  }
}

}  // namespace

struct PcArgs {
  float* gpyr;
  long long g_img;
  long long off[kScales];  // plane offsets of this octave in the image block
  const float* src;        // octave 0: the input images; else this octave's plane 0
  long long s_pitch, s_img;
  long long nxt_off;       // next octave's plane 0 (fused decimation), or -1
  int n_pitch, n_rows, n_cols;
  int pitch, rows, cols;
  int strips, columns;
  int n_full, grid_full;
  int chunk, chunks;
  int* err;                // sticky error word err[3] (kErrStall: a bounded wait expired)
};

namespace {

// ---- producer, octave 0: the base blur of the strip's 100 base columns ----
// Step s (base rows [Ys, Ys + 8), Ys = Ystart + 8 s): row pass of image rows
// [Ys + 4, Ys + 12) (image slot s % kPImg, LDS-DMA'd during step s - 1) into
// the hb ring, column pass of hb rows [Ys - 4, Ys + 12) into base ring slot
// s % kPD (zero outside [0, rows-1) x [0, cols-1): getSubMatrix applied to the
// base as the scales' source) and plane 0 (columns [x0, x0 + 64), rows
// [y0, y1)).  Step -1 runs the row pass only (hb rows [Ys0 - 4, Ys0 + 4)).
template <int kPoll>
__device__ __forceinline__ void pc_producer0(const PcArgs& A, PcLds0& L, int b, int x0, int y0, int y1) {
  const int lane = threadIdx.x & 63;
  const int rows = A.rows, cols = A.cols;
  const int Ystart = y0 - kPLead;
  const int nsteps = (y1 + kPH - Ystart + kPB - 1) / kPB;
  float* const gimg = A.gpyr + b * A.g_img;
  const PRsrc r0 = pc_rsrc(gimg + A.off[0], (long long)A.rows * A.pitch * 4);
  const unsigned pitch4 = A.pitch * 4;
  const PRsrc rsrc = pc_rsrc(A.src + b * A.s_img, (long long)rows * A.s_pitch * 4);
  // image columns [x0 - 24, x0 + 88): lanes 0-63, then lanes 0-47
  unsigned voff[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int c = x0 - 24 + lane + 64 * hh;
    voff[hh] = (c >= 0 && c < cols - 1) ? (unsigned)c * 4u : kPDropV;
  }
  auto issue = [&](int s) {  // image rows [Ystart + 8 s + 4, + 8) -> image slot s % kPImg
    float* slot = &L.img[(s + 2 * kPImg) % kPImg][0][0];
#pragma unroll
    for (int i = 0; i < kPB; ++i) {
      const int r = Ystart + kPB * s + 4 + i;
      const unsigned soff = (r >= 0 && r < rows - 1) ? (unsigned)(r * A.s_pitch * 4) : kPDropV;
      pc_dma(pc_lds_addr(slot + i * kPIW), voff[0], rsrc, soff);
      if (lane < kPIW - 64) pc_dma(pc_lds_addr(slot + i * kPIW + 64), voff[1], rsrc, soff);
    }
  };
  auto hb_row = [&](int Y) { return (Y - Ystart + 4 * kPHbRows) & (kPHbRows - 1); };
  // row pass of image slot s: 8 rows x 26 column groups of 4 (208 tasks, 4
  // per lane); every window is read before any arithmetic (the producer's
  // step is latency-bound: profiles/r5_pc_stamps.txt)
  auto row_pass = [&](int s) {
    const int sl = (s + 2 * kPImg) % kPImg, Yr = Ystart + kPB * s + 4;
    constexpr int kTasks = kPB * (kPHb / 4), kIt = (kTasks + 63) / 64;
    float4 win[kIt][3];
#pragma unroll
    for (int t = 0; t < kIt; ++t) {
      const int it = min(64 * t + lane, kTasks - 1);
      const int j = it / (kPHb / 4), g = it - j * (kPHb / 4);
      // row-pass column 4g + u is image column x0 - 20 + 4g + u = ring column 4g + 4 + u
      const float4* p = reinterpret_cast<const float4*>(&L.img[sl][j][4 * g]);
#pragma unroll
      for (int q = 0; q < 3; ++q) win[t][q] = p[q];
    }
#pragma unroll
    for (int t = 0; t < kIt; ++t) {
      const int it = 64 * t + lane;
      const int itc = min(it, kTasks - 1);
      const int j = itc / (kPHb / 4), g = itc - j * (kPHb / 4);
      const float v[12] = {win[t][0].x, win[t][0].y, win[t][0].z, win[t][0].w, win[t][1].x, win[t][1].y,
                           win[t][1].z, win[t][1].w, win[t][2].x, win[t][2].y, win[t][2].z, win[t][2].w};
      float hv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) hv[u] = kFastT0[0] * v[4 + u];
#pragma unroll
      for (int k = 1; k <= 4; ++k) {
        float pk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pk[u] = v[4 + u - k] + v[4 + u + k];
        asm("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]));
#pragma unroll
        for (int u = 0; u < 4; ++u) hv[u] = fmaf(kFastT0[k], pk[u], hv[u]);
      }
      if (it < kTasks)
        *reinterpret_cast<float4*>(&L.hb[hb_row(Yr + j)][4 * g]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
    }
  };
  // plane-0 stores: lane = (row sr of a 4-row round, columns 4 sg .. + 3)
  const int sg = lane & 15, sr = lane >> 4, sx = x0 + 4 * sg;
  const bool sok = sx < cols;
  // VMEM operations per step, in issue order: step s + 1's image rows (2 per
  // row), then step s's plane-0 stores (kStores0)
  constexpr int kDma0 = 2 * kPB, kStores0 = kPB / 4;
  static_assert(kPIW > 64 && kPIW - 64 < 64, "two DMA instructions per image row");
  // prologue: image rows of steps -1 and 0
  issue(-1);
  issue(0);
  PC_WAIT_VM(kDma0);  // step -1's rows
  pc_wave_sync();
  row_pass(-1);
  for (int s = 0; s < nsteps; ++s) {
    const int Ys = Ystart + kPB * s;
    // step s's image rows landed; only the kStores0 plane-0 stores of step
    // s - 1 were issued after them and may stay in flight
    if (s == 0)
      PC_WAIT_VM(0);
    else
      PC_WAIT_VM(kStores0);
    pc_wave_sync();
    if (s + 1 < nsteps) issue(s + 1);  // into the slot step s - 1 used (its row pass is done)
    row_pass(s);
    // slot s % kPD is free once every consumer has read step s - kPD
    pc_wait_done(L.f, s - kPD + 1, A.err, kPoll);
    pc_wave_sync();
    float* const bslot = &L.base[s % kPD][0][0];
    // column pass: lane = base column bc (100: lanes 0-63, then 0-35), all
    // eight base rows from one 16-row window, every read issued first
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int bc = pass == 0 ? lane : min(64 + lane, kPBC - 1);
      const bool own = pass == 0 || lane < kPBC - 64;
      const int hc = bc + 2;         // hb column: image column x0 - 20 + hc
      const int xb = x0 - kPH + bc;  // image column of this base column
      const bool cpad = xb >= 0 && xb < cols - 1;
      const bool out0 = own && xb >= x0 && xb < x0 + kPW;
      float hv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) hv[q] = L.hb[hb_row(Ys - 4 + q)][hc];
      float bv[kPB];
#pragma unroll
      for (int j = 0; j < kPB; ++j) bv[j] = kFastT0[0] * hv[4 + j];
#pragma unroll
      for (int k = 1; k <= 4; ++k) {
        float pk[kPB];
#pragma unroll
        for (int j = 0; j < kPB; ++j) pk[j] = hv[4 + j - k] + hv[4 + j + k];
        asm("" : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]), "+v"(pk[4]), "+v"(pk[5]), "+v"(pk[6]),
            "+v"(pk[7]));
#pragma unroll
        for (int j = 0; j < kPB; ++j) bv[j] = fmaf(kFastT0[k], pk[j], bv[j]);
      }
#pragma unroll
      for (int j = 0; j < kPB; ++j) {
        const int y = Ys + j;
        if (own) bslot[j * kPPit + bc] = (cpad && y >= 0 && y < rows - 1) ? bv[j] : 0.f;
        if (out0) L.tr0[j][xb - x0] = bv[j];
      }
    }
    pc_publish(&L.f.pub, s + 1);
    pc_wave_sync();
#pragma unroll
    for (int r4 = 0; r4 < kPB; r4 += 4) {
      const float4 v = *reinterpret_cast<const float4*>(&L.tr0[r4 + sr][4 * sg]);
      const int y = Ys + r4 + sr;
      pc_store4(r0, (sok && y >= y0 && y < y1) ? (unsigned)y * pitch4 + (unsigned)sx * 4u : kPDropV, v);
    }
    pc_wave_sync();  // tr0 reads before the next step's writes (program order)
  }
}

// ---- producer, octave > 0: plane-0 rows by LDS-DMA straight into the ring,
// two steps ahead ----
template <int kPoll>
__device__ __forceinline__ void pc_producerN(const PcArgs& A, PcLdsN& L, int b, int x0, int y0, int y1) {
  const int lane = threadIdx.x & 63;
  const int rows = A.rows, cols = A.cols;
  const int Ystart = y0 - kPLead;
  const int nsteps = (y1 + kPH - Ystart + kPB - 1) / kPB;
  const PRsrc rsrc = pc_rsrc(A.src + b * A.s_img, (long long)rows * A.s_pitch * 4);
  unsigned voff[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int c = x0 - kPH + lane + 64 * hh;
    voff[hh] = (c >= 0 && c < cols - 1) ? (unsigned)c * 4u : kPDropV;
  }
  auto issue = [&](int s) {
    float* slot = &L.base[s % kPD][0][0];
#pragma unroll
    for (int i = 0; i < kPB; ++i) {
      const int r = Ystart + kPB * s + i;
      const unsigned soff = (r >= 0 && r < rows - 1) ? (unsigned)(r * A.s_pitch * 4) : kPDropV;
      pc_dma(pc_lds_addr(slot + i * kPPit), voff[0], rsrc, soff);
      if (lane < kPBC - 64) pc_dma(pc_lds_addr(slot + i * kPPit + 64), voff[1], rsrc, soff);
    }
  };
  constexpr int kPerStep = 2 * kPB;  // DMA instructions per step
  issue(0);
  if (nsteps > 1) issue(1);
  for (int s = 0; s < nsteps; ++s) {
    const int Ys = Ystart + kPB * s;
    // step s's rows landed: everything but step s + 1's loads (if issued)
    if (s + 1 < nsteps)
      PC_WAIT_VM(kPerStep);
    else
      PC_WAIT_VM(0);
    pc_publish(&L.f.pub, s + 1);
    // The w = 18 row pass (consumer 0's, which would otherwise be the pole of
    // every octave > 0 -- profiles/r5_pc_stamps.txt -- while this wave idles)
    // into h18 slot s % kPH18, read by consumer 0 as lane = column 4i + R
    if (Ys + kPB - 1 + kPH >= y0 && Ys - kPH < y1) {
      pc_wait_ge(&L.f.hdone, s - kPH18 + 1, A.err, kPoll);
      const float* brow = &L.base[s % kPD][lane >> 4][4 * (lane & 15)];
      float* hs = &L.h18[s % kPH18][0][0];
#pragma unroll
      for (int r4 = 0; r4 < kPB; r4 += 4) {
        float h1[4], h2[4];
        pc_rows<kPH, 0>(brow + r4 * kPPit, h1, h2);
        pc_xpose4(h1);
#pragma unroll
        for (int k = 0; k < 4; ++k) hs[(r4 + k) * kPW + lane] = h1[k];
      }
    }
    pc_publish(&L.f.hpub, s + 1);
    if (s + 2 < nsteps) {
      pc_wait_done(L.f, s + 2 - kPD + 1, A.err, kPoll);  // slot (s + 2) % kPD free
      issue(s + 2);
    }
  }
}

// ---- consumer C: its scales over the strip, reading the ring ----
template <bool OCT0, int C, int kPoll, class LdsT>
__device__ __forceinline__ void pc_consumer(const PcArgs& A, LdsT& L, int b, int x0, int y0, int y1) {
  using R_ = PcRole<C>;
  constexpr int W1 = R_::W1, W2 = R_::W2, P1 = R_::P1, P2 = R_::P2, NC = R_::NC;
  constexpr bool kDec = C == 2;
  const int lane = threadIdx.x & 63;
  float* const gimg = A.gpyr + b * A.g_img;
  const long long plane_bytes = (long long)A.rows * A.pitch * 4;
  const PRsrc ra = pc_rsrc(gimg + A.off[R_::pl1], plane_bytes);
  const PRsrc rb = pc_rsrc(gimg + A.off[R_::pl2], W2 ? plane_bytes : 0);
  const bool nxt = kDec && A.nxt_off >= 0;
  const PRsrc rn = pc_rsrc(gimg + (nxt ? A.nxt_off : 0), nxt ? (long long)A.n_rows * A.n_pitch * 4 : 0);
  const unsigned pitch4 = A.pitch * 4, n_pitch4 = A.n_pitch * 4;
  // wide stores: lane = (row lane >> 4 of a 4-row round, columns xg .. xg + 3);
  // a group past cols writes the row's pitch padding (common.hpp, kPitchAlign)
  const int sr = lane >> 4, xg = x0 + 4 * (lane & 15);
  const bool xok = xg < A.cols;
  const int Ystart = y0 - kPLead;
  const int nsteps = (y1 + kPH - Ystart + kPB - 1) / kPB;
  float a1[P1], a2[P2];
#pragma unroll
  for (int k = 0; k < P1; ++k) a1[k] = 0.f;
#pragma unroll
  for (int k = 0; k < P2; ++k) a2[k] = 0.f;
  int s = 0;
  auto step = [&](auto Mc) -> bool {
    constexpr int M = decltype(Mc)::value;
    if (s >= nsteps) return false;
    __builtin_amdgcn_sched_barrier(0);  // steps do not interleave (register pressure)
    const int Ys = Ystart + kPB * s;
    // the step's source rows [Ys, Ys + 8) reach outputs [Ys - W1, Ys + 7 + W1] only
    const bool live = Ys + kPB - 1 + W1 >= y0 && Ys - W1 < y1;
    if (live) {
      float c1[kPB], c2[kPB], o1[kPB], o2[kPB];
      if constexpr (!OCT0 && C == 0) {
        // octaves > 0: the producer ran this scale's row pass (pc_producerN)
        pc_wait_ge(&L.f.hpub, s + 1, A.err, kPoll);
        const float* hs = &reinterpret_cast<PcLdsN&>(L).h18[s % kPH18][0][0];
#pragma unroll
        for (int j = 0; j < kPB; ++j) c1[j] = hs[j * kPW + lane];
      } else {
      pc_wait_ge(&L.f.pub, s + 1, A.err, kPoll);
      const float* brow = &L.base[s % kPD][lane >> 4][4 * (lane & 15)];
      // ---- row pass (lane = row R, 4 columns), two rounds of 4 rows, turned
      // into lane = column 4i + R by the register transpose ----
#pragma unroll
      for (int r4 = 0; r4 < kPB; r4 += 4) {
        float h1[4], h2[4];
        pc_rows<W1, W2>(brow + r4 * kPPit, h1, h2);
        pc_xpose4(h1);
#pragma unroll
        for (int k = 0; k < 4; ++k) c1[r4 + k] = h1[k];
        if constexpr (W2 != 0) {
          pc_xpose4(h2);
#pragma unroll
          for (int k = 0; k < 4; ++k) c2[r4 + k] = h2[k];
        }
      }
      }
      // ---- column pass (lane = column 4i + R), phase M of the role's slot cycle ----
      pc_col<W1, P1, M>(a1, c1, o1, std::make_integer_sequence<int, kPB>{});
      if constexpr (W2 != 0) pc_col<W2, P2, M>(a2, c2, o2, std::make_integer_sequence<int, kPB>{});
      // ---- stores: transposed back, a lane stores 4 columns of row r4 + R ----
#pragma unroll
      for (int r4 = 0; r4 < kPB; r4 += 4) {
        float t1[4] = {o1[r4], o1[r4 + 1], o1[r4 + 2], o1[r4 + 3]};
        pc_xpose4(t1);
        const float4 v1 = make_float4(t1[0], t1[1], t1[2], t1[3]);
        const int ya = Ys + r4 + sr - W1;  // this lane's output row
        pc_store4(ra, (xok && ya >= y0 && ya < y1) ? (unsigned)ya * pitch4 + (unsigned)xg * 4u : kPDropV, v1);
        if constexpr (W2 != 0) {
          float t2[4] = {o2[r4], o2[r4 + 1], o2[r4 + 2], o2[r4 + 3]};
          pc_xpose4(t2);
          const int yb = Ys + r4 + sr - W2;
          pc_store4(rb, (xok && yb >= y0 && yb < y1) ? (unsigned)yb * pitch4 + (unsigned)xg * 4u : kPDropV,
                    make_float4(t2[0], t2[1], t2[2], t2[3]));
        }
        if constexpr (kDec) {  // plane nOctaveLayers (src/sift.cpp:252) -> next octave's plane 0 at (y/2, x/2)
          const bool dn = xok && (ya & 1) == 0 && ya >= y0 && ya < y1;
          pc_store2(rn, dn ? (unsigned)(ya >> 1) * n_pitch4 + (unsigned)(xg >> 1) * 4u : kPDropV, v1.x, v1.z);
        }
      }
    }
    // every ring (h18) read of this step has been consumed: the slot may be refilled
    if constexpr (!OCT0 && C == 0)
      pc_publish(&L.f.hdone, s + 1);
    else
      pc_publish(&L.f.done[C], s + 1);
    ++s;
    return true;
  };
  while (pc_cycle(step, std::make_integer_sequence<int, NC>{})) {
  }
  pc_publish(&L.f.done[C], 1 << 30);  // never the producer's bottleneck again
  if constexpr (!OCT0 && C == 0) pc_publish(&L.f.hdone, 1 << 30);
}

// kPoll: the bound of every LDS-counter wait -- kPollMax, or 0 for the test
// hook pc_stall_once (every wait that is not already satisfied expires: the
// stall path without a hang; a separate instance, so the shipped ones keep
// their registers and vmcnt accounting, tools/check_pc_isa.py)
template <bool OCT0, int kPoll = kPollMax>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void pyr_pc_kernel(PcArgs A) {
  __shared__ __attribute__((aligned(16))) char lds[OCT0 ? sizeof(PcLds0) : sizeof(PcLdsN)];
  using LdsT = typename std::conditional<OCT0, PcLds0, PcLdsN>::type;
  LdsT& L = *reinterpret_cast<LdsT*>(lds);
  // XCD-aware order within each phase (speed only): blocks b and b + 8 share
  // an XCD, so XCD x takes a contiguous run of the phase's items and
  // neighbouring strips, which read each other's halo columns, meet in one L2.
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
  const int b = col / A.strips, x0 = (col - b * A.strips) * kPW;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x == 0) {
    L.f.pub = L.f.hpub = L.f.hdone = 0;
    L.f.done[0] = OCT0 ? 0 : 1 << 30;  // octaves > 0: consumer 0 reads h18, not the ring
    L.f.done[1] = L.f.done[2] = 0;
  }
  __syncthreads();  // the one workgroup barrier: counters initialised
  if (wv == 0) {
    if constexpr (OCT0)
      pc_producer0<kPoll>(A, L, b, x0, y0, y1);
    else
      pc_producerN<kPoll>(A, L, b, x0, y0, y1);
    PC_WAIT_VM(0);  // the last loads land before the wave ends
  } else if (wv == 1) {
    pc_consumer<OCT0, 0, kPoll>(A, L, b, x0, y0, y1);
  } else if (wv == 2) {
    pc_consumer<OCT0, 1, kPoll>(A, L, b, x0, y0, y1);
  } else {
    pc_consumer<OCT0, 2, kPoll>(A, L, b, x0, y0, y1);
  }
}

#undef PC_WAIT_VM

}  // namespace

bool pyramid_fuses_decimation(const Layout& L, int o) {
  return o > 0 && L.oct[o - 1].rows == 2 * L.oct[o].rows && L.oct[o - 1].cols == 2 * L.oct[o].cols;
}

bool pyramid_fast_fits(const Layout& L, long long src_row_stride) {
  // every plane and the input rows below the dropped-offset part (octave 0 is
  // the largest plane), and the input's row offsets in 32 bits
  const long long plane = (long long)L.oct[0].rows * L.oct[0].pitch * 4;
  const long long srcb = (long long)L.oct[0].rows * src_row_stride * 4;
  return plane < (long long)kPDropV && srcb < (long long)kPDropV;
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
FastPlan fast_plan(int columns, int rows, int slots, int halo) {
  static std::mutex mu;
  static std::map<std::array<int, 4>, FastPlan> cache;
  const std::array<int, 4> key{columns, rows, slots, halo};
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  FastPlan best{columns, rows, 1};
  long long best_cost = -1, best_items = 0;
  std::vector<int> fulls;
  for (long long f = 0; f < columns; f += slots) fulls.push_back((int)f);
  fulls.push_back(columns);
  for (int nf : fulls)
    for (int c = 1; c <= (nf == columns ? 1 : 32); ++c) {
      const int ch = nf == columns ? rows : ((rows + c - 1) / c + kPB - 1) / kPB * kPB;
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
        best = FastPlan{nf, ch, cc};
      }
    }
  // A chunked plan that fits one round starts every workgroup at once, and
  // they then run their phases in lockstep (all DMA, then all arithmetic):
  // one 8K image's octave 0 (1,200 items on 1,280 slots) ran 5 % faster with
  // twice the chunks (0.397-0.401 vs 0.417-0.422 ms of pyramid,
  // profiles/r5_pc_chunks_ab.txt), while three times was slower and the
  // many-round 64 x 1080p plans do not change.  So such a plan takes twice
  // the chunks when they stay at least twice the halo tall.
  if (best.n_full < columns && (long long)(columns - best.n_full) * best.chunks + best.n_full <= slots) {
    const int ch2 = ((rows + 2 * best.chunks - 1) / (2 * best.chunks) + kPB - 1) / kPB * kPB;
    if (ch2 >= 2 * halo) best = FastPlan{best.n_full, ch2, (rows + ch2 - 1) / ch2};
  }
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = best;
  return best;
}

// Octave o of the pyramid, all five planes, and the next octave's plane 0 when
// it is an exact half (pyramid_fuses_decimation).  src: octave 0's input
// images (ignored for o > 0: the source is plane 0 of octave o).
void launch_pyramid_pc(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch, int* err,
                       bool stall_test) {
  const Octave& O = L.oct[o];
  PcArgs A{};
  A.gpyr = gpyr;
  A.g_img = L.g_img;
  for (int s = 0; s < kScales; ++s) A.off[s] = O.g_off[s];
  A.pitch = O.pitch;
  A.rows = O.rows;
  A.cols = O.cols;
  A.err = err;
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
  A.strips = (O.cols + kPW - 1) / kPW;
  A.columns = A.strips * batch;
  const int resident = resident_grid(o > 0 ? (const void*)pyr_pc_kernel<false> : (const void*)pyr_pc_kernel<true>,
                                     256, 0, 1024);
  const FastPlan P = fast_plan(A.columns, O.rows, resident, kPLead + kPH + 2 + (o == 0 ? kPB : 0));
  A.n_full = P.n_full;
  A.chunk = P.chunk;
  A.chunks = P.chunks;
  A.grid_full = (A.n_full + 7) / 8 * 8;
  const long long rest = (long long)(A.columns - A.n_full) * A.chunks;
  const int grid = A.grid_full + (int)((rest + 7) / 8 * 8);
  if (stall_test && o > 0)
    hipLaunchKernelGGL((pyr_pc_kernel<false, 0>), dim3(grid), dim3(256), 0, st, A);
  else if (stall_test)
    hipLaunchKernelGGL((pyr_pc_kernel<true, 0>), dim3(grid), dim3(256), 0, st, A);
  else if (o > 0)
    hipLaunchKernelGGL((pyr_pc_kernel<false>), dim3(grid), dim3(256), 0, st, A);
  else
    hipLaunchKernelGGL((pyr_pc_kernel<true>), dim3(grid), dim3(256), 0, st, A);
}

}  // namespace sift
