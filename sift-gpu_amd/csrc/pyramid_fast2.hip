// pyramid_fast2.hip -- SIFT_FLAG_FAST Gaussian pyramid, 64-column strips fed
// by LDS DMA.
//
// The same arithmetic as pyramid_fast.hip (separable row / column passes of
// the reference's per-scale sigmas from the octave base, src/sift.cpp:229-263,
// the base's padding rule of getSubMatrix :116; every output a fused
// multiply-add chain over the taps in the same order), so the planes are bit
// for bit those of pyramid_fast.hip (tests/test_gpu_fast.py checks it) -- laid
// out for latency hiding instead:
//
//  * phase ablations of pyramid_fast.hip on MI355X showed its source fetch and
//    plane stores adding to the FMA time rather than overlapping it: one
//    8-row step of prefetch in registers (13 KB per CU in flight) cannot cover
//    HBM latency.  Here the base rows arrive by global_load_lds_dwordx4 into
//    three stage buffers, issued two steps ahead, with no VGPRs held and no
//    LDS re-staging instructions;
//  * every octave reads its base from plane 0 (octave 0: base9_kernel, the
//    9-tap blur of the image; octave o > 0: the exact path's INTER_NEAREST
//    decimate_kernel, :252-254), so the walk has one source pattern;
//  * a workgroup owns a 64-column strip: 40 KB of LDS, four workgroups
//    (16 waves) per CU;
//  * wave w runs one scale's row pass (4 columns x 2 rows per lane, 8 scalar
//    FMA chains) and another scale's column pass (one column x 8 rows per
//    lane), pairing sigma4's row pass with sigma1's column pass and so on.
#include "common.hpp"

#include <math.h>
#include <stdlib.h>

namespace sift {

struct FastCoefs2 {  // layout of pyramid_fast.hip's FastCoefs (checked by the launcher)
  float base[9];
  float s1[9], s2[17], s3[25], s4[37];
};

struct FastArgs2 {
  float* gpyr;
  long long g_img;
  long long off[kScales];  // plane offsets of this octave in the image block
  int pitch, rows, cols;
  int chunk;
  int abl;                 // SIFT_HIP_ABL ablation bits (timing experiments only, 0 otherwise)
  FastCoefs2 coef;
};

namespace {

constexpr int kSW = 64;                // output columns per strip
constexpr int kRB2 = 8;                // rows per step
constexpr int kH2 = 18;                // widest scale half-width
constexpr int kLead2 = 24;             // base rows walked above the chunk (>= kH2, multiple of 8)
constexpr int kX0 = 20;                // stage column 0 = plane column x0 - 20 (16-B aligned: pitch % 16 == 0)
constexpr int kSC4 = (kSW + 2 * kX0) / 4;  // 26 float4 per stage row
constexpr int kSItems = kRB2 * kSC4;   // 208 float4 per step: waves 0-2 all lanes, wave 3 lanes 0-15
constexpr int kNSt = 3;                // stage buffers (DMA two steps ahead)
constexpr int kRP2 = 64;               // ring row pitch (floats)
constexpr int kDrop2 = 0x7ffffff0;     // buffer offset past every plane: the store is dropped

template <int W> struct Ring2;
template <> struct Ring2<4> { static constexpr int off = 0, M = 16; };
template <> struct Ring2<8> { static constexpr int off = 16, M = 24; };
template <> struct Ring2<12> { static constexpr int off = 40, M = 32; };
template <> struct Ring2<18> { static constexpr int off = 72, M = 48; };
constexpr int kRingRows2 = 120;

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* LdsPtr;
typedef const __attribute__((address_space(4))) FastArgs2* KArgs2;

__device__ __forceinline__ Rsrc plane_rsrc2(float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_plane4(Rsrc rs, int off, float4 v) {
  const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 0);
}

template <int W>
__device__ __forceinline__ void taps_v(const __attribute__((address_space(4))) float* k, f2 (&g)[W + 1]) {
#pragma unroll
  for (int j = 0; j <= W; ++j) {
    g[j] = f2{k[2 * j], 2 * j + 1 <= 2 * W ? k[2 * j + 1] : 0.f};
    asm volatile("" : "+v"(g[j]));  // taps live in VGPRs (SGPRs run out)
  }
}

__device__ __forceinline__ float tap(const f2* g, int b) { return (b & 1) ? g[b >> 1].y : g[b >> 1].x; }

template <int W> __device__ __forceinline__ const __attribute__((address_space(4))) float* taps_of(KArgs2 KA) {
  return W == 4 ? KA->coef.s1 : W == 8 ? KA->coef.s2 : W == 12 ? KA->coef.s3 : KA->coef.s4;
}
template <int W> constexpr int plane_of() { return W == 4 ? 1 : W == 8 ? 2 : W == 12 ? 3 : 4; }

// ---- stage: base rows [Z, Z+8) x plane columns [x0-20, x0+84), row-major,
// 0 outside [0, rows-1) x [0, cols-1) (the blur's source padding) ----------

struct StageItem {  // this lane's float4 of a step
  bool on;          // lane carries an item (it < 208)
  int r, q;         // stage row, float4 column
};

__device__ __forceinline__ StageItem stage_item() {
  const int it = threadIdx.x;  // wave w: items 64w + lane
  return StageItem{it < kSItems, it / kSC4, it % kSC4};
}

// Issue step Z's DMA into buffer `buf` (every wave issues exactly one
// global_load_lds_dwordx4: wave 3 has lanes 0-15 on).  Lanes whose float4 is
// entirely padding load row 0 of the plane and are zeroed by stage_fix.
__device__ __forceinline__ void stage_dma(const float* __restrict__ base, int pitch, int rows, int cols,
                                          float4* buf, int x0, int Z, const StageItem& I) {
  const int y = Z + I.r, x = x0 - kX0 + 4 * I.q;
  const bool live = y >= 0 && y < rows - 1 && x >= 0 && x < cols - 1;
  const float* p = base + (live ? (long long)y * pitch + x : 0);
  // Inline asm, not __builtin_amdgcn_global_load_lds: the compiler fences a
  // builtin LDS DMA with vmcnt(0) before every s_barrier, which would wait
  // out the two steps of lead and every plane store in flight.
  // M0 = the wave's LDS destination (lane i's 16 bytes land at M0 + 16 i).
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(LdsPtr)(buf + (threadIdx.x & ~63)));
  if (I.on)
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p), "s"(m0) : "memory");
}

// After the lane's own DMA has landed: zero its float4 if it is padding, or
// the elements from column cols-1 on if it straddles that column.
__device__ __forceinline__ void stage_fix(int rows, int cols, float4* buf, int x0, int Z, const StageItem& I) {
  if (!I.on) return;
  const int y = Z + I.r, x = x0 - kX0 + 4 * I.q;
  const bool live = y >= 0 && y < rows - 1 && x >= 0 && x < cols - 1;
  if (!live) {
    buf[threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);
  } else if (x + 3 >= cols - 1) {
    float* e = reinterpret_cast<float*>(buf + threadIdx.x);
    for (int k = cols - 1 - x; k < 4; ++k) e[k] = 0.f;
  }
}

// ---- row pass of one scale by one wave: lane (s, j) takes base rows 2s,
// 2s+1 x strip columns [4j, 4j+4).  h[r][4j+i] = sum_b g[b] base[r][4j+i-W+b]
// = stage[r][4j + i + 20 - W + b]; the window is read as aligned float4s
// from stage column 4j + A (A = (20 - W) & ~3) with the taps starting D = 20 -
// W - A into it.  The 16 lanes of each ds_read_b128 group share s and take
// j = 0..15: consecutive float4s, conflict free.
template <int W>
__device__ __forceinline__ void row_pass4(const float4* __restrict__ st4, float* __restrict__ rings, const f2* g,
                                          int s, int j, int slot) {
  constexpr int A = (kX0 - W) & ~3, D = kX0 - W - A;
  constexpr int NF = (D + 2 * W + 4 + 3) / 4;  // float4s of the window
  // both rows' windows are read before the taps: row 1's reads are in flight
  // under row 0's FMAs (3 workgroups per CU leave 168 VGPRs)
  float w[2][4 * NF];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const float4* src = st4 + (2 * s + rr) * kSC4 + j + A / 4;
#pragma unroll
    for (int q = 0; q < NF; ++q) {
      const float4 v = src[q];
      w[rr][4 * q] = v.x;
      w[rr][4 * q + 1] = v.y;
      w[rr][4 * q + 2] = v.z;
      w[rr][4 * q + 3] = v.w;
    }
  }
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b <= 2 * W; ++b) {
      const float gb = tap(g, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_fmaf(w[rr][D + i + b], gb, acc[i]);
    }
    // slot + 1 never wraps: slot = (Z - rbase) mod M + 2s, Z - rbase and M multiples of 8
    reinterpret_cast<float4*>(rings + (Ring2<W>::off + slot + rr) * kRP2)[j] =
        make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

// ---- column pass of one scale, one column per lane: plane rows [Y, Y + 8)
// from ring rows starting at slot S0 (compile-time LDS offsets per body).
// Always issues 8 stores; rows outside [y0, y1) and columns past the image
// are dropped through the buffer range check.
template <int W, int S0>
__device__ __forceinline__ void col_fixed2(const float* __restrict__ rings, const f2* g, int lane, Rsrc rs,
                                           int pitch, float* __restrict__ tp, int x4, int Y, int y0, int y1,
                                           bool colok, int abl) {
  constexpr int NR = 8, M = Ring2<W>::M, N = NR + 2 * W;
  const float* base = rings + Ring2<W>::off * kRP2 + lane;
  constexpr int K1 = N;  // (one pass: 3 workgroups per CU leave 168 VGPRs for the whole window)
  constexpr int A1 = K1 - NR;                         // last tap of the first half
  float win[N];
  float acc[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) acc[i] = 0.f;
  if (!(abl & 2)) {
#pragma unroll
    for (int k = 0; k < K1; ++k) win[k] = base[((S0 + k) % M) * kRP2];
#pragma unroll
    for (int a = 0; a <= (K1 == N ? 2 * W : A1); ++a) {
      const float ga = tap(g, a);
#pragma unroll
      for (int i = 0; i < NR; ++i) acc[i] = __builtin_fmaf(win[i + a], ga, acc[i]);
    }
    if constexpr (K1 < N) {
      asm volatile("" ::: "memory");  // keeps the second half's reads behind the first half's taps
#pragma unroll
      for (int k = K1; k < N; ++k) win[k] = base[((S0 + k) % M) * kRP2];
#pragma unroll
      for (int a = A1 + 1; a <= 2 * W; ++a) {
        const float ga = tap(g, a);
#pragma unroll
        for (int i = 0; i < NR; ++i) acc[i] = __builtin_fmaf(win[i + a], ga, acc[i]);
      }
    }
  }
  // 8 rows x 64 columns out as 2 float4 stores per lane (store instructions,
  // not bytes, set the cost of the plane writes): through the wave's 4 x 64
  // transpose slice, 4 rows at a time -- the lane writes its column, reads
  // row lane >> 4 x columns 4 (lane & 15) .. +3
  const int rr = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) tp[i * 64 + lane] = acc[4 * h + i];
    __builtin_amdgcn_wave_barrier();
    const float4 v = reinterpret_cast<const float4*>(tp)[rr * 16 + (lane & 15)];
    __builtin_amdgcn_wave_barrier();
    const int y = Y + 4 * h + rr;
    st_plane4(rs, (colok && y >= y0 && y < y1 && !(abl & 4)) ? (y * pitch + x4) * 4 : kDrop2, v);
  }
  asm volatile("; col_fixed2 %0 %1" ::"n"(W), "n"(S0));  // distinct tail per body
}

template <int W, int C>
__device__ __forceinline__ void col_pass2(int c, const float* __restrict__ rings, const f2* g, int lane, Rsrc rs,
                                          int pitch, float* tp, int x4, int Z, int y0, int y1, bool colok, int abl) {
  constexpr int R0 = (((-2 * W) % 8) + 8) % 8;
  if constexpr (C + 1 < Ring2<W>::M / 8) {
    if (c == C)
      col_fixed2<W, 8 * C + R0>(rings, g, lane, rs, pitch, tp, x4, Z - W, y0, y1, colok, abl);
    else
      col_pass2<W, C + 1>(c, rings, g, lane, rs, pitch, tp, x4, Z, y0, y1, colok, abl);
  } else {
    col_fixed2<W, 8 * C + R0>(rings, g, lane, rs, pitch, tp, x4, Z - W, y0, y1, colok, abl);
  }
}

#define SIFT_VM_WAIT2(CNT) asm volatile("s_waitcnt vmcnt(" #CNT ")" ::: "memory")

// One wave's walk: the row pass of scale WR and the column pass of scale WC.
// Waves 0-3 take (18,4), (4,18), (12,8), (8,12): 296 + 72, 72 + 296, 200 +
// 136, 136 + 200 FMAs per lane a step.
//
// Step k (base rows Z = Zbeg + 8k) uses stage buffer k % 3.  Its DMA was
// issued at step k-2 (the prologue issues steps 0 and 1), after which this
// wave issued 2 plane stores (step k-2), one DMA (step k+1, if any) and 2
// plane stores (step k-1): vmcnt(5) waits for exactly step k's DMA.
template <int WR, int WC>
__device__ __forceinline__ void walk4(const FastArgs2& A, float4* stage4, float* rings, float* tpose, float* gimg,
                                      const float* base, long long plane_bytes, int x0, int y0, int y1, int rbase,
                                      int Zbeg, int nsteps) {
  const KArgs2 KA = (KArgs2)__builtin_amdgcn_kernarg_segment_ptr();
  f2 kr[WR + 1], kc[WC + 1];
  taps_v<WR>(taps_of<WR>(KA), kr);
  taps_v<WC>(taps_of<WC>(KA), kc);
  const int lane = threadIdx.x & 63;
  // row-pass lane map: ds_read_b128 serves a wave in four 16-lane groups
  // ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32): group = row pair s, index
  // in the group = float4 column j (group of lane L: the bit parity of its
  // 4-lane block L>>2 & 7, upper half by L>>5; index (block>>1)*4 + L%4)
  const int blk = (lane >> 2) & 7;
  const int rs = 2 * (lane >> 5) + (__builtin_popcount(blk) & 1);
  const int rj = (blk >> 1) * 4 + (lane & 3);
  const int x4 = x0 + 4 * (lane & 15);  // column of the lane's float4 plane stores
  const bool colok = x4 < A.cols;        // (x4 + 3 < pitch: pitch is a multiple of 16)
  float* tp = tpose + (threadIdx.x >> 6) * 256;
  const Rsrc rsc = plane_rsrc2(gimg + A.off[plane_of<WC>()], plane_bytes);
  const int abl = A.abl;
  const StageItem I = stage_item();
  for (int k = 0; k < nsteps; ++k) {
    const int Z = Zbeg + kRB2 * k;
    float4* cur = stage4 + (k % kNSt) * kSItems;
    if (k >= 2 && k + 1 < nsteps)
      SIFT_VM_WAIT2(5);
    else if (k == 1 && nsteps > 2)
      SIFT_VM_WAIT2(3);
    else if (k == 0 && nsteps > 1)
      SIFT_VM_WAIT2(1);
    else
      SIFT_VM_WAIT2(0);
    stage_fix(A.rows, A.cols, cur, x0, Z, I);
    __syncthreads();  // base rows [Z, Z+8) staged; every wave is done with step k-1
    if (k + 2 < nsteps && !(abl & 8))
      stage_dma(base, A.pitch, A.rows, A.cols, stage4 + ((k + 2) % kNSt) * kSItems, x0, Z + 2 * kRB2, I);
    if (Z + kRB2 > y0 - WR && Z < y1 + WR && !(abl & 1))
      row_pass4<WR>(cur, rings, kr, rs, rj, (Z - rbase) % Ring2<WR>::M + 2 * rs);
    __syncthreads();
    col_pass2<WC, 0>(((Z - 2 * WC - rbase) % Ring2<WC>::M) >> 3, rings, kc, lane, rsc, A.pitch, tp, x4, Z, y0,
                     y1, colok, abl);
  }
  SIFT_VM_WAIT2(0);
}

__global__ __launch_bounds__(256, 3) void pyr_scales_kernel(FastArgs2 A) {
  __shared__ float4 stage4[kNSt * kSItems];
  __shared__ float4 rings4[kRingRows2 * kRP2 / 4];
  __shared__ float4 tpose4[4 * 64];  // per wave a 4 x 64 store transpose slice
  float* rings = reinterpret_cast<float*>(rings4);
  const int b = blockIdx.z;
  const int x0 = blockIdx.x * kSW;
  const int y0 = blockIdx.y * A.chunk;
  const int y1 = min(y0 + A.chunk, A.rows);
  float* gimg = A.gpyr + b * A.g_img;
  const long long plane_bytes = (long long)A.rows * A.pitch * 4;
  const float* base = gimg + A.off[0];
  const int rbase = y0 - 64;
  const int Zbeg = y0 - kLead2;
  const int nsteps = (y1 + kH2 - Zbeg + kRB2 - 1) / kRB2;
  const StageItem I = stage_item();
  if (!(A.abl & 8)) {
    stage_dma(base, A.pitch, A.rows, A.cols, stage4, x0, Zbeg, I);
    if (nsteps > 1) stage_dma(base, A.pitch, A.rows, A.cols, stage4 + kSItems, x0, Zbeg + kRB2, I);
  }
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wv == 0)
    walk4<18, 4>(A, stage4, rings, reinterpret_cast<float*>(tpose4), gimg, base, plane_bytes, x0, y0, y1, rbase, Zbeg, nsteps);
  else if (wv == 1)
    walk4<4, 18>(A, stage4, rings, reinterpret_cast<float*>(tpose4), gimg, base, plane_bytes, x0, y0, y1, rbase, Zbeg, nsteps);
  else if (wv == 2)
    walk4<12, 8>(A, stage4, rings, reinterpret_cast<float*>(tpose4), gimg, base, plane_bytes, x0, y0, y1, rbase, Zbeg, nsteps);
  else
    walk4<8, 12>(A, stage4, rings, reinterpret_cast<float*>(tpose4), gimg, base, plane_bytes, x0, y0, y1, rbase, Zbeg, nsteps);
}

#undef SIFT_VM_WAIT2

// Octave-0 base: image -> plane 0, the 9-tap row pass then the 9-tap column
// pass (FMA chains in tap order, as pyramid_fast.hip's base phase) on a
// 64 x 32 output tile staged with its 4-pixel halo; float4 loads (VEC: the
// image rows 16-B aligned), row-pass outputs and plane stores.
constexpr int kBTW = 64, kBTH = 32, kBSW4 = (kBTW + 8) / 4, kBSH = kBTH + 8;

template <bool VEC>
__global__ __launch_bounds__(256) void base9_kernel(const float* __restrict__ img, long long s_pitch, long long s_img,
                                                    float* __restrict__ gpyr, long long g_img, int pitch, int rows,
                                                    int cols, FastCoefs2 coef) {
  __shared__ float4 sst[kBSH][kBSW4];  // image columns x0-4 .. x0+68
  __shared__ float4 tmp[kBSH][kBTW / 4];
  const int t = threadIdx.x;
  const int b = blockIdx.z;
  const int x0 = blockIdx.x * kBTW, y0 = blockIdx.y * kBTH;
  const float* im = img + b * s_img;
  for (int i = t; i < kBSH * kBSW4; i += 256) {
    const int r = i / kBSW4, q = i - r * kBSW4;
    const int y = y0 - 4 + r, x = x0 - 4 + 4 * q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y >= 0 && y < rows - 1) {  // getSubMatrix padding (:116): row rows-1 and column cols-1 read as 0
      const float* row = im + (long long)y * s_pitch;
      if (VEC && x >= 0 && x + 3 < cols - 1) {
        v = *reinterpret_cast<const float4*>(row + x);
      } else {
        float e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = (x + k >= 0 && x + k < cols - 1) ? row[x + k] : 0.f;
        v = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
    sst[r][q] = v;
  }
  __syncthreads();
  for (int i = t; i < kBSH * (kBTW / 4); i += 256) {
    const int r = i >> 4, g = i & 15;
    float w[12];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float4 v = sst[r][g + q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(w[e + k], coef.base[k], acc[e]);
    }
    tmp[r][g] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
  __syncthreads();
  // column pass: lane (r2, g) -> output rows 2 r2, 2 r2 + 1 x columns 4g..4g+3
  const int g = t & 15, r2 = t >> 4;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const float4 v = tmp[2 * r2 + k][g];
    if (k < 9) {
      const float c = coef.base[k];
      a0 = make_float4(__builtin_fmaf(v.x, c, a0.x), __builtin_fmaf(v.y, c, a0.y), __builtin_fmaf(v.z, c, a0.z),
                       __builtin_fmaf(v.w, c, a0.w));
    }
    if (k > 0) {
      const float c = coef.base[k - 1];
      a1 = make_float4(__builtin_fmaf(v.x, c, a1.x), __builtin_fmaf(v.y, c, a1.y), __builtin_fmaf(v.z, c, a1.z),
                       __builtin_fmaf(v.w, c, a1.w));
    }
  }
  float* out = gpyr + b * g_img;
  const int x = x0 + 4 * g, y = y0 + 2 * r2;
  if (x < cols) {  // x + 3 < pitch (a multiple of 16)
    if (y < rows) *reinterpret_cast<float4*>(out + (long long)y * pitch + x) = a0;
    if (y + 1 < rows) *reinterpret_cast<float4*>(out + (long long)(y + 1) * pitch + x) = a1;
  }
}

}  // namespace

void launch_pyramid_fast2(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch,
                          const void* coef) {
  static_assert(sizeof(FastCoefs2) == (9 + 9 + 17 + 25 + 37) * sizeof(float), "FastCoefs layout");
  const Octave& O = L.oct[o];
  FastArgs2 A{};
  A.gpyr = gpyr;
  A.g_img = L.g_img;
  for (int s = 0; s < kScales; ++s) A.off[s] = O.g_off[s];
  A.coef = *static_cast<const FastCoefs2*>(coef);
  static const int abl = getenv("SIFT_HIP_ABL") ? atoi(getenv("SIFT_HIP_ABL")) : 0;
  A.abl = abl;
  A.pitch = O.pitch;
  A.rows = O.rows;
  A.cols = O.cols;
  if (o == 0) {
    dim3 g0((O.cols + kBTW - 1) / kBTW, (O.rows + kBTH - 1) / kBTH, batch);
    const bool vec =
        src.pitch % 4 == 0 && src.img_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(src.p) & 15) == 0;
    if (vec)
      hipLaunchKernelGGL(base9_kernel<true>, g0, dim3(256), 0, st, src.p, src.pitch, src.img_stride,
                         gpyr + O.g_off[0], L.g_img, O.pitch, O.rows, O.cols, A.coef);
    else
      hipLaunchKernelGGL(base9_kernel<false>, g0, dim3(256), 0, st, src.p, src.pitch, src.img_stride,
                         gpyr + O.g_off[0], L.g_img, O.pitch, O.rows, O.cols, A.coef);
  } else {
    launch_decimate(st, L, o, gpyr, batch);
  }
  // Row chunks per strip: every chunk walks kLead2 + kH2 = 42 rows it does
  // not output, and the grid runs in rounds of `resident` workgroups (4 per
  // CU): the chunk count that minimises rounds x rows walked per chunk.
  const int strips = (O.cols + kSW - 1) / kSW;
  const long long per = (long long)strips * batch;
  const int resident = resident_grid((const void*)pyr_scales_kernel, 256, 0, 1024);
  int ch = 0;
  double best = 0;
  for (int c = 1; c <= (O.rows + kRB2 - 1) / kRB2; ++c) {
    const int h = ((O.rows + c - 1) / c + kRB2 - 1) / kRB2 * kRB2;
    const int cc = (O.rows + h - 1) / h;
    const double cost = (double)((per * cc + resident - 1) / resident) * (h + kLead2 + kH2);
    if (ch == 0 || cost < best) {
      best = cost;
      ch = h;
    }
  }
  A.chunk = ch;
  dim3 grid(strips, (O.rows + ch - 1) / ch, batch);
  hipLaunchKernelGGL(pyr_scales_kernel, grid, dim3(256), 0, st, A);
}

}  // namespace sift
