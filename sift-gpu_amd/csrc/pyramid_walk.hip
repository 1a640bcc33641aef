// pyramid_walk.hip -- SIFT_FLAG_FAST Gaussian pyramid as independent column
// walks (gfx950).
//
// The separable form of buildGaussianPyramid (src/sift.cpp:229-263) that
// SURVEY §8(d) names: every scale is blurred from its octave base with the
// reference's sigma and width (sig[] :240-245, w = floor(3 sigma) :97) and the
// reference's padding (rows / cols outside [0, rows-1) x [0, cols-1) read as
// 0, getSubMatrix :116), but the 2-D kernel K[a][b] = 8192 g(a) g(b) is
// applied as a row pass and a column pass with fused multiply-adds: agreement
// with the exact path within tolerance, not bit parity (DESIGN.md §9,
// tests/test_gpu_fast.py).
//
// Layout of the work: one wave = 64 output columns (one per lane) x a chunk of
// rows of one octave, walking down the source rows; no workgroup barriers.
//   * a source row segment [x0 - h, x0 + 64 + h) is staged into the wave's own
//     LDS ring (zero where the reference pads); rows arrive one block ahead;
//   * row pass in folded form: p_k = x[-k] + x[+k] once per row, then each
//     scale is g(0) x[0] + sum_k g(k) p_k -- the pair sums are shared by the
//     scales of the wave;
//   * column pass in scatter form: the row-pass value of source row r is
//     added into the 2w+1 outputs it touches, whose accumulators stay in
//     registers; an output is stored the row it completes, so plane stores are
//     spread evenly over the walk instead of bunched behind barriers.
// Two waves per strip (scales {4, 1} and {3, 2}, w = 18 + 4 and 12 + 8) keep
// the accumulators near 100 VGPRs (four waves per SIMD).  Octave 0's base is
// its own launch (the image's 9-tap blur); octave o > 0 decimates the previous
// octave's scale 2 on the fly (resize INTER_NEAREST, :252-254) and stores it as
// plane 0.  Taps are compile-time literals (build/sym_coefs.inc, from
// gauss_host.hpp's fast_taps_host, the runtime formula of pyramid_fast.hip).
#include "common.hpp"

#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "../build/sym_coefs.inc"

namespace sift {

namespace {

constexpr int kWRows = 4;  // source rows per walk step

template <int T>
__device__ __forceinline__ constexpr float fg(int a) {
  if constexpr (T == 0) return kFastG0[a];
  else if constexpr (T == 1) return kFastG1[a];
  else if constexpr (T == 2) return kFastG2[a];
  else if constexpr (T == 3) return kFastG3[a];
  else return kFastG4[a];
}
template <int T> struct FW;
template <> struct FW<0> { static constexpr int W = kSymW0; };
template <> struct FW<1> { static constexpr int W = kSymW1; };
template <> struct FW<2> { static constexpr int W = kSymW2; };
template <> struct FW<3> { static constexpr int W = kSymW3; };
template <> struct FW<4> { static constexpr int W = kSymW4; };

struct WalkArgs {
  const float* src;       // the walk's source plane, image 0 (mode 2: the previous octave's scale 2)
  long long s_pitch, s_img;
  float* dst[5];          // planes 0..4 of this octave, image 0
  long long d_pitch, d_img;
  int rows, cols, strips, batch, chunk;
  int srows, scols;       // mode 2: previous octave's shape
  double ify, ifx;        // mode 2: resize NN scale factors
  int ify2;               // mode 2: ify is exactly 2
};

// One scale's column accumulators: acc[j] is output row r0 - W + j of the
// current step (r0 = its first source row).
template <int T>
struct ColAcc {
  static constexpr int W = FW<T>::W, N = 2 * W + kWRows;
  float v[N];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = 0.f;
  }
  // row r0 + i of the step, row-pass value h
  __device__ __forceinline__ void add(int i, float h) {
#pragma unroll
    for (int m = 0; m <= 2 * W; ++m) v[i + m] = fmaf(h, fg<T>(m < W ? W - m : m - W), v[i + m]);
  }
  __device__ __forceinline__ void shift() {
#pragma unroll
    for (int j = 0; j < 2 * W; ++j) v[j] = v[j + kWRows];
#pragma unroll
    for (int j = 2 * W; j < N; ++j) v[j] = 0.f;
  }
};

// Plane stores through a buffer resource: a position outside the plane gets
// an offset past its end and the hardware drops the store, so every wave
// issues a fixed number of stores per step (no branches around them) and the
// explicit wait for the next rows' loads can leave them in flight.
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr int kDrop = 0x7ffffff0;

__device__ __forceinline__ Rsrc plane_rsrc(float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void st_plane(Rsrc rs, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, off, 0, 0);
}

// Source loads hipcc does not track (inline asm): issued at the end of a step,
// waited for with vmcnt(n) at the end of the next, n = the stores issued in
// between (VMEM operations retire in order), so the wait never covers this
// step's plane stores.  The destination registers are operands of the wait.
__device__ __forceinline__ float ld_async(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}

template <int N>
__device__ __forceinline__ void wait_loads(float (&a)[4], float (&b)[4]) {
  static_assert(N == 0 || N == 4 || N == 8 || N == 16, "store count");
  if constexpr (N == 0)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]),
                 "+v"(b[2]), "+v"(b[3])::"memory");
  else if constexpr (N == 4)
    asm volatile("s_waitcnt vmcnt(4)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]),
                 "+v"(b[2]), "+v"(b[3])::"memory");
  else if constexpr (N == 8)
    asm volatile("s_waitcnt vmcnt(8)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]),
                 "+v"(b[2]), "+v"(b[3])::"memory");
  else
    asm volatile("s_waitcnt vmcnt(16)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]),
                 "+v"(b[2]), "+v"(b[3])::"memory");
}

// Row pass of table T centred on x[H] with pair sums p[k] = x[H-k] + x[H+k].
template <int T, int H>
__device__ __forceinline__ float row_fold(const float* x, const float* p) {
  float h = x[H] * fg<T>(0);
#pragma unroll
  for (int k = 1; k <= FW<T>::W; ++k) h = fmaf(p[k], fg<T>(k), h);
  return h;
}

// MODE 0: the octave-0 base from the image (table 0); MODE 1: octave 0's
// scales from its base plane; MODE 2: octave o > 0, decimating the previous
// octave's scale 2.  TA / TB: the wave's two tables (TB < 0: none).
template <int MODE, int TA, int TB>
__device__ __forceinline__ void walk(const WalkArgs& A, int local, float* __restrict__ ring) {
  constexpr int H = FW<TA>::W;  // row window half-width (the wave's widest table)
  constexpr int SEG = 64 + 2 * H, R = kWRows;
  const int lane = threadIdx.x & 63;
  const int strip = local % A.strips, t = local / A.strips;
  const int b = t % A.batch, ck = t / A.batch;
  const int x0 = strip * 64, y0 = ck * A.chunk, y1 = min(y0 + A.chunk, A.rows);
  if (y0 >= A.rows) return;  // grid padding of the slot pairing
  const int rows = A.rows, cols = A.cols;
  const float* __restrict__ src = A.src + b * A.s_img;
  const long long dimg = b * A.d_img;
  // segment elements e = lane and lane + 64 (< SEG) <-> columns x0 - H + e
  const int xa = x0 - H + lane, xb = xa + 64;
  const bool hasb = lane + 64 < SEG;
  const bool pa = xa >= 0 && xa < cols - 1, pb = hasb && xb >= 0 && xb < cols - 1;  // nonzero filter input
  int ca, cb;
  if (MODE == 2) {  // resize NN column map
    ca = (xa >= 0 && xa < cols) ? min((int)floor(xa * A.ifx), A.scols - 1) : 0;
    cb = (xb >= 0 && xb < cols) ? min((int)floor(xb * A.ifx), A.scols - 1) : 0;
  } else {
    ca = min(max(xa, 0), cols - 1);
    cb = min(max(xb, 0), cols - 1);
  }
  // mode 2 stores the (unpadded) decimated base as plane 0 from the lane that
  // fetched it: element e is output column x0 + e - H
  const bool owna = MODE == 2 && TB == 2 && lane >= H && xa < cols;
  const bool ownb = MODE == 2 && TB == 2 && hasb && lane < H && xb < cols;
  const long long pbytes = (long long)rows * A.d_pitch * 4;
  const Rsrc rs0 = plane_rsrc(A.dst[0] + dimg, pbytes);
  static_assert(R == 4, "wait_loads operand list");
  float va[R], vb[R];
  auto fetch = [&](int r0) {  // untracked loads, clamped addresses
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = min(r0 + i, rows - 1);
      int sr = r;
      if (MODE == 2) {
        sr = A.ify2 ? 2 * r : (int)floor(r * A.ify);
        sr = min(sr, A.srows - 1);
      }
      const float* row = src + (long long)sr * A.s_pitch;
      va[i] = ld_async(row + ca);
      vb[i] = ld_async(row + cb);
    }
  };
  auto stage = [&](int slot, int r0) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = r0 + i;
      const bool rok = r < rows - 1;
      float* d = ring + (slot * R + i) * SEG;
      d[lane] = (rok && pa) ? va[i] : 0.f;
      if (hasb) d[lane + 64] = (rok && pb) ? vb[i] : 0.f;
      if constexpr (MODE == 2 && TB == 2) {  // plane 0, unpadded
        const bool rin = r >= y0 && r < y1;
        st_plane(rs0, (rin && owna) ? (int)((long long)r * A.d_pitch + xa) * 4 : kDrop, va[i]);
        st_plane(rs0, (rin && ownb) ? (int)((long long)r * A.d_pitch + xb) * 4 : kDrop, vb[i]);
      }
    }
  };
  ColAcc<TA> acA;
  ColAcc<(TB < 0 ? 0 : TB)> acB;
  acA.zero();
  acB.zero();
  constexpr int PA = MODE == 0 ? 0 : TA, PB = TB;  // output planes
  const Rsrc rsA = plane_rsrc(A.dst[PA] + dimg, pbytes);
  const Rsrc rsB = plane_rsrc(A.dst[TB < 0 ? 0 : PB] + dimg, pbytes);
  constexpr int NST = R * (TB >= 0 ? 2 : 1);  // plane stores per step
  const int xo = x0 + lane;
  const bool colok = xo < cols;
  int r0 = max(y0 - H, 0);
  const int rend = y1 + H;
  fetch(r0);
  wait_loads<0>(va, vb);
  stage(0, r0);
  fetch(r0 + R);
  int slot = 0;
  for (; r0 < rend; r0 += R) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = r0 + i;
      if (r < rows - 1) {  // uniform; rows past the last contribute 0
        const float* lr = ring + (slot * R + i) * SEG + lane;
        float x[2 * H + 1];
#pragma unroll
        for (int c = 0; c <= 2 * H; ++c) x[c] = lr[c];
        float p[H + 1];
#pragma unroll
        for (int k = 1; k <= H; ++k) p[k] = x[H - k] + x[H + k];
        acA.add(i, row_fold<TA, H>(x, p));
        if constexpr (TB >= 0) acB.add(i, row_fold<TB, H>(x, p));
      }
      // outputs completed by row r: r - W (stores always issued, dropped off-plane)
      const int ya = r - FW<TA>::W;
      st_plane(rsA, (colok && ya >= y0 && ya < y1) ? (ya * (int)A.d_pitch + xo) * 4 : kDrop, acA.v[i]);
      if constexpr (TB >= 0) {
        const int yb = r - FW<TB>::W;
        st_plane(rsB, (colok && yb >= y0 && yb < y1) ? (yb * (int)A.d_pitch + xo) * 4 : kDrop, acB.v[i]);
      }
    }
    acA.shift();
    if constexpr (TB >= 0) acB.shift();
    wait_loads<NST>(va, vb);  // the next rows' loads, not this step's stores
    slot ^= 1;
    stage(slot, r0 + R);
    fetch(r0 + 2 * R);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load in flight past the end
}

// Waves are independent; octave launches pair the two slots of a strip on one
// XCD (workgroups w and w + 8 share an XCD): slot = bit 3 of the id.
template <int MODE>
__global__ __launch_bounds__(64) void pyr_walk_kernel(WalkArgs A) {
  __shared__ float ring[2 * kWRows * (64 + 2 * (MODE == 0 ? kSymW0 : kSymW4))];
  const int wid = blockIdx.x;
  if (MODE == 0) {
    walk<0, 0, -1>(A, wid, ring);
    return;
  }
  const int slot = (wid >> 3) & 1, local = (wid & 7) | ((wid >> 4) << 3);
  if (slot == 0)
    walk<MODE, 4, 1>(A, local, ring);
  else
    walk<MODE, 3, 2>(A, local, ring);
}

int walk_chunk(int rows, long long units, int halo) {
  // about 8192 waves per launch, chunks >= 4 halos tall
  const long long want = 8192;
  int ch = (int)std::max<long long>(1, (want + units - 1) / units);
  ch = std::min(ch, std::max(1, rows / (4 * halo)));
  return (rows + ch - 1) / ch;
}

}  // namespace

// The SIFT_FLAG_FAST pyramid of octave o for the batch: octave 0 = base launch
// + scale launch, octave o > 0 = one launch.
void launch_pyramid_walk(hipStream_t st, const Layout& L, int o, float* gpyr, Plane src, int batch) {
  const Octave& O = L.oct[o];
  WalkArgs A{};
  for (int s = 0; s < kScales; ++s) A.dst[s] = gpyr + O.g_off[s];
  A.d_pitch = O.pitch;
  A.d_img = L.g_img;
  A.rows = O.rows;
  A.cols = O.cols;
  A.strips = (O.cols + 63) / 64;
  A.batch = batch;
  const long long units = (long long)A.strips * batch;
  if (o == 0) {
    A.src = src.p;
    A.s_pitch = src.pitch;
    A.s_img = src.img_stride;
    A.chunk = walk_chunk(O.rows, units, kSymW0);
    const int n = (int)(units * ((O.rows + A.chunk - 1) / A.chunk));
    hipLaunchKernelGGL(pyr_walk_kernel<0>, dim3(n), dim3(64), 0, st, A);
    A.src = gpyr + O.g_off[0];
    A.s_pitch = O.pitch;
    A.s_img = L.g_img;
  } else {
    const Octave& P = L.oct[o - 1];
    A.src = gpyr + P.g_off[kLayers];
    A.s_pitch = P.pitch;
    A.s_img = L.g_img;
    A.srows = P.rows;
    A.scols = P.cols;
    A.ifx = 1. / ((double)O.cols / P.cols);
    A.ify = 1. / ((double)O.rows / P.rows);
    A.ify2 = P.rows == 2 * O.rows && A.ify == 2.0;
  }
  A.chunk = walk_chunk(O.rows, 2 * units, kSymW4);
  // slot pairs: ids (w & 7) | (slot << 3) | ((w >> 3) << 4) over units x chunks waves per slot
  const long long per_slot = units * ((O.rows + A.chunk - 1) / A.chunk);
  const long long n = ((per_slot + 7) / 8) * 16;
  if (o == 0)
    hipLaunchKernelGGL(pyr_walk_kernel<1>, dim3((unsigned)n), dim3(64), 0, st, A);
  else
    hipLaunchKernelGGL(pyr_walk_kernel<2>, dim3((unsigned)n), dim3(64), 0, st, A);
}

}  // namespace sift
