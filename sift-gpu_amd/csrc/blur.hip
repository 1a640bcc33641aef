// blur.hip -- Gaussian scale-space kernels for gfx950 (exact mode).
//
// The reference blur (src/sift.cpp:110-153, Gaussian_Blur) is a direct 2-D
// convolution whose result is the float chain
//     acc = 0; for a in -w..w: for b in -w..w: acc = acc + src'(y+a, x+b) * K[a][b]
//     out = acc / 8192
// with separate multiply and add and src' = 0 outside [0, rows-1) x [0, cols-1)
// (the last source row and column never contribute, :116).  To be bit-exact
// the GPU keeps exactly that chain per output pixel; the parallelism is across
// pixels.  Design for CDNA4:
//   * one 256-thread workgroup per TILE_W x TILE_H output tile; the tile plus
//     its w-halo is staged once into LDS (zero-filled, so the padding rule is a
//     branch-free read);
//   * each lane owns PX consecutive outputs of one row and slides a register
//     window of PX + 2w source values per kernel row (bank-conflict-free
//     ds_read_b128, see lane_to_pixel), so one LDS word feeds ~2w+1
//     multiply-adds;
//   * kernel rows are uniform across the wave, so the 2w+1 coefficients of a
//     row come from the scalar cache into SGPRs (VALU ops take them directly);
//   * the four scales of an octave are blurred by ONE launch (blockIdx.z picks
//     scale and image, heaviest scale dispatched first) -- every scale reads
//     the same octave base (src/sift.cpp:256-258), so the base tile stays hot
//     in L2 across the four scale workgroups.
// Bound: VALU (2 instructions per tap, FMA forbidden by the parity contract).
#include "common.hpp"

#include <math.h>
#include <stdlib.h>

#include <algorithm>

namespace sift {

// ---- exact 2-D tile -----------------------------------------------------------
constexpr int kPX = 8;    // outputs per lane along a row
constexpr int kTY = 32;   // tile rows (one lane row each)
constexpr int kTX = 256 / kTY;
constexpr int kTileW = kTX * kPX;

// Window reads are ds_read_b128, whose wave64 access is served in four
// 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32.  Lanes
// are assigned to output pixels so that each group holds two whole tile rows
// (ty, ty+1) x 8 lanes; with the LDS row pitch LP = 4 (mod 8) words the 16
// lanes' 16-byte slots (ty*LP/4 + 2*tx + k) mod 16 are all distinct:
// bank-conflict free.
__device__ __forceinline__ void lane_to_pixel(int lane, int& ty, int& tx) {
  const int l = lane & 31;
  const bool g2 = (l >= 4 && l < 12) || (l >= 16 && l < 20) || l >= 28;  // group 2 of the half
  // position of l inside its group (lanes listed in ascending order)
  int pos;
  if (!g2) pos = l < 4 ? l : l < 16 ? l - 8 : l - 12;      // 0-3, 12-15, 20-27
  else pos = l < 12 ? l - 4 : l < 20 ? l - 8 : l - 16;     // 4-11, 16-19, 28-31
  ty = ((lane >> 5) * 2 + (g2 ? 1 : 0)) * 2 + (pos >> 3);
  tx = pos & 7;
}

template <int W>
struct BlurTile {
  static constexpr int KS = 2 * W + 1;
  static constexpr int LW = kTileW + 2 * W;
  static constexpr int LP = ((LW + 3) / 8) * 8 + 4;
  static constexpr int LR = kTY + 2 * W;
  static constexpr int LDS_FLOATS = LR * LP;
  static constexpr int NWIN = kPX + 2 * W;
  static_assert(NWIN % 4 == 0 && LP % 8 == 4 && LP >= LW, "window layout");
};

// Next octave's plane 0 written by the blur of plane nOctaveLayers = 2
// (src/sift.cpp:252-254, INTER_NEAREST at exactly half size: (y, x) <- (2y, 2x)),
// so no decimation launch; p == nullptr: not fused.
struct NextPlane {
  float* p;
  long long pitch;
  int rows, cols;
};

template <int W>
__device__ __forceinline__ void blur_tile(const float* __restrict__ src, long long spitch, int rows,
                                          int cols, float* __restrict__ dst, long long dpitch,
                                          const float* __restrict__ coef, int x0, int y0,
                                          float* __restrict__ lds, NextPlane nx = NextPlane{nullptr, 0, 0, 0}) {
  using T = BlurTile<W>;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int r = wv; r < T::LR; r += 4) {
    const int gy = y0 - W + r;
    const bool rok = gy >= 0 && gy < rows - 1;
    const float* srow = src + (long long)(rok ? gy : 0) * spitch;
    float* lrow = lds + r * T::LP;
    for (int c = lane; c < T::LW; c += 64) {
      const int gx = x0 - W + c;
      lrow[c] = (rok && gx >= 0 && gx < cols - 1) ? srow[gx] : 0.f;
    }
  }
  __syncthreads();
  int tx, ty;
  lane_to_pixel(lane, ty, tx);
  ty += wv * 8;
  float acc[kPX];
#pragma unroll
  for (int p = 0; p < kPX; ++p) acc[p] = 0.f;
  const float* base = lds + ty * T::LP + tx * kPX;
  for (int a = 0; a < T::KS; ++a) {
    float win[T::NWIN];
    const float4* l4 = reinterpret_cast<const float4*>(base + a * T::LP);
#pragma unroll
    for (int q = 0; q < T::NWIN / 4; ++q) {
      const float4 t = l4[q];
      win[4 * q] = t.x;
      win[4 * q + 1] = t.y;
      win[4 * q + 2] = t.z;
      win[4 * q + 3] = t.w;
    }
    const float* kr = coef + a * T::KS;
#pragma unroll
    for (int b = 0; b < T::KS; ++b) {
      const float k = kr[b];
      // all kPX products first (distinct registers, pinned by the empty asm),
      // then the kPX adds: no multiply feeds the very next instruction
      float t[kPX];
#pragma unroll
      for (int p = 0; p < kPX; ++p) t[p] = win[p + b] * k;
      asm volatile("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]),
                   "+v"(t[6]), "+v"(t[7]));
#pragma unroll
      for (int p = 0; p < kPX; ++p) acc[p] = acc[p] + t[p];
    }
  }
  const int y = y0 + ty;
  const int x = x0 + tx * kPX;
  if (y < rows) {
    float* drow = dst + (long long)y * dpitch + x;
    if (x + kPX <= cols) {
      float4* d4 = reinterpret_cast<float4*>(drow);
#pragma unroll
      for (int q = 0; q < kPX / 4; ++q)
        d4[q] = make_float4(acc[4 * q] / 8192.f, acc[4 * q + 1] / 8192.f, acc[4 * q + 2] / 8192.f,
                            acc[4 * q + 3] / 8192.f);
    } else {
#pragma unroll
      for (int p = 0; p < kPX; ++p)
        if (x + p < cols) drow[p] = acc[p] / 8192.f;
    }
    // x is even (kPX-aligned); even rows: outputs 0, 2, 4, 6 -> next plane (y/2, x/2 + q)
    if (nx.p && (y & 1) == 0 && (y >> 1) < nx.rows) {
      float* nrow = nx.p + (long long)(y >> 1) * nx.pitch + (x >> 1);
#pragma unroll
      for (int q = 0; q < kPX / 2; ++q)
        if ((x >> 1) + q < nx.cols) nrow[q] = acc[2 * q] / 8192.f;
    }
  }
}

// One plane per image: base blur of the input (octave 0, scale 0) and the
// Gaussian_Blur entry point when w is one of the unrolled widths.
template <int W>
__global__ __launch_bounds__(256) void blur_plane_kernel(const float* __restrict__ src,
                                                         long long spitch, long long simg,
                                                         float* __restrict__ dst, long long dpitch,
                                                         long long dimg, int rows, int cols,
                                                         const float* __restrict__ coef) {
  extern __shared__ float4 lds4[];
  const int b = blockIdx.z;
  blur_tile<W>(src + b * simg, spitch, rows, cols, dst + b * dimg, dpitch, coef,
               blockIdx.x * kTileW, blockIdx.y * kTY, reinterpret_cast<float*>(lds4));
}

struct OctaveArgs {
  float* gpyr;
  long long g_img;
  long long base_off;
  long long dst_off[4];
  const float* coef[4];
  int pitch, rows, cols, pad_;
  NextPlane nx;  // fused decimation of plane 2 (scale index 1), or p == nullptr
};

// The four non-base scales of one octave (src/sift.cpp:256-258): each is
// blurred from the octave base.  w = 4, 8, 12, 18 for sigma 1.6, 2.77, 4.23,
// 6.20 (sig[] at src/sift.cpp:240-245).
__global__ __launch_bounds__(256) void blur_octave_kernel(OctaveArgs A) {
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int z = blockIdx.z;
  const int b = z >> 2;
  const int si = 3 - (z & 3);  // heaviest scale first
  const float* src = A.gpyr + b * A.g_img + A.base_off;
  float* dst = A.gpyr + b * A.g_img + A.dst_off[si];
  const int x0 = blockIdx.x * kTileW, y0 = blockIdx.y * kTY;
  NextPlane nx = A.nx;
  if (nx.p) nx.p += b * A.g_img;
  switch (si) {
    case 0: blur_tile<4>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[0], x0, y0, lds); break;
    case 1: blur_tile<8>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[1], x0, y0, lds, nx); break;
    case 2: blur_tile<12>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[2], x0, y0, lds); break;
    default: blur_tile<18>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[3], x0, y0, lds); break;
  }
}

// Any kernel width (Gaussian_Blur with an arbitrary sigma): one output per
// lane, same tap chain, reads through L1/L2.
__global__ __launch_bounds__(256) void blur_generic_kernel(const float* __restrict__ src,
                                                           long long spitch, long long simg,
                                                           float* __restrict__ dst, long long dpitch,
                                                           long long dimg, int rows, int cols,
                                                           const float* __restrict__ coef, int w) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= cols || y >= rows) return;
  const float* s = src + b * simg;
  const int ks = 2 * w + 1;
  float acc = 0.f;
  for (int a = -w; a <= w; ++a) {
    const int yy = y + a;
    const bool rok = yy >= 0 && yy < rows - 1;
    for (int c = -w; c <= w; ++c) {
      const int xx = x + c;
      const float e = (rok && xx >= 0 && xx < cols - 1) ? s[(long long)yy * spitch + xx] : 0.f;
      acc = acc + e * coef[(a + w) * ks + (c + w)];
    }
  }
  dst[b * dimg + (long long)y * dpitch + x] = acc / 8192.f;
}

static size_t lds_bytes_for(int w) {
  switch (w) {
    case 4: return BlurTile<4>::LDS_FLOATS * 4;
    case 8: return BlurTile<8>::LDS_FLOATS * 4;
    case 12: return BlurTile<12>::LDS_FLOATS * 4;
    case 18: return BlurTile<18>::LDS_FLOATS * 4;
    default: return 0;
  }
}

void launch_blur_plane(hipStream_t st, int w, const float* coef, Plane src, float* dst,
                       long long dpitch, long long dimg, int rows, int cols, int batch) {
  const size_t lds = lds_bytes_for(w);
  if (lds) {
    dim3 grid((cols + kTileW - 1) / kTileW, (rows + kTY - 1) / kTY, batch);
    switch (w) {
      case 4: hipLaunchKernelGGL(blur_plane_kernel<4>, grid, dim3(256), lds, st, src.p, src.pitch, src.img_stride, dst, dpitch, dimg, rows, cols, coef); break;
      case 8: hipLaunchKernelGGL(blur_plane_kernel<8>, grid, dim3(256), lds, st, src.p, src.pitch, src.img_stride, dst, dpitch, dimg, rows, cols, coef); break;
      case 12: hipLaunchKernelGGL(blur_plane_kernel<12>, grid, dim3(256), lds, st, src.p, src.pitch, src.img_stride, dst, dpitch, dimg, rows, cols, coef); break;
      default: hipLaunchKernelGGL(blur_plane_kernel<18>, grid, dim3(256), lds, st, src.p, src.pitch, src.img_stride, dst, dpitch, dimg, rows, cols, coef); break;
    }
  } else {
    dim3 grid((cols + 63) / 64, (rows + 3) / 4, batch);
    hipLaunchKernelGGL(blur_generic_kernel, grid, dim3(256), 0, st, src.p, src.pitch, src.img_stride,
                       dst, dpitch, dimg, rows, cols, coef, w);
  }
}

// Octave o+1's plane 0 from this launch's plane 2 when it is an exact half
// (the caller then skips the decimation); else not fused.
static NextPlane next_plane(const Layout& L, int o, float* gpyr, bool fuse) {
  if (!fuse || o + 1 >= L.n_oct || L.oct[o].rows != 2 * L.oct[o + 1].rows || L.oct[o].cols != 2 * L.oct[o + 1].cols)
    return NextPlane{nullptr, 0, 0, 0};
  const Octave& N = L.oct[o + 1];
  return NextPlane{gpyr + N.g_off[0], N.pitch, N.rows, N.cols};
}

bool blur_fuses_decimation(const Layout& L, int o) {
  return o > 0 && L.oct[o - 1].rows == 2 * L.oct[o].rows && L.oct[o - 1].cols == 2 * L.oct[o].cols;
}

void launch_blur_octave(hipStream_t st, const Layout& L, int o, float* gpyr, const float* coefs,
                        const int* wsz, int batch, bool fuse_next) {
  const Octave& O = L.oct[o];
  OctaveArgs A;
  A.gpyr = gpyr;
  A.g_img = L.g_img;
  A.base_off = O.g_off[0];
  size_t coff = 0;
  for (int s = 0; s < 4; ++s) {
    A.dst_off[s] = O.g_off[s + 1];
    A.coef[s] = coefs + coff;
    coff += (size_t)(2 * wsz[s] + 1) * (2 * wsz[s] + 1);
  }
  A.pitch = O.pitch;
  A.rows = O.rows;
  A.cols = O.cols;
  A.pad_ = 0;
  A.nx = next_plane(L, o, gpyr, fuse_next);
  dim3 grid((O.cols + kTileW - 1) / kTileW, (O.rows + kTY - 1) / kTY, batch * 4);
  hipLaunchKernelGGL(blur_octave_kernel, grid, dim3(256), lds_bytes_for(18), st, A);
}

// ---- exact 2-D blur, small launches (round 3) ---------------------------------
// One 1080p image's octaves 1-3 give the 8-pixel-per-lane tiles only 80-1020
// workgroups: a wave then sits alone on its SIMD and issues 8 x 2 x (2w+1)^2
// instructions at one per 4 cycles (octaves 1-3: 81 / 63 / 65 us per launch,
// round 2's single-image trace).  Here a lane owns 2 adjacent outputs of a
// 32 x 16 tile, so a launch has 4x the waves and each wave a quarter of the
// chain.  Same float chain per output as blur_tile (kernel rows ascending,
// columns ascending, acc = acc + x * K, one / 8192 at the end), so the planes
// are bit-identical.  The (2w+1)^2 table sits in LDS and each kernel row's
// coefficients are read as broadcast ds_read_b128 into VGPRs (a VGPR operand
// issues at full rate, an SGPR one at half); the window is 19 ds_read_b64 per
// row for w = 18 (row pitch 96 = 32 mod 64 words: the two tile rows of a
// 32-lane pass fill opposite bank halves, conflict free).
// PX = 4 (round 6; a launch of >= kSmall4Min workgroups: one 1080p image's
// octave 1): 4 outputs per lane of a 64 x 16 tile, the window as ds_read_b128
// (row pitch 128 words: a 16-lane group's reads cover 64 distinct banks), so
// a kernel row costs 20 LDS reads per 296 VALU instead of 29 per 148 -- the
// 2-output form was LDS-issue-bound there (SQ_WAIT_INST_LDS 0.40 of the wave
// cycles, VALU issue 0.52).
constexpr int kSH = 16;
#ifndef SIFT_SMALL4_MIN
#define SIFT_SMALL4_MIN 1024  // A/B builds only (tools/build_var.sh)
#endif
constexpr long long kSmall4Min = SIFT_SMALL4_MIN;

template <int W, int PX = 2>
struct SmallTile {
  static constexpr int SW = 16 * PX;            // tile width
  static constexpr int SLP = PX == 4 ? 128 : 96;  // LDS row pitch (words)
  static constexpr int KS = 2 * W + 1;
  static constexpr int KP = (KS + 3) / 4 * 4;  // coefficient row pitch (b128 reads)
  static constexpr int NW = (KS + PX - 1 + PX - 1) / PX * PX;  // window values a lane reads per row
  static constexpr int LR = kSH + 2 * W, LW = SW + 2 * W;
  static constexpr int LDS_FLOATS = LR * SLP + KS * KP;
  static_assert(LW <= SLP && PX * 15 + NW <= LW, "row pitch / window reads inside the staged row");
};

template <int W, int PX = 2>
__device__ __forceinline__ void blur_small_tile(const float* __restrict__ src, long long spitch, int rows, int cols,
                                                float* __restrict__ dst, long long dpitch,
                                                const float* __restrict__ coef, int x0, int y0,
                                                float* __restrict__ lds,
                                                NextPlane nx = NextPlane{nullptr, 0, 0, 0}) {
  using T = SmallTile<W, PX>;
  constexpr int kSLP = T::SLP;
  const int t = threadIdx.x;
  float* kt = lds + T::LR * kSLP;
  for (int i = t; i < T::KS * T::KS; i += 256) {
    const int a = i / T::KS, b = i - a * T::KS;
    kt[a * T::KP + b] = coef[i];
  }
  for (int i = t; i < T::LR * T::LW; i += 256) {
    const int r = i / T::LW, c = i - r * T::LW;
    const int gy = y0 - W + r, gx = x0 - W + c;
    const bool ok = gy >= 0 && gy < rows - 1 && gx >= 0 && gx < cols - 1;
    lds[r * kSLP + c] = ok ? src[(long long)gy * spitch + gx] : 0.f;
  }
  __syncthreads();
  const int tx = t & 15, ty = t >> 4;
  float acc[PX];
#pragma unroll
  for (int i = 0; i < PX; ++i) acc[i] = 0.f;
#pragma unroll 1
  for (int a = 0; a < T::KS; ++a) {
    float k[T::KP];
    const float4* k4 = reinterpret_cast<const float4*>(kt + a * T::KP);
#pragma unroll
    for (int q = 0; q < T::KP / 4; ++q) {
      const float4 v = k4[q];
      k[4 * q] = v.x;
      k[4 * q + 1] = v.y;
      k[4 * q + 2] = v.z;
      k[4 * q + 3] = v.w;
    }
    float win[T::NW];
    if constexpr (PX == 4) {
      const float4* w4 = reinterpret_cast<const float4*>(lds + (ty + a) * kSLP + 4 * tx);
#pragma unroll
      for (int q = 0; q < T::NW / 4; ++q) {
        const float4 v = w4[q];
        win[4 * q] = v.x;
        win[4 * q + 1] = v.y;
        win[4 * q + 2] = v.z;
        win[4 * q + 3] = v.w;
      }
    } else {
      const float2* w2 = reinterpret_cast<const float2*>(lds + (ty + a) * kSLP + 2 * tx);
#pragma unroll
      for (int q = 0; q < T::NW / 2; ++q) {
        const float2 v = w2[q];
        win[2 * q] = v.x;
        win[2 * q + 1] = v.y;
      }
    }
#pragma unroll
    for (int b = 0; b < T::KS; ++b) {
      float p[PX];
#pragma unroll
      for (int i = 0; i < PX; ++i) p[i] = win[b + i] * k[b];
#pragma unroll
      for (int i = 0; i < PX; ++i) acc[i] = acc[i] + p[i];
    }
  }
  const int y = y0 + ty, x = x0 + PX * tx;
  if (y < rows) {
    float* drow = dst + (long long)y * dpitch + x;
#pragma unroll
    for (int i = 0; i < PX; ++i)
      if (x + i < cols) drow[i] = acc[i] / 8192.f;
    // x is even: outputs 0 (and 2) -> next plane (y/2, x/2 (+1)) on even rows
    if (nx.p && (y & 1) == 0 && (y >> 1) < nx.rows) {
#pragma unroll
      for (int i = 0; i < PX; i += 2)
        if (((x + i) >> 1) < nx.cols) nx.p[(long long)(y >> 1) * nx.pitch + ((x + i) >> 1)] = acc[i] / 8192.f;
    }
  }
}

template <int PX>
__global__ __launch_bounds__(256) void blur_small_kernel(OctaveArgs A) {
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int z = blockIdx.z;
  const int b = z >> 2;
  const int si = 3 - (z & 3);  // heaviest scale first
  const float* src = A.gpyr + b * A.g_img + A.base_off;
  float* dst = A.gpyr + b * A.g_img + A.dst_off[si];
  const int x0 = blockIdx.x * SmallTile<4, PX>::SW, y0 = blockIdx.y * kSH;
  NextPlane nx = A.nx;
  if (nx.p) nx.p += b * A.g_img;
  switch (si) {
    case 0: blur_small_tile<4, PX>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[0], x0, y0, lds); break;
    case 1: blur_small_tile<8, PX>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[1], x0, y0, lds, nx); break;
    case 2: blur_small_tile<12, PX>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[2], x0, y0, lds); break;
    default: blur_small_tile<18, PX>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[3], x0, y0, lds); break;
  }
}

// Workgroups of launch_blur_octave (8-pixel tiles) for this octave and batch.
long long blur_octave_tiles(const Layout& L, int o, int batch) {
  const Octave& O = L.oct[o];
  return (long long)((O.cols + kTileW - 1) / kTileW) * ((O.rows + kTY - 1) / kTY) * batch * 4;
}

void launch_blur_octave_small(hipStream_t st, const Layout& L, int o, float* gpyr, const float* coefs,
                              const int* wsz, int batch, bool fuse_next) {
  const Octave& O = L.oct[o];
  OctaveArgs A;
  A.gpyr = gpyr;
  A.g_img = L.g_img;
  A.base_off = O.g_off[0];
  size_t coff = 0;
  for (int s = 0; s < 4; ++s) {
    A.dst_off[s] = O.g_off[s + 1];
    A.coef[s] = coefs + coff;
    coff += (size_t)(2 * wsz[s] + 1) * (2 * wsz[s] + 1);
  }
  A.pitch = O.pitch;
  A.rows = O.rows;
  A.cols = O.cols;
  A.pad_ = 0;
  A.nx = next_plane(L, o, gpyr, fuse_next);
  const int rt = (O.rows + kSH - 1) / kSH;
  const long long wg4 = (long long)((O.cols + SmallTile<4, 4>::SW - 1) / SmallTile<4, 4>::SW) * rt * batch * 4;
  constexpr size_t lds4 = SmallTile<18, 4>::LDS_FLOATS * 4, lds2 = SmallTile<18, 2>::LDS_FLOATS * 4;
  constexpr int sw4 = SmallTile<4, 4>::SW, sw2 = SmallTile<4, 2>::SW;
  if (wg4 >= kSmall4Min)
    hipLaunchKernelGGL(blur_small_kernel<4>, dim3((O.cols + sw4 - 1) / sw4, rt, batch * 4), dim3(256), lds4, st, A);
  else
    hipLaunchKernelGGL(blur_small_kernel<2>, dim3((O.cols + sw2 - 1) / sw2, rt, batch * 4), dim3(256), lds2, st, A);
}

// ---- exact 2-D blur, symmetric scatter form (the SIFT_NCL tables) ----------
// Same float chain per output as blur_tile, about 24 % fewer VALU instructions.
// K[a][b] depends on a^2 + b^2 only (src/sift.cpp:103), so the product
// src'(r, x+b) * K[a][b] that output row r - a needs (its kernel row +a) is the
// same float as the one output row r + a needs (kernel row -a).  A lane owns
// one output column and walks down the source rows; accumulators for the
// 2w+1 outputs a source row touches stay in registers, and each source row is
// applied to all of them at once: per column offset b (ascending) and
// |a| = 0..w, one multiply feeds two adds.  Every output still receives its
// terms row by row (ascending r, i.e. ascending kernel row) and within a row
// by ascending b -- the reference's raster order -- so the result is the
// reference's chain bit for bit.  Rows outside [0, rows-1) contribute +0.0
// products (getSubMatrix padding, :116), which leave any sum that starts at
// +0.0 unchanged, so they are skipped.  Multiplies: (2w+1)(w+1) instead of
// (2w+1)^2 per output; adds unchanged.
//
// The tables are compile-time constants (build/sym_coefs.inc, printed by
// gen_sym_coefs.cpp from the library's own gauss_host.hpp): every multiply
// takes its coefficient as a literal operand, no scalar loads in the walk.
// sym_tables_match() re-checks them against the context's tables.
#include "../build/sym_coefs.inc"

template <int T> struct SymTab;
template <> struct SymTab<0> { static constexpr int W = kSymW0; };
template <> struct SymTab<1> { static constexpr int W = kSymW1; };
template <> struct SymTab<2> { static constexpr int W = kSymW2; };
template <> struct SymTab<3> { static constexpr int W = kSymW3; };
template <> struct SymTab<4> { static constexpr int W = kSymW4; };

template <int T>
__device__ __forceinline__ constexpr float symk(int a, int b) {
  if constexpr (T == 0) return kSymK0[a][b];
  else if constexpr (T == 1) return kSymK1[a][b];
  else if constexpr (T == 2) return kSymK2[a][b];
  else if constexpr (T == 3) return kSymK3[a][b];
  else return kSymK4[a][b];
}

static_assert(kSymW0 == 4 && kSymW1 == 4 && kSymW2 == 8 && kSymW3 == 12 && kSymW4 == 18,
              "SIFT_NCL kernel widths");

// One empty asm naming every product register: the multiplies of a column
// offset stay ahead of all its adds (separate asm statements would let the
// scheduler sink each multiply next to its first add again).
#define SIFT_V(i) "+v"(p[i])
__device__ __forceinline__ void pin_regs(float (&p)[5]) {
  asm volatile("" : SIFT_V(0), SIFT_V(1), SIFT_V(2), SIFT_V(3), SIFT_V(4));
}
__device__ __forceinline__ void pin_regs(float (&p)[9]) {
  asm volatile("" : SIFT_V(0), SIFT_V(1), SIFT_V(2), SIFT_V(3), SIFT_V(4), SIFT_V(5), SIFT_V(6), SIFT_V(7),
               SIFT_V(8));
}
__device__ __forceinline__ void pin_regs(float (&p)[13]) {
  asm volatile("" : SIFT_V(0), SIFT_V(1), SIFT_V(2), SIFT_V(3), SIFT_V(4), SIFT_V(5), SIFT_V(6), SIFT_V(7),
               SIFT_V(8), SIFT_V(9), SIFT_V(10), SIFT_V(11), SIFT_V(12));
}
__device__ __forceinline__ void pin_regs(float (&p)[19]) {
  asm volatile("" : SIFT_V(0), SIFT_V(1), SIFT_V(2), SIFT_V(3), SIFT_V(4), SIFT_V(5), SIFT_V(6), SIFT_V(7),
               SIFT_V(8), SIFT_V(9), SIFT_V(10), SIFT_V(11), SIFT_V(12), SIFT_V(13), SIFT_V(14), SIFT_V(15),
               SIFT_V(16), SIFT_V(17), SIFT_V(18));
}
#undef SIFT_V

// Source rows per loop step: narrow kernels take several so the loop and
// staging overhead is spread over enough arithmetic.
template <int W> struct SymRows { static constexpr int R = W <= 4 ? 4 : W <= 8 ? 2 : 1; };
template <int W> struct SymSeg {
  static constexpr int SEG = 64 + 2 * W;  // staged source columns [x0 - w, x0 + 64 + w)
  static constexpr int RING = 2 * SymRows<W>::R * SEG;  // two halves of R staged rows
};
constexpr int kSymRing = SymSeg<4>::RING;  // the largest (R = 4)
static_assert(SymSeg<8>::RING <= kSymRing && SymSeg<12>::RING <= kSymRing && SymSeg<18>::RING <= kSymRing,
              "ring size");

struct SymArgs {
  const float* src;
  long long s_pitch, s_img;
  float* dst[4];       // per slot, image 0
  long long d_pitch, d_img;
  float* nxt;          // the next octave's plane 0 (image 0) when it is plane 2's exact half, else null
  long long n_pitch;
  int rows, cols, strips, batch;
  int start[5];        // first wave of each slot; start[nslot] = grid size
  int chunk[4];        // output rows per wave, per slot
  int count[4];        // waves of each slot (start[] spaced by count rounded up to 8: whole XCD runs)
};

// Wave index within slot `slot` of block `wid`; -1: a padding block.  The
// blocks of one XCD (b, b + 8, ... under round-robin placement, speed only)
// take a contiguous run of the slot's waves, so neighbouring strips -- which
// read each other's w halo columns -- meet in one L2 (round 5: -36 % read
// traffic, same time -- the kernel is VALU-bound; profiles/r5_blur_xcd_ab.txt).
__device__ __forceinline__ int sym_local(const SymArgs& A, int slot, int wid) {
  const int n8 = A.start[slot + 1] - A.start[slot];
  const int local = ((wid - A.start[slot]) & 7) * (n8 >> 3) + ((wid - A.start[slot]) >> 3);
  return local < A.count[slot] ? local : -1;
}

// Wave-scope ordering of LDS accesses across lanes: no instruction, but the
// compiler may not move loads or stores across it.
__device__ __forceinline__ void wave_sync_b() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave: output columns [x0, x0 + 64) x rows [y0, y1) of one plane.
template <int T>
__device__ __forceinline__ void sym_walk(const SymArgs& A, int slot, int local, float* __restrict__ ring) {
  constexpr int W = SymTab<T>::W, R = SymRows<W>::R, NA = 2 * W + R, SEG = SymSeg<W>::SEG;
  const int lane = threadIdx.x & 63;
  const int strip = local % A.strips, t = local / A.strips;
  const int b = t % A.batch, ck = t / A.batch;
  const int x0 = strip * 64, y0 = ck * A.chunk[slot], y1 = min(y0 + A.chunk[slot], A.rows);
  const int rows = A.rows, cols = A.cols;
  const float* __restrict__ src = A.src + b * A.s_img;
  float* __restrict__ dst = A.dst[slot] + b * A.d_img;
  const int xo = x0 + lane;
  // staging: lane stages segment elements lane and lane + 64 (< SEG)
  const int cl = x0 - W + lane, ch = cl + 64;
  const bool okl = cl >= 0 && cl < cols - 1;
  const bool okh = lane < 2 * W && ch >= 0 && ch < cols - 1;
  const float* pl = src + (okl ? cl : 0);
  const float* ph = src + (okh ? ch : 0);
  float vl[R], vh[R];
  auto fetch = [&](int r0) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const long long ro = (long long)min(max(r0 + i, 0), rows - 1) * A.s_pitch;
      vl[i] = pl[ro];
      vh[i] = okh ? ph[ro] : 0.f;
    }
  };
  auto stage = [&](int h) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float* d = ring + (h * R + i) * SEG;
      d[lane] = okl ? vl[i] : 0.f;
      if (lane < 2 * W) d[lane + 64] = vh[i];
    }
  };
  float acc[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) acc[k] = 0.f;
  // acc[k] is output row r0 - W + k; rows above 0 add nothing, so the walk
  // starts at the first row that can: max(y0 - W, 0)
  int r0 = max(y0 - W, 0);
  fetch(r0);
  stage(0);
  // Lanes read ring words other lanes wrote: order the stores before every
  // later read and every read before the next reuse of that ring half (each
  // wave_sync sits between the reads of a half and its next stage).
  wave_sync_b();
  int h = 0;
  for (; r0 < y1 + W; r0 += R) {
    fetch(r0 + R);  // next step's rows, in flight during this step
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = r0 + i;
      if (r < rows - 1) {  // uniform; r >= 0 always
        const float* lr = ring + (h * R + i) * SEG + lane;
        float x[2 * W + 1];
#pragma unroll
        for (int c = 0; c <= 2 * W; ++c) x[c] = lr[c];
#pragma unroll
        for (int c = 0; c <= 2 * W; ++c) {
          const int bb = c < W ? W - c : c - W;
          // the w+1 products of this column offset first, in distinct
          // registers (pinned by the empty asm), then their 2w+1 adds: no add
          // waits on the multiply right before it
          float p[W + 1];
#pragma unroll
          for (int a = 0; a <= W; ++a) p[a] = x[c] * symk<T>(a, bb);
          pin_regs(p);
#pragma unroll
          for (int a = 0; a <= W; ++a) {
            acc[i + W - a] = acc[i + W - a] + p[a];  // output r - a (kernel row +a)
            if (a) acc[i + W + a] = acc[i + W + a] + p[a];  // output r + a (kernel row -a)
          }
        }
      }
      const int y = r - W;  // complete: its last kernel row was r
      if (y >= y0 && y < y1 && xo < cols) {
        const float v = acc[i] / 8192.f;
        dst[(long long)y * A.d_pitch + xo] = v;
        // plane nOctaveLayers (slot 2) -> the next octave's plane 0, INTER_NEAREST
        // exact half (src/sift.cpp:252-254): pixel (2y', 2x') -> (y', x')
        if constexpr (T == 2)
          if (A.nxt && ((y | xo) & 1) == 0) A.nxt[b * A.d_img + (long long)(y >> 1) * A.n_pitch + (xo >> 1)] = v;
      }
    }
#pragma unroll
    for (int k = 0; k < NA - R; ++k) acc[k] = acc[k + R];
#pragma unroll
    for (int k = NA - R; k < NA; ++k) acc[k] = 0.f;
    h ^= 1;
    stage(h);
    wave_sync_b();
  }
}

// Waves are independent (one 64-lane workgroup each).  The octave kernel's
// slots run in launch order, widest kernel first: slot s blurs scale 4 - s.
// The kernel holds 168 VGPRs, 3 waves per SIMD instead of the 4 its 101
// allow.  Alone it runs as fast (3 waves keep the 2-cycle VALU issue full);
// beside another stream's latency-bound kernels (bench.py's 2 streams) the
// step is 3-4 % shorter, measured in rounds 2-3 (4 waves per SIMD: 6,448-6,499
// vs 6,513-6,552 Mpix/s).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void blur_sym_kernel(SymArgs A) {
  __shared__ float ring[kSymRing];
  asm volatile("; hold v160-v167" ::: "v160", "v167");
  const int wid = blockIdx.x;
  const int slot = wid >= A.start[3] ? 3 : wid >= A.start[2] ? 2 : wid >= A.start[1] ? 1 : 0;
  const int local = sym_local(A, slot, wid);
  if (local < 0) return;
  switch (slot) {
    case 0: sym_walk<4>(A, 0, local, ring); break;
    case 1: sym_walk<3>(A, 1, local, ring); break;
    case 2: sym_walk<2>(A, 2, local, ring); break;
    default: sym_walk<1>(A, 3, local, ring); break;
  }
}

// The octave-0 base (createInitialImage's blur of the input, table 0).
__global__ __launch_bounds__(64) void blur_sym_base_kernel(SymArgs A) {
  __shared__ float ring[SymSeg<kSymW0>::RING];
  const int local = sym_local(A, 0, blockIdx.x);
  if (local < 0) return;
  sym_walk<0>(A, 0, local, ring);
}

bool sym_tables_match(const float* coefs) {
  // api.hip's layout: the base table, then sig[1..4]'s, each (2w+1)^2 row-major
  const int ws[5] = {kSymW0, kSymW1, kSymW2, kSymW3, kSymW4};
  size_t at = 0;
  for (int t = 0; t < 5; ++t) {
    const int w = ws[t], ks = 2 * w + 1;
    for (int a = -w; a <= w; ++a)
      for (int b = -w; b <= w; ++b) {
        const int aa = a < 0 ? -a : a, bb = b < 0 ? -b : b;
        float k = 0;
        switch (t) {
          case 0: k = kSymK0[aa][bb]; break;
          case 1: k = kSymK1[aa][bb]; break;
          case 2: k = kSymK2[aa][bb]; break;
          case 3: k = kSymK3[aa][bb]; break;
          default: k = kSymK4[aa][bb]; break;
        }
        if (__builtin_memcmp(&k, &coefs[at + (a + w) * ks + (b + w)], 4) != 0) return false;
      }
    at += (size_t)ks * ks;
  }
  return true;
}

// VALU instructions per source row and output column of table width w (the
// multiplies and adds of the walk plus the accumulator shift).
static double sym_row_cost(int w) { return (2. * w + 1) * (w + 1) + (2. * w + 1) * (2. * w + 1) + 2. * w + 8; }

// Output rows per wave for each slot.  A wave issues at most one VALU
// instruction per 4 cycles (two waves per SIMD fill the 2-cycle issue), so a
// launch cannot end before its longest wave: the widest kernel's chunk is
// sized so that wave needs at most cp (0.7 for the octaves, measured) of the
// launch's whole-chip time (a 64 x 1080p octave 0: one 1080-row chunk; 16
// images per launch, as on one of bench.py's 4 streams: 270-row chunks).
// Taller chunks recompute less halo (w rows above and below a chunk); the
// other slots get chunks of about the same work (rows x row cost).
static int sym_simds() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
    return 4 * cus;
  }();
  return n;
}

static void sym_plan(SymArgs& A, const int* w, int nslot, double cp) {
  double total = 0;
  for (int s = 0; s < nslot; ++s) total += (double)A.strips * A.batch * A.rows * sym_row_cost(w[s]);
  // longest wave (rows_w0 x cost x 4 cycles) <= cp x whole-chip time (total x 2 cycles / SIMDs)
  int rows_w0 = (int)(cp * total / (2.0 * sym_simds() * sym_row_cost(w[0])));
  rows_w0 = std::max(64, rows_w0);
  const double per = sym_row_cost(w[0]) * rows_w0;
  int start = 0;
  for (int s = 0; s < nslot; ++s) {
    int ch = std::max(1, (int)ceil(A.rows * sym_row_cost(w[s]) / per - 1e-9));
    const int h = (A.rows + ch - 1) / ch;
    ch = (A.rows + h - 1) / h;
    A.chunk[s] = h;
    A.start[s] = start;
    A.count[s] = A.strips * A.batch * ch;
    start += (A.count[s] + 7) / 8 * 8;
  }
  for (int s = nslot; s < 5; ++s) A.start[s] = start;
}

void launch_blur_base_sym(hipStream_t st, Plane src, float* dst, long long dpitch, long long dimg, int rows,
                          int cols, int batch) {
  SymArgs A{};
  A.src = src.p;
  A.s_pitch = src.pitch;
  A.s_img = src.img_stride;
  A.dst[0] = dst;
  A.d_pitch = dpitch;
  A.d_img = dimg;
  A.rows = rows;
  A.cols = cols;
  A.strips = (cols + 63) / 64;
  A.batch = batch;
  const int w[1] = {kSymW0};
#ifndef SIFT_SYM_BASE_CP
#define SIFT_SYM_BASE_CP 0.35  // A/B builds only (tools/build_var.sh)
#endif
  sym_plan(A, w, 1, SIFT_SYM_BASE_CP);  // measured: 4 chunks of a 1080p base, not 2
  hipLaunchKernelGGL(blur_sym_base_kernel, dim3(A.start[1]), dim3(64), 0, st, A);
}

void launch_blur_octave_sym(hipStream_t st, const Layout& L, int o, float* gpyr, int batch, bool fuse_next) {
  const Octave& O = L.oct[o];
  SymArgs A{};
  const NextPlane nx = next_plane(L, o, gpyr, fuse_next);
  A.nxt = nx.p;
  A.n_pitch = nx.pitch;
  A.src = gpyr + O.g_off[0];
  A.s_pitch = O.pitch;
  A.s_img = L.g_img;
  for (int s = 0; s < 4; ++s) A.dst[s] = gpyr + O.g_off[4 - s];
  A.d_pitch = O.pitch;
  A.d_img = L.g_img;
  A.rows = O.rows;
  A.cols = O.cols;
  A.strips = (O.cols + 63) / 64;
  A.batch = batch;
  const int w[4] = {kSymW4, kSymW3, kSymW2, kSymW1};
  sym_plan(A, w, 4, 0.7);
  hipLaunchKernelGGL(blur_sym_kernel, dim3(A.start[4]), dim3(64), 0, st, A);
}

// ---- resize INTER_NEAREST to the next octave (src/sift.cpp:252-254) -------
__global__ __launch_bounds__(256) void decimate_kernel(const float* __restrict__ gpyr, float* out,
                                                       long long g_img, long long src_off,
                                                       long long dst_off, int spitch, int srows,
                                                       int scols, int dpitch, int drows, int dcols,
                                                       double ify, double ifx) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= dcols || y >= drows) return;
  int sy = (int)floor(y * ify);
  sy = sy < srows - 1 ? sy : srows - 1;
  int sx = (int)floor(x * ifx);
  sx = sx < scols - 1 ? sx : scols - 1;
  out[b * g_img + dst_off + (long long)y * dpitch + x] =
      gpyr[b * g_img + src_off + (long long)sy * spitch + sx];
}

void launch_decimate(hipStream_t st, const Layout& L, int o, float* gpyr, int batch) {
  const Octave& S = L.oct[o - 1];
  const Octave& D = L.oct[o];
  const double ifx = 1. / ((double)D.cols / S.cols), ify = 1. / ((double)D.rows / S.rows);
  dim3 grid((D.cols + 63) / 64, (D.rows + 3) / 4, batch);
  hipLaunchKernelGGL(decimate_kernel, grid, dim3(256), 0, st, gpyr, gpyr, L.g_img, S.g_off[kLayers],
                     D.g_off[0], S.pitch, S.rows, S.cols, D.pitch, D.rows, D.cols, ify, ifx);
}

// ---- DoG, src/sift.cpp:265-283: dog[s] = g[s+1] - g[s] ---------------------
__global__ __launch_bounds__(256) void dog_kernel(const float* __restrict__ gpyr, float* __restrict__ dog,
                                                  long long g_img, long long d_img, long long g0,
                                                  long long plane, long long d0, long long n4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int z = blockIdx.y;
  const int b = z >> 2, s = z & 3;
  const float4* a = reinterpret_cast<const float4*>(gpyr + b * g_img + g0 + s * plane);
  const float4* c = reinterpret_cast<const float4*>(gpyr + b * g_img + g0 + (s + 1) * plane);
  float4* d = reinterpret_cast<float4*>(dog + b * d_img + d0 + s * plane);
  const float4 x = a[i], y = c[i];
  d[i] = make_float4(y.x - x.x, y.y - x.y, y.z - x.z, y.w - x.w);
}

void launch_dog(hipStream_t st, const Layout& L, int o, const float* gpyr, float* dog, int batch) {
  const Octave& O = L.oct[o];
  const long long plane = (long long)O.rows * O.pitch;
  const long long n4 = plane / 4;
  dim3 grid((unsigned)((n4 + 255) / 256), batch * 4);
  hipLaunchKernelGGL(dog_kernel, grid, dim3(256), 0, st, gpyr, dog, L.g_img, L.d_img, O.g_off[0],
                     plane, O.d_off[0], n4);
}

// ---- Gaussian_Blur_1D, src/sift.cpp:170-217 ---------------------------------
// Taps k in [-ks/2, ks/2 - 1] (the reference's asymmetric loop, :196, :207);
// vertical pass zeroes rows >= rows-1, horizontal pass columns >= cols-1.
__global__ __launch_bounds__(256) void blur1d_v_kernel(const float* __restrict__ src, long long spitch,
                                                       long long simg, float* __restrict__ tmp,
                                                       long long pitch, long long img, int rows,
                                                       int cols, const float* __restrict__ k, int ks) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= cols || y >= rows) return;
  const float* s = src + b * simg;
  float acc = 0;
  for (int t = -ks / 2; t < ks / 2; ++t)
    acc += (y + t < 0 || y + t >= rows - 1) ? 0 : s[(long long)(y + t) * spitch + x] * k[t + ks / 2];
  tmp[b * img + (long long)y * pitch + x] = acc;
}

__global__ __launch_bounds__(256) void blur1d_h_kernel(const float* __restrict__ tmp, float* __restrict__ dst,
                                                       long long pitch, long long img, int rows,
                                                       int cols, const float* __restrict__ k, int ks) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= cols || y >= rows) return;
  const float* r = tmp + b * img + (long long)y * pitch;
  float acc = 0;
  for (int t = -ks / 2; t < ks / 2; ++t)
    acc += (x + t < 0 || x + t >= cols - 1) ? 0 : r[x + t] * k[t + ks / 2];
  dst[b * img + (long long)y * pitch + x] = acc;
}

void launch_blur_1d(hipStream_t st, int w, const float* coef1d, Plane src, float* tmp, float* dst,
                    long long pitch, long long img, int rows, int cols, int batch) {
  dim3 grid((cols + 63) / 64, (rows + 3) / 4, batch);
  const int ks = 2 * w + 1;
  hipLaunchKernelGGL(blur1d_v_kernel, grid, dim3(256), 0, st, src.p, src.pitch, src.img_stride, tmp,
                     pitch, img, rows, cols, coef1d, ks);
  hipLaunchKernelGGL(blur1d_h_kernel, grid, dim3(256), 0, st, tmp, dst, pitch, img, rows, cols,
                     coef1d, ks);
}

// ---- synthetic input, SURVEY.md 8(d) row d2 ---------------------------------
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256) void synth_kernel(float* out, int rows, int cols, long long pitch,
                                                    long long img_stride, int seed_base) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= cols || y >= rows) return;
  const int S[6] = {3, 6, 12, 24, 48, 96};
  const int A[6] = {48, 56, 56, 48, 40, 32};
  const uint32_t s = 0x5EED0000u + (uint32_t)(seed_base + b);
  int acc = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t salt = s * 0x9E3779B1u + (uint32_t)k * 0x85EBCA6Bu;
    const int gx = x / S[k], gy = y / S[k];
    const int fx = (x % S[k]) * 256 / S[k], fy = (y % S[k]) * 256 / S[k];
    const uint32_t ax0 = (uint32_t)gx * 73856093u, ax1 = (uint32_t)(gx + 1) * 73856093u;
    const uint32_t by0 = (uint32_t)gy * 19349663u, by1 = (uint32_t)(gy + 1) * 19349663u;
    const int l00 = (int)(lowbias32(ax0 ^ by0 ^ salt) & 255) - 128;
    const int l10 = (int)(lowbias32(ax1 ^ by0 ^ salt) & 255) - 128;
    const int l01 = (int)(lowbias32(ax0 ^ by1 ^ salt) & 255) - 128;
    const int l11 = (int)(lowbias32(ax1 ^ by1 ^ salt) & 255) - 128;
    const int v = ((l00 * (256 - fx) + l10 * fx) * (256 - fy) + (l01 * (256 - fx) + l11 * fx) * fy) >> 16;
    acc += A[k] * v;
  }
  int p = 128 + (acc >> 7);
  p = p < 0 ? 0 : p > 255 ? 255 : p;
  out[b * img_stride + (long long)y * pitch + x] = (float)p;
}

void launch_synth(hipStream_t st, float* out, int batch, int rows, int cols, long long pitch,
                  long long img_stride, int seed_base) {
  dim3 grid((cols + 63) / 64, (rows + 3) / 4, batch);
  hipLaunchKernelGGL(synth_kernel, grid, dim3(256), 0, st, out, rows, cols, pitch, img_stride,
                     seed_base);
}

}  // namespace sift
