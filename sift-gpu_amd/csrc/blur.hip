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

namespace sift {

// ---- coefficients (host), src/sift.cpp:95-108 -----------------------------
int gaussian_kernel_host(float sigma, float* coeff) {
  int w = (int)floor(3 * sigma);
  int size = 2 * w + 1;
  double norm = 1. / (2 * kRefPi * sigma * sigma);  // double chain
  double den = (double)(2 * sigma * sigma);          // float chain, then double
  if (coeff)
    for (int a = -w; a <= w; ++a)
      for (int b = -w; b <= w; ++b) {
        double g = norm * exp(-(a * a + b * b) * 1. / den);
        g = g * 8192;
        coeff[(a + w) * size + (b + w)] = (float)g;
      }
  return size;
}

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

template <int W>
__device__ __forceinline__ void blur_tile(const float* __restrict__ src, long long spitch, int rows,
                                          int cols, float* __restrict__ dst, long long dpitch,
                                          const float* __restrict__ coef, int x0, int y0,
                                          float* __restrict__ lds) {
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
  switch (si) {
    case 0: blur_tile<4>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[0], x0, y0, lds); break;
    case 1: blur_tile<8>(src, A.pitch, A.rows, A.cols, dst, A.pitch, A.coef[1], x0, y0, lds); break;
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

void launch_blur_octave(hipStream_t st, const Layout& L, int o, float* gpyr, const float* coefs,
                        const int* wsz, int batch) {
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
  dim3 grid((O.cols + kTileW - 1) / kTileW, (O.rows + kTY - 1) / kTY, batch * 4);
  hipLaunchKernelGGL(blur_octave_kernel, grid, dim3(256), lds_bytes_for(18), st, A);
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
