// frontend.hip -- the reference's image front end for gfx950.
//
// readImage (src/main.cpp:79-87): imread -> BGR bytes; for the scene,
// resize(img, img, Size(960, 960)) (INTER_LINEAR on 8UC3); cvtColor with
// COLOR_RGB2GRAY applied to those BGR bytes; convertTo CV_32F.  Decoding stays
// on the host (PIL / libjpeg); this kernel takes the decoded bytes so a caller
// uploads 3 B per pixel instead of a 4-B float plane and the conversion runs
// beside the rest of the path.
//
// Arithmetic (OpenCV 4.x, x86 SSE2 path; restated in oracle/frontend.py):
//   * resize coefficients: fx = (float)((dx + 0.5) * (W / W') - 0.5),
//     sx = cvFloor(fx), fx -= sx, clamped to [0, W-1] with fx = 0 at the
//     edges; alpha = cvRound((1 - fx) * 2048), cvRound(fx * 2048) as shorts;
//     the same for rows, except that fy is not clamped and the two tap rows
//     are clipped to [0, H-1].  Horizontal pass: h = S[sx]*a0 + S[sx+1]*a1 (exact
//     ints, the second tap dropped at the right edge); vertical pass in the
//     SIMD form VResizeLinearVec_32s8u:
//       v = (((h0 >> 4) * b0 >> 16) + ((h1 >> 4) * b1 >> 16) + 2) >> 2
//     (saturated to 8 bits) for the elements its 16- and 8-lane loops cover,
//     the scalar (h0*b0 + h1*b1 + 2^21) >> 22 for the row's last few.  Parity against OpenCV itself is unpinned (its
//     IPP / scalar-tail paths round differently; no OpenCV here).
//   * COLOR_RGB2GRAY on BGR data: Y = (4899*B + 9617*G + 1868*R + 8192) >> 14
//     (the R coefficient lands on B) -- the same formula that built the
//     committed fixture tests/golden/book_gray.pgm.
// Bound: HBM / launch (3 B in, 4 B out per pixel); one lane per output pixel.
#include "common.hpp"

namespace sift {

namespace {

struct Taps1 {
  int s;       // first source index (second is min(s + 1, n - 1))
  int a0, a1;  // short coefficients, sum 2048
};

// Resize coefficients of output index d (OpenCV resizeGeneric setup,
// INTER_LINEAR).  Columns (CLAMP): the source index is clamped with f = 0 at
// both edges.  Rows: f is not clamped; the two tap rows are clipped to
// [0, n-1] when fetched (both taps may read the same row).
template <bool CLAMP>
__device__ __forceinline__ Taps1 lin_taps(int d, double scale, int n) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = cv_floor(f);
  f -= s;
  if (CLAMP && s < 0) {
    f = 0.f;
    s = 0;
  }
  if (CLAMP && s >= n - 1) {
    f = 0.f;
    s = n - 1;
  }
  Taps1 t;
  t.s = s;
  t.a0 = cv_round((1.f - f) * 2048.f);
  t.a1 = cv_round(f * 2048.f);
  return t;
}

__global__ __launch_bounds__(256) void bgr8_gray_kernel(const uint8_t* __restrict__ src, long long sstride,
                                                        long long simg, int srows, int scols,
                                                        float* __restrict__ dst, long long dpitch, long long dimg,
                                                        int drows, int dcols, int resize) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  if (x >= dcols || y >= drows) return;
  const uint8_t* s = src + b * simg;
  int bgr[3];
  if (!resize) {
    const uint8_t* p = s + (long long)y * sstride + 3 * x;
    bgr[0] = p[0];
    bgr[1] = p[1];
    bgr[2] = p[2];
  } else {
    const Taps1 tx = lin_taps<true>(x, (double)scols / dcols, scols);
    const Taps1 ty = lin_taps<false>(y, (double)srows / drows, srows);
    const int x1 = tx.s + 1 < scols ? tx.s + 1 : tx.s;  // a1 == 0 there
    const int y0 = min(max(ty.s, 0), srows - 1), y1 = min(max(ty.s + 1, 0), srows - 1);
    const uint8_t* r0 = s + (long long)y0 * sstride;
    const uint8_t* r1 = s + (long long)y1 * sstride;
    // elements [0, vtail) of a row go through the 16- then 8-lane SIMD loops,
    // the rest through the scalar FixedPtCast tail
    const int n = 3 * dcols;
    int vtail = n / 16 * 16;
    while (vtail < n - 8) vtail += 8;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int h0 = r0[3 * tx.s + c] * tx.a0 + r0[3 * x1 + c] * tx.a1;
      const int h1 = r1[3 * tx.s + c] * tx.a0 + r1[3 * x1 + c] * tx.a1;
      int v = 3 * x + c < vtail ? ((((h0 >> 4) * ty.a0) >> 16) + (((h1 >> 4) * ty.a1) >> 16) + 2) >> 2
                                : (h0 * ty.a0 + h1 * ty.a1 + (1 << 21)) >> 22;
      bgr[c] = v < 0 ? 0 : v > 255 ? 255 : v;
    }
  }
  const int g = (4899 * bgr[0] + 9617 * bgr[1] + 1868 * bgr[2] + 8192) >> 14;
  dst[b * dimg + (long long)y * dpitch + x] = (float)g;
}

}  // namespace

void launch_bgr8_gray(hipStream_t st, const uint8_t* src, long long sstride, long long simg, int srows, int scols,
                      float* dst, long long dpitch, long long dimg, int drows, int dcols, int batch) {
  const int resize = srows != drows || scols != dcols;
  dim3 grid((dcols + 63) / 64, (drows + 3) / 4, batch);
  hipLaunchKernelGGL(bgr8_gray_kernel, grid, dim3(256), 0, st, src, sstride, simg, srows, scols, dst, dpitch,
                     dimg, drows, dcols, resize);
}

}  // namespace sift
