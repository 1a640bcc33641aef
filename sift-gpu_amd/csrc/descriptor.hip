// descriptor.hip -- 128-D descriptor (reference src/sift.cpp:579-753) for gfx950.
//
// One wave per keypoint.  The reference builds the 6x6x10 trilinear
// histogram by adding samples in window raster order, so each bin's float
// sum has a fixed order.  The wave keeps that order:
//   * the (2r+1)^2 window (r <= 40, so <= 6561 samples) is walked in chunks of
//     64 raster-consecutive samples, one per lane: rotation, bounds, gradient
//     (4 neighbour loads), exp32f / fastAtan2 / magnitude and the 8 trilinear
//     weights are computed in parallel and parked in LDS;
//   * the chunk's valid samples (a wave-uniform ballot mask) are then added in
//     lane order; the 8 corners of one sample hit 8 distinct bins, so lanes
//     0-7 add one corner each -- one LDS read-modify-write per sample;
//   * fold, 0.2 clamp, uchar quantisation and the RootSIFT-style
//     normalisation (src/sift.cpp:676-721) keep the reference's sequential
//     sums (one lane) and run the element-wise parts across the wave.
#include "common.hpp"

#include <float.h>

namespace sift {

__device__ __forceinline__ void wave_sync_d() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kHistLen = (kDescW + 2) * (kDescW + 2) * (kDescBins + 2);  // 360

struct DescArgs {
  Layout L;
  const float* gpyr;
  const MathConsts* mc;
  const sift_keypoint* kpts;
  const int* img_kp_off;  // [batch+1]
  int batch;
  int kp_cap;
  float* desc;
  int first_octave;
  int* err_flag;
};

__global__ __launch_bounds__(256) void descriptor_kernel(DescArgs A) {
  __shared__ float hist[4][kHistLen + 8];
  __shared__ int ridx[4][64];
  __shared__ float rval[4][8][64];
  __shared__ float vec[4][kDescLen];
  __shared__ float bc[4][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int d = kDescW, nb = kDescBins;
  int n = A.img_kp_off[A.batch];
  if (n > A.kp_cap) n = A.kp_cap;
  const ExpConsts ek = A.mc->e;
  const AtanConsts ak = A.mc->t;
  const float* etab = A.mc->exptab;
  // corner offsets of hist[idx] += v_rco000 ... v_rco111 (src/sift.cpp:665-672)
  const int coff[8] = {0, 1, nb + 2, nb + 3, (d + 2) * (nb + 2), (d + 2) * (nb + 2) + 1,
                       (d + 3) * (nb + 2), (d + 3) * (nb + 2) + 1};
  const int my_off = coff[lane & 7];

  for (int k = blockIdx.x * 4 + wv; k < n; k += gridDim.x * 4) {
    // image of keypoint k: offsets are ascending, batch is small
    int b = 0;
    while (b + 1 < A.batch && A.img_kp_off[b + 1] <= k) ++b;
    const sift_keypoint kp = A.kpts[k];
    // ---- unpackOctave + calDescriptor body, src/sift.cpp:724-751 ----
    int octave = kp.octave & 255;
    const int layer = (kp.octave >> 8) & 255;
    octave = octave < 128 ? octave : (-128 | octave);
    const float scale = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
    const int oi = octave - A.first_octave;
    if (oi < 0 || oi >= A.L.n_oct || layer > kLayers + 2) {  // CV_Assert at :744
      if (lane == 0) atomicOr(A.err_flag, 1);
      for (int q = lane; q < kDescLen; q += 64) A.desc[(long long)k * kDescLen + q] = 0.f;
      continue;
    }
    const float size = kp.size * scale;
    const float ptx = kp.x * scale, pty = kp.y * scale;
    float ori = 360.f - kp.angle;
    if (fabsf(ori - 360.f) < FLT_EPSILON) ori = 0.f;
    const float scl = size * 0.5f;
    const Octave& O = A.L.oct[oi];
    const long long pitch = O.pitch;
    const float* img = A.gpyr + b * A.L.g_img + O.g_off[layer];
    const int rows = O.rows, cols = O.cols;
    // ---- calcSIFTDescriptor, src/sift.cpp:579-722 ----
    const int px = cv_round(ptx), py = cv_round(pty);
    float cos_t = cosf_cr(ori * (float)(kCvPi / 180));
    float sin_t = sinf_cr(ori * (float)(kCvPi / 180));
    const float bins_per_rad = nb / 360.f;
    const float exp_scale = -1.f / (d * d * 0.5f);
    const float hist_width = 3.f * scl;
    int radius = cv_round(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    const int diag = (int)sqrt(((double)cols) * cols + ((double)rows) * rows);
    radius = radius < diag ? radius : diag;
    cos_t /= hist_width;
    sin_t /= hist_width;
    for (int q = lane; q < kHistLen; q += 64) hist[wv][q] = 0.f;
    wave_sync_d();
    const int D = 2 * radius + 1;
    const int ns = D * D;
    for (int base = 0; base < ns; base += 64) {
      const int s = base + lane;
      bool valid = false;
      int idx = 0;
      float v[8];
      if (s < ns) {
        const int i = s / D - radius, j = s % D - radius;
        const float c_rot = j * cos_t - i * sin_t;
        const float r_rot = j * sin_t + i * cos_t;
        float rbin = r_rot + d / 2 - 0.5f;
        float cbin = c_rot + d / 2 - 0.5f;
        const int r = py + i, c = px + j;
        if (rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < rows - 1 && c > 0 &&
            c < cols - 1) {
          valid = true;
          const float* row = img + (long long)r * pitch;
          const float dx = (float)(row[c + 1] - row[c - 1]);
          const float dy = (float)(row[c - pitch] - row[c + pitch]);
          const float w = exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, etab, ek);
          const float o_deg = fast_atan2(dy, dx, ak);
          const float mag0 = magnitude(dx, dy);
          float obin = (o_deg - ori) * bins_per_rad;
          const float mag = mag0 * w;
          const int r0 = cv_floor(rbin), c0 = cv_floor(cbin);
          int o0 = cv_floor(obin);
          rbin -= r0;
          cbin -= c0;
          obin -= o0;
          if (o0 < 0) o0 += nb;
          if (o0 >= nb) o0 -= nb;
          const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
          const float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
          const float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
          v[7] = v_rc11 * obin;
          v[6] = v_rc11 - v[7];
          v[5] = v_rc10 * obin;
          v[4] = v_rc10 - v[5];
          v[3] = v_rc01 * obin;
          v[2] = v_rc01 - v[3];
          v[1] = v_rc00 * obin;
          v[0] = v_rc00 - v[1];
          idx = ((r0 + 1) * (d + 2) + c0 + 1) * (nb + 2) + o0;
        }
      }
      unsigned long long m = __ballot(valid);
      if (valid) {
        ridx[wv][lane] = idx;
#pragma unroll
        for (int q = 0; q < 8; ++q) rval[wv][q][lane] = v[q];
      }
      wave_sync_d();
      while (m) {  // wave-uniform loop over the chunk's valid samples, in order
        const int sl = __builtin_ctzll(m);
        m &= m - 1;
        if (lane < 8) {
          const int h = ridx[wv][sl] + my_off;
          hist[wv][h] = hist[wv][h] + rval[wv][lane][sl];
        }
      }
      wave_sync_d();
    }
    // ---- circular fold + copy (src/sift.cpp:676-684) ----
    if (lane < d * d) {
      const int i = lane / d, j = lane % d;
      const int idx = ((i + 1) * (d + 2) + (j + 1)) * (nb + 2);
      float* h = hist[wv] + idx;
      h[0] = h[0] + h[nb];
      h[1] = h[1] + h[nb + 1];
#pragma unroll
      for (int q = 0; q < nb; ++q) vec[wv][(i * d + j) * nb + q] = h[q];
    }
    wave_sync_d();
    // ---- hysteresis + quantisation + RootSIFT (src/sift.cpp:689-721) ----
    float* dv = vec[wv];
    if (lane == 0) {
      float nrm2 = 0;
      for (int q = 0; q < kDescLen; ++q) nrm2 = nrm2 + dv[q] * dv[q];
      bc[wv][0] = sqrtf(nrm2) * 0.2f;
    }
    wave_sync_d();
    const float thr = bc[wv][0];
    for (int q = lane; q < kDescLen; q += 64) dv[q] = dv[q] < thr ? dv[q] : thr;
    wave_sync_d();
    if (lane == 0) {
      float nrm2 = 0;
      for (int q = 0; q < kDescLen; ++q) nrm2 = nrm2 + dv[q] * dv[q];
      const float sq = sqrtf(nrm2);
      bc[wv][1] = 512.f / (sq < FLT_EPSILON ? FLT_EPSILON : sq);
    }
    wave_sync_d();
    const float nrm2s = bc[wv][1];
    for (int q = lane; q < kDescLen; q += 64) dv[q] = sat_u8(dv[q] * nrm2s) * nrm2s;
    wave_sync_d();
    if (lane == 0) {
      float nrm1 = 0;
      for (int q = 0; q < kDescLen; ++q) nrm1 = nrm1 + dv[q];
      bc[wv][2] = 1.f / (nrm1 < FLT_EPSILON ? FLT_EPSILON : nrm1);
    }
    wave_sync_d();
    const float nrm1 = bc[wv][2];
    float* out = A.desc + (long long)k * kDescLen;
    for (int q = lane; q < kDescLen; q += 64) out[q] = sqrtf(dv[q] * nrm1);
    wave_sync_d();
  }
}

// Element-wise evaluation of the device helpers (sift_selftest_math).
__global__ __launch_bounds__(256) void math_selftest_kernel(int op, const float* __restrict__ a,
                                                            const float* __restrict__ b,
                                                            float* __restrict__ out, int n,
                                                            const MathConsts* __restrict__ mc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = a[i];
  float r = 0.f;
  switch (op) {
    case 0: r = exp32f(x, mc->exptab, mc->e); break;
    case 1: r = fast_atan2(x, b[i], mc->t); break;
    case 2: r = magnitude(x, b[i]); break;
    case 3: r = cosf_cr(x); break;
    case 4: r = sinf_cr(x); break;
    case 5: r = pow2f_cr(x); break;
    case 6: r = (float)cv_round(x); break;
    default: r = (float)cv_floor(x); break;
  }
  out[i] = r;
}

void launch_math_selftest(hipStream_t st, int op, const float* a, const float* b, float* out, int n,
                          const MathConsts* mc) {
  hipLaunchKernelGGL(math_selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, st, op, a, b, out, n,
                     mc);
}

void launch_descriptors(hipStream_t st, const Layout& L, const float* gpyr, const MathConsts* mc,
                        const sift_keypoint* kpts, const int* img_kp_off, int batch, int kp_cap,
                        float* desc, int first_octave, int* err_flag) {
  DescArgs A;
  A.L = L;
  A.gpyr = gpyr;
  A.mc = mc;
  A.kpts = kpts;
  A.img_kp_off = img_kp_off;
  A.batch = batch;
  A.kp_cap = kp_cap;
  A.desc = desc;
  A.first_octave = first_octave;
  A.err_flag = err_flag;
  hipLaunchKernelGGL(descriptor_kernel, dim3(2048), dim3(256), 0, st, A);
}

}  // namespace sift
