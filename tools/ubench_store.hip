// ubench_store.hip -- HBM write rate of the pyramid's store patterns on
// MI355X: 64 images x 5 planes of 1080 x 1920 floats (3.98 GB), written as
//   0 linear: consecutive 256-B wave stores over the whole buffer (grid-stride)
//   1 strips: a workgroup = one wave over a 64-column strip of one image,
//     walking its 1080 rows; per row one dword store per plane (the
//     pyramid kernels' pattern), `rows_per_step` rows between waits
//   2 strips x4: the same with 4 waves side by side (a 256-column strip)
//   3 wide: one wave over a 256-column strip, dwordx4 stores (4 columns / lane)
// One JSON line per mode: ms, TB/s.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_store.hip -o /tmp/ubs && /tmp/ubs
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int B = 64, R = 1080, C = 1920, NP = 5;
constexpr long long PLANE = (long long)R * C, IMG = PLANE * NP;

__global__ __launch_bounds__(256) void linear_kernel(float* __restrict__ p, long long n4) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) p[i] = (float)(i & 1023);
}

// MODE 1: 64-thread blocks; MODE 2: 256-thread blocks (4 waves side by side)
template <int W>
__global__ __launch_bounds__(W * 64) void strip_kernel(float* __restrict__ p, int strips) {
  const int item = blockIdx.x;
  const int b = item / strips, s = item % strips;
  const int x = s * (64 * W) + threadIdx.x;
  float* img = p + b * IMG;
  float v = (float)threadIdx.x;
  for (int y = 0; y < R; ++y) {
#pragma unroll
    for (int q = 0; q < NP; ++q) img[q * PLANE + (long long)y * C + x] = v + q;
    v += 1.f;
  }
}

__global__ __launch_bounds__(64) void wide_kernel(float* __restrict__ p, int strips) {
  const int item = blockIdx.x;
  const int b = item / strips, s = item % strips;
  const int x = s * 256 + threadIdx.x * 4;
  float* img = p + b * IMG;
  float v = (float)threadIdx.x;
  for (int y = 0; y < R; ++y) {
#pragma unroll
    for (int q = 0; q < NP; ++q)
      *reinterpret_cast<float4*>(img + q * PLANE + (long long)y * C + x) = make_float4(v, v + 1, v + 2, v + q);
    v += 1.f;
  }
}

int main() {
  float* p;
  const size_t bytes = (size_t)B * IMG * 4;
  if (hipMalloc(&p, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 4; ++mode) {
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      if (mode == 0)
        hipLaunchKernelGGL(linear_kernel, dim3(256 * 32), dim3(256), 0, 0, p, (long long)(bytes / 4));
      else if (mode == 1)
        hipLaunchKernelGGL(strip_kernel<1>, dim3(B * (C / 64)), dim3(64), 0, 0, p, C / 64);
      else if (mode == 2)
        hipLaunchKernelGGL(strip_kernel<4>, dim3(B * (C / 256)), dim3(256), 0, 0, p, C / 256);
      else
        hipLaunchKernelGGL(wide_kernel, dim3(B * (C / 256)), dim3(64), 0, 0, p, C / 256);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const char* names[4] = {"linear", "strip64_dword", "strip256_4waves_dword", "strip256_1wave_dwordx4"};
    printf("{\"mode\": \"%s\", \"ms\": %.3f, \"TBs\": %.3f}\n", names[mode], best, bytes / (best * 1e-3) / 1e12);
  }
  hipFree(p);
  return 0;
}
