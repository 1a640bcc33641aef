// ubench_fma.hip -- issue rate of v_fma_f32 vs v_pk_fma_f32 at 1 and 2 waves
// per SIMD (the fast pyramid's FMA streams).  Standalone: hipcc -O3 -fno-slp-vectorize
// --offload-arch=gfx950 tools/ubench_fma.hip -o gpurun_out/ubench_fma
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ __launch_bounds__(256) void fma_kernel(float* out, int iters, float k) {
  extern __shared__ float pad[];
  if (iters < 0) pad[threadIdx.x] = 0.f;  // keeps the LDS allocation (occupancy control)
  const float s = threadIdx.x * 1e-3f;
  float r = 0.f;
  if (PK) {
    f2 a[8];
    const f2 kk = {k, k}, c = {1e-3f, 2e-3f};
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = f2{s + j, s - j};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = __builtin_elementwise_fma(a[j], kk, c);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r += a[j].x + a[j].y;
  } else {
    float a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = s + j;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = __builtin_fmaf(a[j], k, 1e-3f);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) r += a[j];
  }
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, 256 * 4096 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int pk = 0; pk < 2; ++pk) {
    for (int wps = 1; wps <= 2; ++wps) {
      const int lds = (160 * 1024) / wps - 8192;  // wps workgroups (of 4 waves) per CU
      const int grid = ncu * wps;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (pk)
          hipLaunchKernelGGL(fma_kernel<true>, dim3(grid), dim3(256), lds, 0, out, iters, 0.999f);
        else
          hipLaunchKernelGGL(fma_kernel<false>, dim3(grid), dim3(256), lds, 0, out, iters, 0.999f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double fmas = (double)grid * 256 * iters * 8 * 16;
        if (rep)
          printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n",
                 pk ? "v_pk_fma_f32" : "v_fma_f32", wps, ms, 2 * fmas / ms / 1e9);
      }
    }
  }
  hipFree(out);
  return 0;
}
