// ubench_fma.hip -- issue rate of scalar vs packed f32 VALU ops (v_fma_f32,
// v_pk_fma_f32, v_add_f32, v_pk_add_f32) at 1, 2, 4 and 8 waves per SIMD, on
// independent chains (8 per lane).  Standalone, prints one JSON line per case:
//   hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 tools/ubench_fma.hip -o /tmp/ubf && /tmp/ubf
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

// OP: 0 v_fma_f32, 1 v_pk_fma_f32, 2 v_add_f32, 3 v_pk_add_f32.  Every case
// does 16 lane-ops per inner step (16 scalar or 8 packed instructions).
// VG: the addend / multiplier in a VGPR (k + s * 0, not foldable under IEEE
// rules) instead of the kernel-argument SGPR.
template <int OP, bool VG>
__global__ __launch_bounds__(256) void op_kernel(float* out, int iters, float k0) {
  extern __shared__ float pad[];
  if (iters < 0) pad[threadIdx.x] = 0.f;  // keeps the LDS allocation (occupancy control)
  const float s = threadIdx.x * 1e-3f;
  const float k = VG ? k0 + s * 0.f : k0;
  float r = 0.f;
  if (OP == 1 || OP == 3) {
    f2 a[8];
    const f2 kk = {k, k}, c = {1e-3f, 2e-3f};
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = f2{s + j, s - j};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = OP == 1 ? __builtin_elementwise_fma(a[j], kk, c) : a[j] + kk;
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
        for (int j = 0; j < 16; ++j) a[j] = OP == 0 ? __builtin_fmaf(a[j], k, 1e-3f) : a[j] + k;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) r += a[j];
  }
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP, bool VG>
void run(const char* name, int ncu, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int lds = (160 * 1024) / wps - 2048;  // wps workgroups (of 4 waves) per CU
    const int grid = ncu * wps;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL((op_kernel<OP, VG>), dim3(grid), dim3(256), lds, 0, out, iters, 0.999f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double lane_ops = (double)grid * 256 * iters * 8 * 16;
      const double instr_per_simd = lane_ops / 64 / (OP == 1 || OP == 3 ? 2 : 1) / (ncu * 4);
      if (rep)
        printf("{\"op\": \"%s\", \"operand\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"Tlane_ops\": %.1f, "
               "\"ns_per_instr_per_simd\": %.3f}\n",
               name, VG ? "vgpr" : "sgpr", wps, ms, lane_ops / ms / 1e9, ms * 1e6 / instr_per_simd);
    }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
  float* out = nullptr;
  if (hipMalloc(&out, 256 * 8 * 4096 * sizeof(float)) != hipSuccess) return 1;
  run<0, false>("v_fma_f32", ncu, out);
  run<1, false>("v_pk_fma_f32", ncu, out);
  run<2, false>("v_add_f32", ncu, out);
  run<3, false>("v_pk_add_f32", ncu, out);
  run<2, true>("v_add_f32", ncu, out);
  run<3, true>("v_pk_add_f32", ncu, out);
  (void)hipFree(out);
  return 0;
}
