// ubench_lit.hip -- issue rate of f32 FMA-class VALU ops by operand kind
// (32-bit literal, VGPR, inline constant, SGPR), 16 independent chains per
// lane, 1..8 waves per SIMD.  One JSON line per case:
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_lit.hip -o /tmp/ubl && /tmp/ubl
#include <hip/hip_runtime.h>
#include <stdio.h>

// OP: 0 v_fmac_f32 literal, 1 v_fmac_f32 VGPR multiplier, 2 v_fmac_f32 inline
// constant (0.5), 3 v_mul_f32 literal, 4 v_fmac_f32 SGPR multiplier, 5 v_add_f32 VGPR
template <int OP>
__global__ __launch_bounds__(256) void lit_kernel(float* out, int iters, float k0) {
  extern __shared__ float pad[];
  if (iters < 0) pad[threadIdx.x] = 0.f;
  const float s = threadIdx.x * 1e-3f;
  float a[16], kv = k0 + s * 0.f;
  asm volatile("" : "+v"(kv));
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = s + j;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (OP == 0) asm volatile("v_fmac_f32 %0, 0x3f7fbe77, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 15]));
        if (OP == 1) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[j]) : "v"(kv), "v"(a[(j + 1) & 15]));
        if (OP == 2) asm volatile("v_fmac_f32 %0, 0.5, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 15]));
        if (OP == 3) asm volatile("v_mul_f32 %0, 0x3f7fbe77, %0" : "+v"(a[j]));
        if (OP == 4) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[j]) : "s"(k0), "v"(a[(j + 1) & 15]));
        if (OP == 5) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[j]) : "v"(kv));
      }
  }
  float r = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) r += a[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
void run(const char* name, int ncu, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int lds = (160 * 1024) / wps - 2048;
    const int grid = ncu * wps;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL((lit_kernel<OP>), dim3(grid), dim3(256), lds, 0, out, iters, 0.999f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_simd = (double)grid * 4 * iters * 8 * 16 / (ncu * 4);
      if (rep)
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"ns_per_instr_per_simd\": %.3f}\n", name, wps,
               ms, ms * 1e6 / instr_per_simd);
    }
  }
}

int main() {
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
  float* out;
  hipMalloc(&out, (size_t)ncu * 8 * 256 * 4);
  run<0>("v_fmac_f32 literal", ncu, out);
  run<1>("v_fmac_f32 vgpr", ncu, out);
  run<2>("v_fmac_f32 inline-const", ncu, out);
  run<3>("v_mul_f32 literal", ncu, out);
  run<4>("v_fmac_f32 sgpr", ncu, out);
  run<5>("v_add_f32 vgpr", ncu, out);
  hipFree(out);
  return 0;
}
