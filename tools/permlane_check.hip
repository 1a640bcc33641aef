// permlane_check.hip -- checks the 4 x 4 register transpose across the four
// 16-lane rows of a wave built from v_permlane32_swap_b32 + v_permlane16_swap_b32
// (gfx950), as pyramid_pc.hip uses it: lane (R = lane >> 4, i = lane & 15)
// holding a[u] = X[R][u] ends with b[k] = X[k][R].
//   hipcc -O3 --offload-arch=gfx950 tools/permlane_check.hip -o tools/permlane_check && ./tools/permlane_check
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ void xpose4(float (&a)[4]) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[0]), __float_as_uint(a[2]), false, false);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[1]), __float_as_uint(a[3]), false, false);
  auto r = __builtin_amdgcn_permlane16_swap(p[0], q[0], false, false);
  auto s = __builtin_amdgcn_permlane16_swap(p[1], q[1], false, false);
  a[0] = __uint_as_float(r[0]);
  a[1] = __uint_as_float(r[1]);
  a[2] = __uint_as_float(s[0]);
  a[3] = __uint_as_float(s[1]);
}

__global__ void k(float* out) {
  const int lane = threadIdx.x, R = lane >> 4, i = lane & 15;
  float a[4];
  for (int u = 0; u < 4; ++u) a[u] = (float)(R * 1000 + i * 10 + u);  // X[R][u] of column group i
  xpose4(a);
  for (int k = 0; k < 4; ++k) out[lane * 4 + k] = a[k];
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int lane = 0; lane < 64; ++lane) {
    const int R = lane >> 4, i = lane & 15;
    for (int k = 0; k < 4; ++k) {
      const float want = (float)(k * 1000 + i * 10 + R);  // X[k][R]
      if (h[lane * 4 + k] != want) {
        if (bad < 8) printf("lane %d k %d: %g want %g\n", lane, k, h[lane * 4 + k], want);
        ++bad;
      }
    }
  }
  printf("permlane xpose4: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
  hipFree(d);
  return bad ? 1 : 0;
}
