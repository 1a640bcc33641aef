// simd_probe.hip -- which SIMD does wave w of a 256-thread workgroup land on?
// pyramid_pc.hip gives wave 0 the producer role and waves 1-3 the consumers;
// if the dispatcher always put wave w of every workgroup on SIMD w, the five
// resident workgroups of a CU would stack their five producers on one SIMD.
// Each wave records HW_REG_HW_ID (gfx9 layout: WAVE_ID [3:0], SIMD_ID [5:4],
// CU_ID [11:8], SH_ID [12], SE_ID [15:13]); the host tabulates wave index x
// SIMD id over a resident grid of 256-thread workgroups at 5 per CU.
//   hipcc -O3 --offload-arch=gfx950 tools/simd_probe.hip -o tools/simd_probe && ./tools/simd_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <vector>

__global__ __launch_bounds__(256) void probe(unsigned* out, int spin) {
  __shared__ char pad[32 * 1024];  // 5 workgroups per CU, as pyr_pc_kernel (32,272 B)
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  const int wv = threadIdx.x >> 6;
  // keep the wave resident a while so the whole grid is co-resident
  long long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  pad[threadIdx.x] = (char)hw;
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + wv] = hw + (pad[(threadIdx.x + 1) & 255] & 0);
}

int main() {
  const int nb = 256 * 5 * 2;
  unsigned* d;
  (void)hipMalloc(&d, nb * 4 * sizeof(unsigned));
  hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 0, 0, d, 200000);
  std::vector<unsigned> h(nb * 4);
  (void)hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
  int tab[4][4] = {};
  int same_simd_blocks = 0;
  for (int b = 0; b < nb; ++b) {
    int simds = 0;
    for (int w = 0; w < 4; ++w) {
      const int simd = (h[b * 4 + w] >> 4) & 3;
      ++tab[w][simd];
      simds |= 1 << simd;
    }
    if (simds != 15) ++same_simd_blocks;
  }
  printf("{\"blocks\": %d, \"wave_x_simd\": [", nb);
  for (int w = 0; w < 4; ++w)
    printf("[%d, %d, %d, %d]%s", tab[w][0], tab[w][1], tab[w][2], tab[w][3], w < 3 ? ", " : "");
  printf("], \"blocks_not_spread_over_4_simds\": %d}\n", same_simd_blocks);
  (void)hipFree(d);
  return 0;
}
