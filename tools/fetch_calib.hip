// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950
// for the access widths this library's kernels use (MI355X_MICROARCH.md:
// only 16-B/lane streaming reads are calibrated there -- FETCH_SIZE reports
// half their bytes; "other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").
//
// Each kernel moves a known number of bytes through a 1 GiB buffer (4x the
// 256 MiB Infinity Cache, so nothing is re-served on die):
//   rd4 / rd8 / rd16 : coalesced streaming reads, 4 / 8 / 16 B per lane
//   wr4 / wr8 / wr16 : coalesced streaming writes
//   gather8          : 8-B reads at random addresses (one per lane)
// Run under `rocprofv3 --kernel-trace --pmc FETCH_SIZE` and again with
// WRITE_SIZE; tools/rocprof_summary.py divides the counters by the bytes this
// program prints.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

template <typename T>
__device__ __forceinline__ float fold(T v);
template <> __device__ __forceinline__ float fold<float>(float v) { return v; }
template <> __device__ __forceinline__ float fold<float2>(float2 v) { return v.x + v.y; }
template <> __device__ __forceinline__ float fold<float4>(float4 v) { return v.x + v.y + v.z + v.w; }

template <typename T>
__global__ __launch_bounds__(256) void rd(const T* __restrict__ p, long long n, float* __restrict__ sink) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) s += fold(p[i]);
  if (s == 12345.678f) sink[0] = s;  // keeps the loads; never true for zero-filled data
}

template <typename T>
__global__ __launch_bounds__(256) void wr(T* __restrict__ p, long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = T{};
}

__global__ __launch_bounds__(256) void gather8(const float2* __restrict__ p, long long n, long long count,
                                               float* __restrict__ sink) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < count; i += (long long)gridDim.x * 256) {
    unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    s += fold(p[h % (unsigned long long)n]);
  }
  if (s == 12345.678f) sink[0] = s;
}

int main() {
  const long long bytes = 1ll << 30;
  char* buf = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 16;
  hipLaunchKernelGGL(rd<float>, dim3(grid), dim3(256), 0, 0, (const float*)buf, bytes / 4, sink);
  hipLaunchKernelGGL(rd<float2>, dim3(grid), dim3(256), 0, 0, (const float2*)buf, bytes / 8, sink);
  hipLaunchKernelGGL(rd<float4>, dim3(grid), dim3(256), 0, 0, (const float4*)buf, bytes / 16, sink);
  hipLaunchKernelGGL(wr<float>, dim3(grid), dim3(256), 0, 0, (float*)buf, bytes / 4);
  hipLaunchKernelGGL(wr<float2>, dim3(grid), dim3(256), 0, 0, (float2*)buf, bytes / 8);
  hipLaunchKernelGGL(wr<float4>, dim3(grid), dim3(256), 0, 0, (float4*)buf, bytes / 16);
  const long long gcount = 1ll << 24;  // 16 M random 8-B reads = 128 MiB requested
  hipLaunchKernelGGL(gather8, dim3(grid), dim3(256), 0, 0, (const float2*)buf, bytes / 8, gcount, sink);
  CK(hipDeviceSynchronize());
  printf("{\"rd_bytes\": %lld, \"wr_bytes\": %lld, \"gather8_requested_bytes\": %lld}\n", bytes, bytes,
         gcount * 8);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
