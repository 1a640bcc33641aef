// ubench_pyrmem.hip -- the separable pyramid's memory stream alone (no
// arithmetic, no synchronisation between waves) on MI355X, to separate the
// memory structure's own rate from the kernel's compute (round 5).
//
// 64 images x 1080 x 1920; a 256-thread workgroup per 64-column strip walks
// the rows 8 per step like pyramid_pc.hip: wave 0 loads the step's source rows
// (columns [x0 - 24, x0 + 88)) into an LDS ring and stores plane 0; waves 1-3
// store plane 4, plane 3, planes 2 + 1 + the decimated next plane 0 as
// dwordx4 stores of 4 rows x 64 columns.  25 B per pixel (4 read, 21 written).
// Modes (one JSON line each):
//   0 stores only
//   1 stores + source rows by LDS-DMA buffer_load_dword (16 per step, the kernel's form)
//   2 stores + source rows by global_load_lds_dwordx4 (4 per step)
//   3 stores + source rows by global_load_dwordx4 into VGPRs + ds_write_b128
//   4 source rows only (LDS-DMA dword)
//   5 stores with 4 waves storing per workgroup, no loads (the pure-store ceiling)
//   6 = 1 in XCD-contiguous block order (blocks b, b + 8, ... take neighbouring strips)
//   7 = 1 with the source rows 64 columns wide (no halo)
//   8 = 7 in XCD-contiguous order
//   9 = 6 with one stored plane (a copy's 1:1 read:write mix)
//  10 = 6 with 128-column strips per workgroup (source rows 176 columns)
//  11 = 6 with 256-column strips per workgroup (source rows 304 columns)
//  12 the same bytes as linear streams: the source read and the five planes
//     (+ the quarter-size next plane 0) written front to back, grid-stride
//     dwordx4 -- the pattern-independent ceiling for this traffic
//  13 calibration: a linear float4 copy (1 read : 1 write)
//  14 calibration: the six linear write streams of 12 without the read
//  15 = 12 with non-temporal stores
//  16 = 6 with four neighbouring 64-column strips per 1024-thread workgroup
//     (four independent groups of four waves, one CU)
//  17 = 6 with STRIP-MAJOR destination planes (round 6, VERDICT r5 #2a): each
//     64-column strip's rows stored contiguously (x -> strip (x >> 6), y,
//     x & 63; the next plane 0 likewise in its own 64-column strips), so every
//     wave's stores form one linear stream; source = the row-major image
//  18 = 17 with a strip-major source too (octaves > 0 read plane 0 of the
//     octave, which would then be strip-major: three contiguous pieces per row)
//  19 ROW BANDS (VERDICT r5 #2b): a workgroup owns a band of 40 rows of one
//     image and walks them 8 per step, all 30 strips per step (inner loop),
//     row-major destination: each step writes 8 full rows of every plane
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_pyrmem.hip -o tools/ubench_pyrmem && ./tools/ubench_pyrmem
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int B = 64, R = 1080, C = 1920, STRIPS = C / 64;
constexpr long long PLANE = (long long)R * C;
constexpr int ROWW = 112;  // source row segment (floats)

typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc mk(const float* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, 0x00020000);
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef float fv4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(MODE == 16 ? 1024 : 256) void pyrmem_kernel(const float* __restrict__ src, float* __restrict__ planes,
                                                      float* __restrict__ nxt) {
  constexpr int SW = MODE == 10 ? 128 : MODE == 11 ? 256 : 64;  // strip width
  constexpr int NSUB = SW / 64, SROW = SW + 48, NDMA = (SROW + 63) / 64;
  constexpr int STR = C / SW;
  __shared__ __attribute__((aligned(16))) float ring4[MODE == 16 ? 4 : 1][2][8][NDMA * 64];
  constexpr bool kXcd = MODE == 6 || MODE == 8 || MODE == 9 || MODE >= 10;
  constexpr bool kSM = MODE == 17 || MODE == 18;  // strip-major destination
  constexpr int kBand = 40;                       // mode 19: rows per workgroup
  const int nb = (int)gridDim.x;
  int item = kXcd ? (int)(blockIdx.x & 7) * (nb >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int grp = MODE == 16 ? (int)(threadIdx.x >> 8) : 0;
  if (MODE == 16) item = __builtin_amdgcn_readfirstlane(item * 4 + grp);
  float(&ring)[2][8][NDMA * 64] = ring4[grp];
  const int b = MODE == 19 ? item / (R / kBand) : item / STR;
  const int band0 = MODE == 19 ? (item % (R / kBand)) * kBand : 0;
  const int wv = (threadIdx.x >> 6) & 3, lane = threadIdx.x & 63;
  const float* simg = src + b * PLANE;
  const Rsrc rs = mk(simg, PLANE * 4);
  float* img = planes + (long long)b * 5 * PLANE;
  const int sr = lane >> 4;
  float4 v = make_float4(lane, 1.f, 2.f, 3.f);
  constexpr int NSTEP = MODE == 19 ? kBand / 8 * STRIPS : R / 8;
  for (int s = 0; s < NSTEP; ++s) {
    const int x0 = MODE == 19 ? (s % STRIPS) * 64 : (item % STR) * SW;
    const int Ys = MODE == 19 ? band0 + 8 * (s / STRIPS) : 8 * s;
    const int xg = x0 + 4 * (lane & 15);
    if (wv == 0 && MODE >= 1 && MODE != 5) {
      float* slot = &ring[s & 1][0][0];
      constexpr bool kHalo = !(MODE == 7 || MODE == 8);
      if constexpr (MODE == 1 || MODE == 4 || MODE >= 6) {
        for (int i = 0; i < 8; ++i) {
          const unsigned so = MODE == 18 ? 0u : (unsigned)((Ys + i) * C * 4);
          const unsigned l0 = __builtin_amdgcn_readfirstlane(
              (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(slot + i * NDMA * 64));
#pragma unroll
          for (int d = 0; d < (kHalo ? NDMA : NSUB); ++d) {
            const int c = x0 - (kHalo ? 24 : 0) + lane + 64 * d;
            // mode 18: the source plane is strip-major too
            const unsigned vo = !(c >= 0 && c < C - 1) ? 0x7f000000u
                                : MODE == 18 ? (unsigned)(((c >> 6) * R * 64 + (Ys + i) * 64 + (c & 63)) * 4)
                                             : c * 4u;
            if (!kHalo || 64 * d + lane < SROW)
              asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, %3 offen lds" ::"s"(l0 + 256 * d), "v"(vo),
                           "s"(rs), "s"(so) : "memory", "m0");
          }
        }
      } else if constexpr (MODE == 2) {
        // 8 rows x 28 chunks of 16 B = 224 chunks: 4 instructions, lane -> (row, chunk)
        for (int t = 0; t < 4; ++t) {
          const int ch = min(64 * t + lane, 8 * 28 - 1);
          const int i = ch / 28, k = ch - i * 28;
          const int c = max(x0 - 24 + 4 * k, 0);
          __builtin_amdgcn_global_load_lds((const void*)(simg + (long long)(Ys + i) * C + c),
                                           (__attribute__((address_space(3))) void*)(slot + 64 * 4 * t), 16, 0, 0);
        }
      } else if constexpr (MODE == 3) {
        float4 r[4];
        for (int t = 0; t < 4; ++t) {
          const int ch = min(64 * t + lane, 8 * 28 - 1);
          const int i = ch / 28, k = ch - i * 28;
          const int c = max(x0 - 24 + 4 * k, 0);
          r[t] = *reinterpret_cast<const float4*>(simg + (long long)(Ys + i) * C + c);
        }
        for (int t = 0; t < 4; ++t) *reinterpret_cast<float4*>(slot + 4 * (64 * t + lane)) = r[t];
      }
    }
    if (MODE == 4) continue;
    // stores: every storing wave writes its planes for rows [Ys, Ys + 8)
    const int nstore = MODE == 9 ? 1 : 4;
    if (wv < nstore) {
      const int pa = wv == 0 ? 0 : wv == 1 ? 4 : wv == 2 ? 3 : 2;
      for (int r4 = 0; r4 < 8 * NSUB; r4 += 4) {
        const int y = Ys + (r4 & 7) + sr;
        const int xw = xg + 64 * (r4 >> 3);
        const unsigned off = kSM ? (unsigned)((xw >> 6) * R * 64 + y * 64 + (xw & 63)) * 4u
                                 : (unsigned)(y * C + xw) * 4u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), mk(img + pa * PLANE, PLANE * 4),
                                               (int)off, 0, 0);
        if (wv == 3) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), mk(img + 1 * PLANE, PLANE * 4),
                                                 (int)off, 0, 0);
          const bool dn = (y & 1) == 0;
          const int xn = xw >> 1;  // next plane: R / 2 rows, C / 2 columns
          const unsigned offn = !dn ? 0x7f000000u
                                : kSM ? (unsigned)((xn >> 6) * (R / 2) * 64 + (y >> 1) * 64 + (xn & 63)) * 4u
                                      : (unsigned)((y >> 1) * (C / 2) + xn) * 4u;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, make_float2(v.x, v.z)),
                                                mk(nxt + b * (PLANE / 4), PLANE), (int)offn, 0, 0);
        }
      }
      v.x += 1.f;
    }
  }
}

template <int K>  // 0: mix, 1: copy, 2: writes only, 3: mix with nt stores
__global__ __launch_bounds__(256) void linear_mix_kernel(const float4* __restrict__ src, float4* __restrict__ planes,
                                                          float4* __restrict__ nxt, long long n4) {
  // one pass, 4 float4 per thread, all loads issued before the stores
  const long long base = ((long long)blockIdx.x * 256 * 4) + threadIdx.x;
  float4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = base + 256 * u;
    v[u] = K == 2 ? make_float4((float)i, 1.f, 2.f, 3.f) : (i < n4 ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f));
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = base + 256 * u;
    if (i >= n4) continue;
    if (K == 1) {
      planes[i] = v[u];
      continue;
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      if (K == 3)
        __builtin_nontemporal_store(__builtin_bit_cast(fv4, v[u]), reinterpret_cast<fv4*>(&planes[q * n4 + i]));
      else
        planes[q * n4 + i] = v[u];
    }
    if ((i & 3) == 0) nxt[i >> 2] = v[u];
  }
}

int main() {
  float *src, *planes, *nxt;
  if (hipMalloc(&src, (size_t)B * PLANE * 4) != hipSuccess || hipMalloc(&planes, (size_t)B * 5 * PLANE * 4) != hipSuccess ||
      hipMalloc(&nxt, (size_t)B * PLANE) != hipSuccess)
    return 1;
  (void)hipMemset(src, 0, (size_t)B * PLANE * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[20] = {"stores_only", "stores+dma_dword", "stores+dma_dwordx4", "stores+load_dwordx4+ds_write",
                           "dma_dword_only", "stores_4waves", "stores+dma_dword_xcd", "stores+dma_dword_nohalo",
                           "stores+dma_dword_nohalo_xcd", "1plane+dma_dword_xcd", "strip128+dma_xcd", "strip256+dma_xcd",
                           "linear_streams", "linear_copy", "linear_writes_only", "linear_streams_nt",
                           "4strips_per_wg+dma_xcd", "strip_major_dst+dma_xcd", "strip_major_dst+strip_major_src_xcd",
                           "row_bands40+dma_xcd"};
  for (int mode = 0; mode < 20; ++mode) {
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0);
      const dim3 g(B * (mode == 10 ? C / 128 : mode == 11 || mode == 16 ? C / 256 : mode == 19 ? R / 40 : STRIPS)),
          blk(mode == 16 ? 1024 : 256);
      switch (mode) {
        case 0: hipLaunchKernelGGL(pyrmem_kernel<0>, g, blk, 0, 0, src, planes, nxt); break;
        case 1: hipLaunchKernelGGL(pyrmem_kernel<1>, g, blk, 0, 0, src, planes, nxt); break;
        case 2: hipLaunchKernelGGL(pyrmem_kernel<2>, g, blk, 0, 0, src, planes, nxt); break;
        case 3: hipLaunchKernelGGL(pyrmem_kernel<3>, g, blk, 0, 0, src, planes, nxt); break;
        case 4: hipLaunchKernelGGL(pyrmem_kernel<4>, g, blk, 0, 0, src, planes, nxt); break;
        case 5: hipLaunchKernelGGL(pyrmem_kernel<5>, g, blk, 0, 0, src, planes, nxt); break;
        case 6: hipLaunchKernelGGL(pyrmem_kernel<6>, g, blk, 0, 0, src, planes, nxt); break;
        case 7: hipLaunchKernelGGL(pyrmem_kernel<7>, g, blk, 0, 0, src, planes, nxt); break;
        case 8: hipLaunchKernelGGL(pyrmem_kernel<8>, g, blk, 0, 0, src, planes, nxt); break;
        case 10: hipLaunchKernelGGL(pyrmem_kernel<10>, g, blk, 0, 0, src, planes, nxt); break;
        case 11: hipLaunchKernelGGL(pyrmem_kernel<11>, g, blk, 0, 0, src, planes, nxt); break;
        case 12:
          hipLaunchKernelGGL(linear_mix_kernel<0>, dim3((unsigned)((long long)B * PLANE / 4 / 1024)), blk, 0, 0, (const float4*)src, (float4*)planes,
                             (float4*)nxt, (long long)B * PLANE / 4);
          break;
        case 16: hipLaunchKernelGGL(pyrmem_kernel<16>, g, blk, 0, 0, src, planes, nxt); break;
        case 17: hipLaunchKernelGGL(pyrmem_kernel<17>, g, blk, 0, 0, src, planes, nxt); break;
        case 18: hipLaunchKernelGGL(pyrmem_kernel<18>, g, blk, 0, 0, src, planes, nxt); break;
        case 19: hipLaunchKernelGGL(pyrmem_kernel<19>, g, blk, 0, 0, src, planes, nxt); break;
        case 13:
          hipLaunchKernelGGL(linear_mix_kernel<1>, dim3((unsigned)((long long)B * PLANE / 4 / 1024)), blk, 0, 0, (const float4*)src, (float4*)planes,
                             (float4*)nxt, (long long)B * PLANE / 4);
          break;
        case 14:
          hipLaunchKernelGGL(linear_mix_kernel<2>, dim3((unsigned)((long long)B * PLANE / 4 / 1024)), blk, 0, 0, (const float4*)src, (float4*)planes,
                             (float4*)nxt, (long long)B * PLANE / 4);
          break;
        case 15:
          hipLaunchKernelGGL(linear_mix_kernel<3>, dim3((unsigned)((long long)B * PLANE / 4 / 1024)), blk, 0, 0, (const float4*)src, (float4*)planes,
                             (float4*)nxt, (long long)B * PLANE / 4);
          break;
        default: hipLaunchKernelGGL(pyrmem_kernel<9>, g, blk, 0, 0, src, planes, nxt); break;
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    // modes 11 and 16 cover C / 256 * 256 = 1,792 of the 1,920 columns: count the bytes they move
    const double px = (double)B * PLANE * (mode == 11 || mode == 16 ? (C / 256 * 256) / (double)C : 1.0);
    const double bytes = mode == 4 ? px * 4 * ROWW / 64 : mode == 0 || mode == 5 ? px * 21 : mode == 9 ? px * 8
                         : mode == 13 ? px * 8 : mode == 14 ? px * 21 : px * 25;
    printf("{\"mode\": \"%s\", \"ms\": %.3f, \"TBs_moved\": %.3f, \"TBs_at_24B_per_px\": %.3f}\n", names[mode], best,
           bytes / (best * 1e-3) / 1e12, px * 24 / (best * 1e-3) / 1e12);
  }
  return 0;
}
