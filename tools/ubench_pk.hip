// ubench_pk.hip -- issue rate of packed f32 VALU (v_pk_add_f32 / v_pk_mul_f32)
// against the scalar forms (v_add_f32 / v_mul_f32) on gfx950: if a packed
// instruction issues at the scalar one's rate, the exact blur's independent
// mul + add chains (blur.hip, blur_sym_kernel) could pair two output columns
// per lane.  Every instruction is independent of the previous 15, so the
// numbers are issue throughput, not latency.  Result (profiles/r5_ubench_pk.txt,
// r5_blur_pk_ab.txt): a packed instruction costs ~1.8-2x a scalar one, so the
// packed blur (tools/patches/blur_sym_pk.patch) ran slower, not faster.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_pk.hip -o tools/ubench_pk && ./tools/ubench_pk
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kIters = 4096;

#define ADD1(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
#define PKADD(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[i]) : "v"(y));
#define MUL1(i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
#define PKMUL(i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(y));
#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

// mode 0: 16 v_add_f32 per iteration; 1: 16 v_pk_add_f32 (32 adds);
// 2: 16 v_mul_f32; 3: 16 v_pk_mul_f32; 4: 8 mul + 16 add (the blur's mix);
// 5: 4 v_pk_mul_f32 + 8 v_pk_add_f32 (the same mix, packed, twice the work);
// 6: the w = 18 scatter blur's column step, scalar: 19 v_mul_f32 (literal
// coefficients) into distinct registers, then 37 v_add_f32 into 37 accumulators;
// 7: the same step on two output columns per lane: 19 v_pk_mul_f32 (SGPR
// coefficient broadcast by op_sel_hi) and 37 v_pk_add_f32
template <int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k(float* out, float xv) {
  float a[16];
  f2 p[16];
  for (int i = 0; i < 16; ++i) {
    a[i] = threadIdx.x + i;
    p[i] = f2{(float)threadIdx.x, (float)i};
  }
  const float x = xv;
  unsigned long long kc[19];
  for (int i = 0; i < 19; ++i) kc[i] = __builtin_amdgcn_readfirstlane((int)(xv * 1000) + i);
  const f2 y = f2{xv, xv};
  for (int it = 0; it < kIters; ++it) {
    if constexpr (MODE == 0) { R16(ADD1) }
    if constexpr (MODE == 1) { R16(PKADD) }
    if constexpr (MODE == 2) { R16(MUL1) }
    if constexpr (MODE == 3) { R16(PKMUL) }
    if constexpr (MODE == 4) {
      MUL1(0) ADD1(1) ADD1(2) MUL1(3) ADD1(4) ADD1(5) MUL1(6) ADD1(7) ADD1(8) MUL1(9) ADD1(10) ADD1(11)
      MUL1(12) ADD1(13) ADD1(14) MUL1(15) ADD1(0) ADD1(1) MUL1(2) ADD1(3) ADD1(4) MUL1(5) ADD1(6) ADD1(7)
    }
    if constexpr (MODE == 6) {
      float pr[19], acc[37];
      for (int i = 0; i < 37; ++i) acc[i] = a[i & 15];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int i = 0; i < 19; ++i)
          asm volatile("v_mul_f32 %0, 0x3f81a2b3, %1" : "=v"(pr[i]) : "v"(a[c]));
#pragma unroll
        for (int i = 0; i < 37; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(pr[i < 19 ? i : 37 - 1 - i]));
      }
      for (int i = 0; i < 16; ++i) a[i] = acc[i] + acc[i + 16];
    }
    if constexpr (MODE == 7) {
      f2 pr[19], acc[37];
      for (int i = 0; i < 37; ++i) acc[i] = p[i & 15];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int i = 0; i < 19; ++i)
          asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(pr[i]) : "v"(p[c]), "s"(kc[i]));
#pragma unroll
        for (int i = 0; i < 37; ++i)
          asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(pr[i < 19 ? i : 37 - 1 - i]));
      }
      for (int i = 0; i < 16; ++i) p[i] = acc[i] + acc[i + 16];
    }
    if constexpr (MODE == 8 || MODE == 9) {
      f2 pr[19], acc[37];
      for (int i = 0; i < 37; ++i) acc[i] = p[i & 15];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        unsigned long long kk[19];
#pragma unroll
        for (int i = 0; i < 19; ++i) {
          if constexpr (MODE == 8) asm volatile("s_mov_b64 %0, 0x3f81a2b3" : "=s"(kk[i]));
          else asm volatile("s_mov_b32 %0, 0x3f81a2b3" : "=s"(kk[i]));
        }
#pragma unroll
        for (int i = 0; i < 19; ++i)
          asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(pr[i]) : "v"(p[c]), "s"(kk[i]));
#pragma unroll
        for (int i = 0; i < 37; ++i)
          asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(pr[i < 19 ? i : 37 - 1 - i]));
      }
      for (int i = 0; i < 16; ++i) p[i] = acc[i] + acc[i + 16];
    }
    if constexpr (MODE == 5) {
      PKMUL(0) PKADD(1) PKADD(2) PKMUL(3) PKADD(4) PKADD(5) PKMUL(6) PKADD(7) PKADD(8) PKMUL(9) PKADD(10)
      PKADD(11)
    }
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += a[i] + p[i].x + p[i].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, double ops_per_iter, int waves_per_simd, float* d) {
  const int blocks = 256 * 4 * waves_per_simd;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, d, 1.0001f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, d, 1.0001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double lane_ops = (double)blocks * 64 * kIters * ops_per_iter;
  printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"lane_ops_per_s_T\": %.3f}\n", name,
         waves_per_simd, ms, lane_ops / (ms * 1e-3) / 1e12);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 4 * 8 * 64 * sizeof(float));
  for (int w : {3}) {
    run<0>("v_add_f32 x16", 16, w, d);
    run<1>("v_pk_add_f32 x16 (32 adds)", 32, w, d);
    run<2>("v_mul_f32 x16", 16, w, d);
    run<3>("v_pk_mul_f32 x16 (32 muls)", 32, w, d);
    run<4>("8 mul + 16 add", 24, w, d);
    run<5>("4 pk_mul + 8 pk_add (24 ops)", 24, w, d);
    run<6>("blur w18 column step x4, scalar (19 mul + 37 add)", 4 * 56, w, d);
    run<7>("blur w18 column step x4, packed (2 columns: 112 ops)", 4 * 112, w, d);
    run<8>("blur w18 column step x4, packed + 19 s_mov_b64 per step", 4 * 112, w, d);
  }
  hipFree(d);
  return 0;
}
