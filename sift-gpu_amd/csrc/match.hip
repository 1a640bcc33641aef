// match.hip -- brute-force L1 k-nearest-neighbour matching (k <= 2) for gfx950.
//
// The consumer of the descriptors in the reference application:
// `BFMatcher(NORM_L1).knnMatch(descriptors1, descriptors0, matches, 2)` and
// the 0.86 ratio test (src/main.cpp:25-40).  SURVEY.md §8(f) row f2.
//
// Distance: OpenCV's float L1 (normL1_, the x86 SSE3 baseline form): eight
// partial sums p[k] = sum_g |a[8g+k] - b[8g+k]| in g order (two 4-lane
// accumulators over 8-element steps), then q = p[0:4] + p[4:8] and the
// horizontal-add reduction (q0 + q1) + (q2 + q3).  oracle/match.py restates the
// same order; real OpenCV may dispatch a wider SIMD form (different float
// rounding), so parity against OpenCV itself is unpinned.
//
// Order: for each query the two smallest (distance, train index) pairs in
// lexicographic order -- OpenCV's batchDistance insertion keeps an earlier
// train index ahead of a later one at equal distance (strict '<').
//
// Layout: a workgroup owns 64 queries (one per lane, descriptor in VGPRs) and
// one split of the train rows; 64-row train chunks are staged in LDS and each
// of the 4 waves scores every fourth row of a chunk (broadcast ds_read_b128:
// all lanes read the same row).  Bound: VALU -- 2 instructions per element
// pair (v_sub, v_add with |x|), 256 per (query, train) pair; the LDS reads are
// 512 B per row per wave.  The 4 waves' top-2 lists merge in LDS; splits merge
// in knn_merge_kernel.
#include "common.hpp"

#include <float.h>

namespace sift {

namespace {

constexpr int kQT = 64;  // queries per workgroup
constexpr int kTC = 64;  // train rows per LDS chunk
constexpr int kV4 = kDescLen / 4;

struct Best2 {
  float d1, d2;
  int i1, i2;
};

// (d, i) < (e, j) lexicographically; i = -1 (empty slot) sorts last via d = +inf.
__device__ __forceinline__ bool lex_lt(float d, int i, float e, int j) { return d < e || (d == e && i < j); }

__device__ __forceinline__ void insert(Best2& b, float d, int i) {
  if (lex_lt(d, i, b.d1, b.i1)) {
    b.d2 = b.d1;
    b.i2 = b.i1;
    b.d1 = d;
    b.i1 = i;
  } else if (lex_lt(d, i, b.d2, b.i2)) {
    b.d2 = d;
    b.i2 = i;
  }
}

__global__ __launch_bounds__(256) void knn_l1_kernel(const float* __restrict__ q, int nq, const float* __restrict__ t,
                                                     int nt, int per_split, float2* __restrict__ part_d,
                                                     int2* __restrict__ part_i) {
  __shared__ float4 tl[kTC * kV4];  // 32 KB
  __shared__ float md[4][2][kQT];
  __shared__ int mi[4][2][kQT];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int qi = blockIdx.x * kQT + lane;
  float4 qv[kV4];
  {
    const float4* qp = reinterpret_cast<const float4*>(q + (long long)min(qi, nq - 1) * kDescLen);
#pragma unroll
    for (int v = 0; v < kV4; ++v) qv[v] = qp[v];
  }
  Best2 best{INFINITY, INFINITY, -1, -1};
  const int t0 = blockIdx.y * per_split, t1 = min(nt, t0 + per_split);
  for (int c0 = t0; c0 < t1; c0 += kTC) {
    const int nrow = min(kTC, t1 - c0);
    __syncthreads();
    const float4* src = reinterpret_cast<const float4*>(t + (long long)c0 * kDescLen);
    for (int u = threadIdx.x; u < nrow * kV4; u += 256) tl[u] = src[u];
    __syncthreads();
    for (int r = wv; r < nrow; r += 4) {
      const float4* tr = tl + r * kV4;
      float p[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) p[k] = 0.f;
#pragma unroll
      for (int g = 0; g < kDescLen / 8; ++g) {
        const float4 a = tr[2 * g], b = tr[2 * g + 1];
        const float4 x = qv[2 * g], y = qv[2 * g + 1];
        p[0] = p[0] + fabsf(x.x - a.x);
        p[1] = p[1] + fabsf(x.y - a.y);
        p[2] = p[2] + fabsf(x.z - a.z);
        p[3] = p[3] + fabsf(x.w - a.w);
        p[4] = p[4] + fabsf(y.x - b.x);
        p[5] = p[5] + fabsf(y.y - b.y);
        p[6] = p[6] + fabsf(y.z - b.z);
        p[7] = p[7] + fabsf(y.w - b.w);
      }
      const float q0 = p[0] + p[4], q1 = p[1] + p[5], q2 = p[2] + p[6], q3 = p[3] + p[7];
      insert(best, (q0 + q1) + (q2 + q3), c0 + r);
    }
  }
  md[wv][0][lane] = best.d1;
  md[wv][1][lane] = best.d2;
  mi[wv][0][lane] = best.i1;
  mi[wv][1][lane] = best.i2;
  __syncthreads();
  if (wv == 0 && qi < nq) {
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      insert(best, md[w][0][lane], mi[w][0][lane]);
      insert(best, md[w][1][lane], mi[w][1][lane]);
    }
    const long long o = (long long)blockIdx.y * nq + qi;
    part_d[o] = make_float2(best.d1, best.d2);
    part_i[o] = make_int2(best.i1, best.i2);
  }
}

__global__ __launch_bounds__(256) void knn_merge_kernel(const float2* __restrict__ part_d,
                                                        const int2* __restrict__ part_i, int nq, int splits, int k,
                                                        int* __restrict__ idx, float* __restrict__ dist) {
  const int qi = blockIdx.x * 256 + threadIdx.x;
  if (qi >= nq) return;
  Best2 best{INFINITY, INFINITY, -1, -1};
  for (int s = 0; s < splits; ++s) {
    const float2 d = part_d[(long long)s * nq + qi];
    const int2 i = part_i[(long long)s * nq + qi];
    insert(best, d.x, i.x);
    insert(best, d.y, i.y);
  }
  idx[(long long)qi * k] = best.i1;
  dist[(long long)qi * k] = best.d1;
  if (k == 2) {
    idx[(long long)qi * k + 1] = best.i2;
    dist[(long long)qi * k + 1] = best.d2;
  }
}

}  // namespace

int knn_splits(int nq, int nt) {
  const int gx = (nq + kQT - 1) / kQT;
  int s = (2048 + gx - 1) / gx;                  // ~2k workgroups to fill 256 CUs
  const int max_s = (nt + kTC - 1) / kTC;         // at least one chunk per split
  s = s < max_s ? s : max_s;
  return s < 1 ? 1 : s;
}

void launch_knn_l1(hipStream_t st, const float* q, int nq, const float* t, int nt, int k, int splits,
                   float2* part_d, int2* part_i, int* idx, float* dist) {
  if (nq <= 0) return;
  const int per = ((nt + splits - 1) / splits + kTC - 1) / kTC * kTC;
  dim3 grid((nq + kQT - 1) / kQT, splits);
  hipLaunchKernelGGL(knn_l1_kernel, grid, dim3(256), 0, st, q, nq, t, nt, per, part_d, part_i);
  hipLaunchKernelGGL(knn_merge_kernel, dim3((nq + 255) / 256), dim3(256), 0, st, part_d, part_i, nq, splits, k,
                     idx, dist);
}

}  // namespace sift
