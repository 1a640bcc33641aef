// detect.hip -- extrema scan, sub-pixel refinement, orientation assignment
// (reference src/sift.cpp:285-577) for gfx950.
//
// Output order must equal the reference's: octave -> layer -> row -> col ->
// histogram peak (src/sift.cpp:556-557, 487-491, 525), duplicates kept.  The
// GPU therefore never appends with atomics:
//   extrema_count  -- one 256-lane workgroup per 2048 consecutive scan
//                     positions of one image (positions enumerated in the
//                     reference order), writes its candidate count;
//   scan           -- exclusive scan of those counts (ordered offsets);
//   extrema_write  -- recomputes the 26-neighbour test and writes candidates
//                     at ballot-ranked positions: the list comes out sorted;
//   refine_orient  -- one wave per candidate: adjustLocalExtrema redundantly
//                     on every lane (uniform control, broadcast loads), then
//                     the 36-bin orientation histogram with per-sample work
//                     spread over the lanes and an owner-computes
//                     accumulation (lane j sums bin j over the samples in
//                     raster order, so every float sum has the reference's
//                     order), smoothing, peak picking via ballot;
//   scan + emit    -- ordered keypoint slots from the per-candidate peak
//                     counts.
#include "common.hpp"

#include <float.h>
#include <limits.h>

namespace sift {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- scan segments: (octave, layer) interiors in reference order ----------
constexpr int kChunk = 2048;  // scan positions per workgroup
constexpr int kMaxSeg = 2 * kMaxOctaves;

struct SegTable {
  int n;
  int bpi;                        // workgroups per image
  long long total;                // scan positions per image
  long long start[kMaxSeg + 1];   // first position of each segment
  int o[kMaxSeg], layer[kMaxSeg], w[kMaxSeg];
  long long d_off[kMaxSeg];       // DoG plane offset of the segment's layer
  long long plane[kMaxSeg];       // elements between consecutive DoG planes
  int pitch[kMaxSeg];
  long long d_img;
};

static SegTable make_segs(const Layout& L) {
  SegTable S{};
  long long t = 0;
  int n = 0;
  for (int o = 0; o < L.n_oct; ++o)
    for (int layer = 1; layer <= kLayers; ++layer) {
      const Octave& O = L.oct[o];
      const int hr = O.rows - 2 * kBorder, wc = O.cols - 2 * kBorder;
      S.start[n] = t;
      S.o[n] = o;
      S.layer[n] = layer;
      S.w[n] = wc > 0 ? wc : 0;
      S.d_off[n] = O.d_off[layer];
      S.plane[n] = (long long)O.rows * O.pitch;
      S.pitch[n] = O.pitch;
      if (hr > 0 && wc > 0) t += (long long)hr * wc;
      ++n;
    }
  S.start[n] = t;
  S.n = n;
  S.total = t;
  S.bpi = (int)((t + kChunk - 1) / kChunk);
  if (S.bpi == 0) S.bpi = 1;
  S.d_img = L.d_img;
  return S;
}

int extrema_blocks_per_image(const Layout& L) { return make_segs(L).bpi; }

// Test of src/sift.cpp:493-511 at scan position g of image b.
__device__ __forceinline__ bool extremum_at(const SegTable& S, const float* __restrict__ dog, int b,
                                            long long g, int* seg_out, int* r_out, int* c_out) {
  int s = 0;
  while (s + 1 < S.n && S.start[s + 1] <= g) ++s;
  const long long loc = g - S.start[s];
  const int w = S.w[s];
  const int r = kBorder + (int)(loc / w), c = kBorder + (int)(loc % w);
  *seg_out = s;
  *r_out = r;
  *c_out = c;
  const long long pitch = S.pitch[s];
  const float* cur = dog + b * S.d_img + S.d_off[s] + r * pitch + c;
  const float v = cur[0];
  if (!(fabsf(v) > kDogThreshold)) return false;
  const float* prv = cur - S.plane[s];
  const float* nxt = cur + S.plane[s];
  bool ok = true;
  if (v > 0) {
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const long long q = dy * pitch + dx;
        ok = ok && v >= prv[q] && v >= nxt[q];
        if (dy != 0 || dx != 0) ok = ok && v >= cur[q];
      }
  } else if (v < 0) {
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const long long q = dy * pitch + dx;
        ok = ok && v <= prv[q] && v <= nxt[q];
        if (dy != 0 || dx != 0) ok = ok && v <= cur[q];
      }
  } else {
    ok = false;
  }
  return ok;
}

__global__ __launch_bounds__(256) void extrema_count_kernel(SegTable S, const float* __restrict__ dog,
                                                            int* __restrict__ blk_counts) {
  __shared__ int wsum[4];
  const int b = blockIdx.y;
  const long long base = (long long)blockIdx.x * kChunk;
  int cnt = 0;
  for (int it = 0; it < kChunk / 256; ++it) {
    const long long g = base + it * 256 + threadIdx.x;
    int sg, r, c;
    if (g < S.total && extremum_at(S, dog, b, g, &sg, &r, &c)) ++cnt;
  }
  // wave reduce then block reduce (integer: order-free)
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) blk_counts[b * S.bpi + blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void extrema_write_kernel(SegTable S, const float* __restrict__ dog,
                                                            const int* __restrict__ blk_off,
                                                            Cand* __restrict__ cands, int cap) {
  __shared__ int wcnt[4];
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long base = (long long)blockIdx.x * kChunk;
  int run = blk_off[b * S.bpi + blockIdx.x];
  for (int it = 0; it < kChunk / 256; ++it) {
    const long long g = base + it * 256 + threadIdx.x;
    int sg = 0, r = 0, c = 0;
    const bool f = g < S.total && extremum_at(S, dog, b, g, &sg, &r, &c);
    const unsigned long long m = __ballot(f);
    if (lane == 0) wcnt[wv] = __popcll(m);
    __syncthreads();
    int before = 0;
    for (int k = 0; k < wv; ++k) before += wcnt[k];
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (f) {
      const unsigned long long lt = (lane == 0) ? 0ull : (m & (~0ull >> (64 - lane)));
      const int pos = run + before + __popcll(lt);
      if (pos < cap) cands[pos] = Cand{b, S.o[sg] | (S.layer[sg] << 8), r, c};
    }
    run += tot;
    __syncthreads();
  }
}

// ---- single-workgroup exclusive scan -----------------------------------------
// out[i] = sum(in[0..i)), out[n] = total.  n from n_dev (clamped to cap) if
// given, else n_host.  Optional: img_out[b] = out[img_idx[b]] / out[b*stride].
__global__ __launch_bounds__(1024) void scan_kernel(const int* __restrict__ in, int in_stride,
                                                    int* __restrict__ out, const int* n_dev,
                                                    int n_host, int cap, int* total_out) {
  __shared__ int wsum[16];
  __shared__ int carry_s;
  int n = n_dev ? *n_dev : n_host;
  if (n > cap) n = cap;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 4096) {
    int v[4];
    int s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = base + tid * 4 + k;
      v[k] = i < n ? in[(long long)i * in_stride] : 0;
      s += v[k];
    }
    int incl = s;  // inclusive wave scan
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(incl, off);
      if (lane >= off) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int wbefore = 0;
    for (int k = 0; k < wv; ++k) wbefore += wsum[k];
    int tot = 0;
    for (int k = 0; k < 16; ++k) tot += wsum[k];
    int run = carry_s + wbefore + incl - s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = base + tid * 4 + k;
      if (i < n) out[i] = run;
      run += v[k];
    }
    __syncthreads();
    if (tid == 0) carry_s += tot;
    __syncthreads();
  }
  if (tid == 0) {
    out[n] = carry_s;
    if (total_out) *total_out = carry_s;
  }
}

// out[b] = scan[b*stride] (idx == nullptr) or scan[min(idx[b], n)] with n the
// clamped length of the scanned list, for b = 0..batch.
__global__ void gather_offsets_kernel(const int* __restrict__ scan, const int* __restrict__ idx,
                                      int stride, int batch, const int* n_dev, int cap,
                                      int* __restrict__ out) {
  const int b = threadIdx.x;
  if (b > batch) return;
  if (!idx) {
    out[b] = scan[b * stride];
  } else {
    int n = *n_dev;
    n = n < cap ? n : cap;
    const int i = idx[b];
    out[b] = scan[i < n ? i : n];
  }
}

void launch_extrema(hipStream_t st, const Layout& L, const float* dog, int batch, DetectBufs& D) {
  SegTable S = make_segs(L);
  dim3 grid(S.bpi, batch);
  hipLaunchKernelGGL(extrema_count_kernel, grid, dim3(256), 0, st, S, dog, D.blk_counts);
  const int nblk = S.bpi * batch;
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, D.blk_counts, 1, D.scan_tmp, nullptr,
                     nblk, nblk, D.cand_total);
  hipLaunchKernelGGL(gather_offsets_kernel, dim3(1), dim3(128), 0, st, D.scan_tmp, nullptr, S.bpi,
                     batch, nullptr, 0, D.img_cand_off);
  hipLaunchKernelGGL(extrema_write_kernel, grid, dim3(256), 0, st, S, dog, D.scan_tmp, D.cands,
                     D.cand_cap);
}

// ---- adjustLocalExtrema + calcOrientationHist + peaks ----------------------
struct RefArgs {
  Layout L;
  const float* gpyr;
  const float* dog;
  const MathConsts* mc;
  const Cand* cands;
  const int* cand_total;
  int cand_cap;
  CandOut* couts;
  int* npeaks;
};

constexpr int kOriMaxSamples = 35 * 35;  // radius <= 17 (scl_octv <= 3.81)

__global__ __launch_bounds__(256) void refine_orient_kernel(RefArgs A) {
  __shared__ int sbin[4][kOriMaxSamples + 3];
  __shared__ float sval[4][kOriMaxSamples + 3];
  __shared__ float sh[4][kOriBins + 4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int n = *A.cand_total;
  if (n > A.cand_cap) n = A.cand_cap;
  const ExpConsts ek = A.mc->e;
  const AtanConsts ak = A.mc->t;
  const float* etab = A.mc->exptab;

  for (int ci = blockIdx.x * 4 + wv; ci < n; ci += gridDim.x * 4) {
    const Cand cd = A.cands[ci];
    const int o = cd.ol & 255;
    int layer = cd.ol >> 8;
    int r = cd.r, c = cd.c;
    const Octave& O = A.L.oct[o];
    const long long pitch = O.pitch;
    const float* dimg = A.dog + cd.b * A.L.d_img;
    // ---- adjustLocalExtrema, src/sift.cpp:287-388 (all lanes, uniform) ----
    const float img_scale = 1. / 255;
    const float deriv_scale = img_scale * 0.5f;
    const float second_scale = img_scale;
    const float cross_scale = img_scale * 0.25f;
    float xi = 0, xr = 0, xc = 0, contr = 0;
    bool ok = true;
    int it = 0;
#define AT(pl, yy, xx) ((pl)[(long long)(yy)*pitch + (xx)])
    for (; it < kMaxInterp; ++it) {
      const float* cur = dimg + O.d_off[layer];
      const float* lo = dimg + O.d_off[layer - 1];
      const float* hi = dimg + O.d_off[layer + 1];
      const float g[3] = {(AT(cur, r, c + 1) - AT(cur, r, c - 1)) * deriv_scale,
                          (AT(cur, r + 1, c) - AT(cur, r - 1, c)) * deriv_scale,
                          (AT(hi, r, c) - AT(lo, r, c)) * deriv_scale};
      const float v2 = (float)AT(cur, r, c) * 2;
      const float dxx = (AT(cur, r, c + 1) + AT(cur, r, c - 1) - v2) * second_scale;
      const float dyy = (AT(cur, r + 1, c) + AT(cur, r - 1, c) - v2) * second_scale;
      const float dss = (AT(hi, r, c) + AT(lo, r, c) - v2) * second_scale;
      const float dxy = (AT(cur, r + 1, c + 1) - AT(cur, r + 1, c - 1) - AT(cur, r - 1, c + 1) +
                         AT(cur, r - 1, c - 1)) * cross_scale;
      const float dxs = (AT(hi, r, c + 1) - AT(hi, r, c - 1) - AT(lo, r, c + 1) + AT(lo, r, c - 1)) *
                        cross_scale;
      const float dys = (AT(hi, r + 1, c) - AT(hi, r - 1, c) - AT(lo, r + 1, c) + AT(lo, r - 1, c)) *
                        cross_scale;
      const float H[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss};
      float X[3];
      solve3(H, g, X);
      xi = -X[2];
      xr = -X[1];
      xc = -X[0];
      if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
      if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) ||
          fabsf(xc) > (float)(INT_MAX / 3)) {
        ok = false;
        break;
      }
      c += cv_round(xc);
      r += cv_round(xr);
      layer += cv_round(xi);
      if (layer < 1 || layer > kLayers || c < kBorder || c >= O.cols - kBorder || r < kBorder ||
          r >= O.rows - kBorder) {
        ok = false;
        break;
      }
    }
    if (ok && it >= kMaxInterp) ok = false;
    if (ok) {
      const float* cur = dimg + O.d_off[layer];
      const float* lo = dimg + O.d_off[layer - 1];
      const float* hi = dimg + O.d_off[layer + 1];
      const float g0 = (AT(cur, r, c + 1) - AT(cur, r, c - 1)) * deriv_scale;
      const float g1 = (AT(cur, r + 1, c) - AT(cur, r - 1, c)) * deriv_scale;
      const float g2 = (AT(hi, r, c) - AT(lo, r, c)) * deriv_scale;
      float t = 0;
      t = t + g0 * xc;
      t = t + g1 * xr;
      t = t + g2 * xi;
      contr = AT(cur, r, c) * img_scale + t * 0.5f;
      if (fabsf(contr) * kLayers < (float)0.04) {
        ok = false;
      } else {
        const float v2 = AT(cur, r, c) * 2.f;
        const float dxx = (AT(cur, r, c + 1) + AT(cur, r, c - 1) - v2) * second_scale;
        const float dyy = (AT(cur, r + 1, c) + AT(cur, r - 1, c) - v2) * second_scale;
        const float dxy = (AT(cur, r + 1, c + 1) - AT(cur, r + 1, c - 1) - AT(cur, r - 1, c + 1) +
                           AT(cur, r - 1, c - 1)) * cross_scale;
        const float tr = dxx + dyy;
        const float det = dxx * dyy - dxy * dxy;
        const float et = 10.f;
        if (det <= 0 || tr * tr * et >= (et + 1) * (et + 1) * det) ok = false;
      }
    }
    if (!ok) {
      if (lane == 0) A.npeaks[ci] = 0;
      continue;
    }
    const float kx = (c + xc) * (1 << o);
    const float ky = (r + xr) * (1 << o);
    const int koct = o + (layer << 8) + (cv_round_d((xi + 0.5) * 255) << 16);
    const float ksize = (float)kSigma * pow2f_cr((layer + xi) / kLayers) * (1 << o) * 2;
    const float kresp = fabsf(contr);

    // ---- calcOrientationHist, src/sift.cpp:389-458 ----
    const float scl = ksize * 0.5f / (1 << o);
    const int radius = cv_round(3 * 1.5f * scl);
    const float sigma = 1.5f * scl;
    const float escale = -1.f / (2.f * sigma * sigma);
    const float* gimg = A.gpyr + cd.b * A.L.g_img + O.g_off[layer];
    const int D = 2 * radius + 1;
    const int ns = D * D;  // <= kOriMaxSamples
    for (int s = lane; s < ns; s += 64) {
      const int i = s / D - radius, j = s % D - radius;
      const int y = r + i, x = c + j;
      int bin = -1;
      float val = 0.f;
      if (!(y <= 0 || y >= O.rows - 1) && !(x <= 0 || x >= O.cols - 1)) {
        const float dx = (float)(AT(gimg, y, x + 1) - AT(gimg, y, x - 1));
        const float dy = (float)(AT(gimg, y - 1, x) - AT(gimg, y + 1, x));
        const float w = exp32f((i * i + j * j) * escale, etab, ek);
        const float ori = fast_atan2(dy, dx, ak);
        const float mag = magnitude(dx, dy);
        bin = cv_round((kOriBins / 360.f) * ori);
        if (bin >= kOriBins) bin -= kOriBins;
        if (bin < 0) bin += kOriBins;
        val = w * mag;
      }
      sbin[wv][s] = bin;
      sval[wv][s] = val;
    }
    wave_sync();
    // owner-computes: lane j accumulates bin j in sample (raster) order
    float acc = 0.f;
    if (lane < kOriBins) {
      for (int s = 0; s < ns; ++s) {
        const float v = sval[wv][s];
        acc = acc + ((sbin[wv][s] == lane) ? v : 0.f);
      }
      sh[wv][lane] = acc;
    }
    wave_sync();
    float h = 0.f;
    if (lane < kOriBins) {
      const float* th = sh[wv];
      const int jm2 = (lane + kOriBins - 2) % kOriBins, jp2 = (lane + 2) % kOriBins;
      const int jm1 = (lane + kOriBins - 1) % kOriBins, jp1 = (lane + 1) % kOriBins;
      h = (th[jm2] + th[jp2]) * (1.f / 16.f) + (th[jm1] + th[jp1]) * (4.f / 16.f) +
          th[lane] * (6.f / 16.f);
    }
    float mx = lane < kOriBins ? h : -1.f;
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    wave_sync();
    if (lane < kOriBins) sh[wv][lane] = h;
    wave_sync();
    const float mag_thr = (float)(mx * 0.8f);
    bool peak = false;
    float angle = 0.f;
    if (lane < kOriBins) {
      const int l = lane > 0 ? lane - 1 : kOriBins - 1;
      const int rr = lane < kOriBins - 1 ? lane + 1 : 0;
      const float hl = sh[wv][l], hr = sh[wv][rr];
      if (h > hl && h > hr && h >= mag_thr) {
        peak = true;
        float bin = lane + 0.5f * (hl - hr) / (hl - 2 * h + hr);
        bin = bin < 0 ? kOriBins + bin : bin >= kOriBins ? bin - kOriBins : bin;
        angle = 360.f - (float)((360.f / kOriBins) * bin);
        if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
      }
    }
    const unsigned long long pm = __ballot(peak);
    CandOut* co = A.couts + ci;
    if (peak) {
      const unsigned long long lt = (lane == 0) ? 0ull : (pm & (~0ull >> (64 - lane)));
      co->angle[__popcll(lt)] = angle;
    }
    if (lane == 0) {
      co->x = kx;
      co->y = ky;
      co->size = ksize;
      co->response = kresp;
      co->octave = koct;
      co->img = cd.b;
      co->npeaks = __popcll(pm);
      A.npeaks[ci] = __popcll(pm);
    }
    wave_sync();
#undef AT
  }
}

void launch_refine_orient(hipStream_t st, const Layout& L, const float* gpyr, const float* dog,
                          const MathConsts* mc, DetectBufs& D, int batch) {
  RefArgs A;
  A.L = L;
  A.gpyr = gpyr;
  A.dog = dog;
  A.mc = mc;
  A.cands = D.cands;
  A.cand_total = D.cand_total;
  A.cand_cap = D.cand_cap;
  A.couts = D.couts;
  A.npeaks = D.npeaks;
  (void)batch;
  hipLaunchKernelGGL(refine_orient_kernel, dim3(2048), dim3(256), 0, st, A);
}

// ---- ordered keypoint emission ------------------------------------------------
__global__ __launch_bounds__(256) void emit_kernel(const CandOut* __restrict__ couts,
                                                   const int* __restrict__ kp_scan,
                                                   const int* __restrict__ cand_total, int cand_cap,
                                                   sift_keypoint* __restrict__ kpts, int kp_cap) {
  int n = *cand_total;
  if (n > cand_cap) n = cand_cap;
  for (int ci = blockIdx.x * 256 + threadIdx.x; ci < n; ci += gridDim.x * 256) {
    const int base = kp_scan[ci];
    const int np = kp_scan[ci + 1] - base;
    if (np == 0) continue;
    const CandOut& co = couts[ci];
    for (int k = 0; k < np; ++k) {
      const int pos = base + k;
      if (pos >= kp_cap) break;
      sift_keypoint kp;
      kp.x = co.x;
      kp.y = co.y;
      kp.size = co.size;
      kp.angle = co.angle[k];
      kp.response = co.response;
      kp.octave = co.octave;
      kp.class_id = -1;
      kpts[pos] = kp;
    }
  }
}

void launch_emit(hipStream_t st, DetectBufs& D, int batch, sift_keypoint* kpts, int kp_cap,
                 int* img_kp_off) {
  // kp_scan = exclusive scan of npeaks over the (clamped) candidate list
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, D.npeaks, 1, D.kp_scan,
                     D.cand_total, 0, D.cand_cap, D.kp_total);
  hipLaunchKernelGGL(gather_offsets_kernel, dim3(1), dim3(128), 0, st, D.kp_scan, D.img_cand_off,
                     0, batch, D.cand_total, D.cand_cap, img_kp_off);
  hipLaunchKernelGGL(emit_kernel, dim3(1024), dim3(256), 0, st, D.couts, D.kp_scan, D.cand_total,
                     D.cand_cap, kpts, kp_cap);
}

}  // namespace sift
