// detect.hip -- extrema scan, sub-pixel refinement, orientation assignment
// (reference src/sift.cpp:285-577) for gfx950.
//
// Output order must equal the reference's: octave -> layer -> row -> col ->
// histogram peak (src/sift.cpp:556-557, 487-491, 525), duplicates kept.  The
// GPU therefore never appends with atomics:
//   extrema_walk   -- one wave per 64-column strip of one octave walks a
//                     chunk of rows: the four DoG rows are formed from the
//                     five Gaussian planes in an LDS ring, both detection
//                     layers are tested, and each row's two ballots are two
//                     32-bit words of a candidate bitmask;
//   mask_count / scan / mask_expand -- the bitmask's word order is the
//                     reference's (octave, layer, row, col) order, so an
//                     exclusive scan of per-chunk popcounts gives every
//                     candidate its slot: the list comes out sorted;
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
#include <stdlib.h>

namespace sift {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- candidate bitmask: one bit per (octave, layer, row, col) -------------
// Plane (o, layer) holds rows x wpr 32-bit words (wpr = ceil(cols/32)), bit c%32
// of word r*wpr + c/32; planes follow in (o, layer) order.  Word order within an
// image is therefore exactly the reference's scan order (src/sift.cpp:556-557,
// 487-491), which makes the ordered compaction a plain scan over words.
constexpr int kMaxSeg = 2 * kMaxOctaves;
#ifndef SIFT_WORD_CHUNK
#define SIFT_WORD_CHUNK 512  // A/B builds only (tools/build_var.sh); round 6: 2048 -> 512, one image's mask_expand 11.4 -> 4.9 us
#endif
constexpr int kWordChunk = SIFT_WORD_CHUNK;  // mask words per workgroup in the count/expand passes

struct MaskLayout {
  int n;                          // segments = n_oct * 2
  int bpw;                        // count/expand workgroups per image
  long long w_img;                // words per image
  long long start[kMaxSeg + 1];
  int o[kMaxSeg], layer[kMaxSeg], wpr[kMaxSeg];
};

static MaskLayout make_mask(const Layout& L) {
  MaskLayout M{};
  long long t = 0;
  int n = 0;
  for (int o = 0; o < L.n_oct; ++o)
    for (int layer = 1; layer <= kLayers; ++layer) {
      M.start[n] = t;
      M.o[n] = o;
      M.layer[n] = layer;
      M.wpr[n] = (L.oct[o].cols + 31) / 32;
      t += (long long)L.oct[o].rows * M.wpr[n];
      ++n;
    }
  M.start[n] = t;
  M.n = n;
  M.w_img = t;
  M.bpw = (int)((t + kWordChunk - 1) / kWordChunk);
  if (M.bpw == 0) M.bpw = 1;
  return M;
}

long long mask_words_per_image(const Layout& L) { return make_mask(L).w_img; }
int mask_blocks_per_image(const Layout& L) { return make_mask(L).bpw; }

// ---- pass 1: DoG (src/sift.cpp:280) fused with the 26-neighbour test --------
// One wave owns a 64-column strip (64-aligned, so its ballots are exactly two
// mask words per row) of one octave and walks a chunk of rows.  Each row of
// the five Gaussian planes (or the caller's DoG planes) is loaded once --
// lanes 0 and 1 also fetch the columns x0-1 and x0+64 -- one row ahead of its
// use, turned into the four DoG rows + Gaussian layers 1, 2 and put into a
// three-row LDS ring; row y is then tested and its gradients written as soon
// as row y+1 is in the ring.  Against round 1's 64x16 tiles (a workgroup per
// tile, 29 KB of LDS, 1.16x the rows with the halo; 2.26 vs 1.56 ms per step,
// tools/patches/r5_variants.patch): no 2-row halo per tile (rows are read
// once per chunk), the loads of the next row fly while the current one is
// tested, and a wave needs 4.9 KB of LDS, so 8 waves per SIMD stay resident.
// Same values, same bits (the 26-neighbour test only compares; the gradients
// and DoG are the same float expressions).
constexpr int kWCols = 64 + 4;  // ring row: column x0 - 1 + c at c (c = 0..65)

struct WalkArgs {
  Layout L;
  MaskLayout M;
  const float* gpyr;
  const float* dog;
  float2* grad;
  const MathConsts* mc;
  unsigned* mask;
  int wave_start[kMaxOctaves + 1];  // first wave (blockIdx.x) of octave o
  int strips[kMaxOctaves];
  int chunk;                        // rows per wave
};

// src/sift.cpp:493-511 at ring column c: lo/cu/hi[k] = row y - 1 + k of the
// layer below / at / above the tested one; ties pass.
__device__ __forceinline__ bool ring_extremum(const float* const (&lo)[3], const float* const (&cu)[3],
                                              const float* const (&hi)[3], int c) {
  const float v = cu[1][c];
  if (!(fabsf(v) > kDogThreshold)) return false;
  bool ok = true;
  if (v > 0) {
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        ok = ok && v >= lo[dy][c + dx] && v >= hi[dy][c + dx];
        if (dy != 1 || dx != 0) ok = ok && v >= cu[dy][c + dx];
      }
  } else if (v < 0) {
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        ok = ok && v <= lo[dy][c + dx] && v <= hi[dy][c + dx];
        if (dy != 1 || dx != 0) ok = ok && v <= cu[dy][c + dx];
      }
  } else {
    ok = false;
  }
  return ok;
}

template <bool FROM_G>
__global__ __launch_bounds__(64) void extrema_walk_kernel(WalkArgs A) {
  __shared__ float ring[3][6][kWCols];  // planes: DoG 0..3, Gaussian layers 1, 2
  const int lane = threadIdx.x;
  const int b = blockIdx.y;
  // XCD-aware order (speed only): blocks b and b + 8 share an XCD, so XCD x
  // takes the contiguous run [x P, (x + 1) P) of the (octave, chunk, strip)
  // raster order and neighbouring strips -- which fetch each other's edge
  // columns -- meet in the same L2
  const int per_xcd = (int)(gridDim.x >> 3);
  const int t = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
  if (t >= A.wave_start[A.L.n_oct]) return;
  int o = 0;
  while (o + 1 < A.L.n_oct && A.wave_start[o + 1] <= t) ++o;
  const int local = t - A.wave_start[o];
  const Octave& O = A.L.oct[o];
  const int x0 = (local % A.strips[o]) * 64, y0 = (local / A.strips[o]) * A.chunk;
  const int y1 = min(y0 + A.chunk, O.rows);
  const int rows = O.rows, cols = O.cols;
  const long long pitch = O.pitch;
  const float* g = A.gpyr + b * A.L.g_img;
  const float* dg = FROM_G ? nullptr : A.dog + b * A.L.d_img;
  const int xm = x0 + lane;                       // this lane's column
  const int xh = lane == 0 ? x0 - 1 : x0 + 64;    // halo column of lanes 0, 1
  const bool hl = lane < 2;
  const int xmc = min(xm, cols - 1), xhc = min(max(xh, 0), cols - 1);
  // loads of row r (clamped addresses; out-of-image values are zeroed when the
  // row is put): G1, G2 and then G0, G3, G4 (FROM_G) or the DoG planes 0..3
  auto load = [&](int r, float (&v)[6], float (&h)[6]) {
    const long long rp = (long long)min(max(r, 0), rows - 1) * pitch;
    const long long pm = rp + xmc, ph = rp + xhc;
    v[0] = g[O.g_off[1] + pm];
    v[1] = g[O.g_off[2] + pm];
    if (FROM_G) {
      v[2] = g[O.g_off[0] + pm];
      v[3] = g[O.g_off[3] + pm];
      v[4] = g[O.g_off[4] + pm];
    } else {
#pragma unroll
      for (int k = 0; k < kDogPer; ++k) v[2 + k] = dg[O.d_off[k] + pm];
    }
    if (hl) {
      h[0] = g[O.g_off[1] + ph];
      h[1] = g[O.g_off[2] + ph];
      if (FROM_G) {
        h[2] = g[O.g_off[0] + ph];
        h[3] = g[O.g_off[3] + ph];
        h[4] = g[O.g_off[4] + ph];
      } else {
#pragma unroll
        for (int k = 0; k < kDogPer; ++k) h[2 + k] = dg[O.d_off[k] + ph];
      }
    }
  };
  // DoG (src/sift.cpp:280: dog = g[i+1] - g[i]) and the Gaussian layers into
  // ring slot s at column c; 0 outside the image, as the tile kernel
  // the lane's own column of the ring, kept in registers as well: od[slot][k]
  // = DoG plane k, og[slot][l] = Gaussian layer 1 + l (slots are compile-time
  // constants in the unrolled walk below)
  float od[3][kDogPer], og[3][2];
  auto put1 = [&](int s, int c, const float (&v)[6], bool ok, float (&d)[kDogPer], float (&gg)[2]) {
    const float g1 = ok ? v[0] : 0.f, g2 = ok ? v[1] : 0.f;
    if (FROM_G) {
      const float g0 = ok ? v[2] : 0.f, g3 = ok ? v[3] : 0.f, g4 = ok ? v[4] : 0.f;
      d[0] = g1 - g0;
      d[1] = g2 - g1;
      d[2] = g3 - g2;
      d[3] = g4 - g3;
    } else {
#pragma unroll
      for (int k = 0; k < kDogPer; ++k) d[k] = ok ? v[2 + k] : 0.f;
    }
    gg[0] = g1;
    gg[1] = g2;
#pragma unroll
    for (int k = 0; k < kDogPer; ++k) ring[s][k][c] = d[k];
    ring[s][4][c] = g1;
    ring[s][5][c] = g2;
  };
  auto put = [&](int s, int r, const float (&v)[6], const float (&h)[6]) {
    const bool rok = r >= 0 && r < rows;
    put1(s, lane + 1, v, rok && xm < cols, od[s], og[s]);
    if (hl) {
      float dh[kDogPer], gh[2];
      put1(s, lane == 0 ? 0 : 65, h, rok && xh >= 0 && xh < cols, dh, gh);
    }
  };
  const AtanConsts ak = A.mc->t;
  float2* gr = A.grad + b * A.L.g_img;
  const int wpr = A.M.wpr[2 * o];
  const long long mbase = b * A.M.w_img;
  // row y from ring slots su (y-1), sm (y), sd (y+1)
  auto process = [&](int y, int su, int sm, int sd) {
    const int c = lane + 1;
    if (y > 0 && y < rows - 1 && xm > 0 && xm < cols - 1) {
#pragma unroll
      for (int ls = 0; ls < 2; ++ls) {
        const float dx = (float)(ring[sm][4 + ls][c + 1] - ring[sm][4 + ls][c - 1]);
        const float dy = (float)(og[su][ls] - og[sd][ls]);
        gr[O.g_off[1 + ls] + (long long)y * pitch + xm] = make_float2(magnitude(dx, dy), fast_atan2(dy, dx, ak));
      }
    }
    // src/sift.cpp:493-511, both detection layers: v at (y, x) of DoG plane
    // 1 (layer 1) / 2 (layer 2) is an extremum when |v| > 8 and v >= (<=)
    // all 26 neighbours -- ties pass -- i.e. v >= the max (v <= the min) of
    // the neighbours (finite values: the order of the comparisons does not
    // matter).  Branch-free: per plane the max / min of the 3x3 block,
    // without its centre for the two planes whose centres are tested.
    const int s3[3] = {su, sm, sd};
    float mx9[kDogPer], mn9[kDogPer], mx8[2], mn8[2];
#pragma unroll
    for (int k = 0; k < kDogPer; ++k) {
      float l3[3], r3[3];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        l3[dy] = ring[s3[dy]][k][c - 1];
        r3[dy] = ring[s3[dy]][k][c + 1];
      }
      const float own_ud_max = fmaxf(od[su][k], od[sd][k]), own_ud_min = fminf(od[su][k], od[sd][k]);
      const float side_max = fmaxf(fmaxf(fmaxf(l3[0], l3[1]), l3[2]), fmaxf(fmaxf(r3[0], r3[1]), r3[2]));
      const float side_min = fminf(fminf(fminf(l3[0], l3[1]), l3[2]), fminf(fminf(r3[0], r3[1]), r3[2]));
      const float m8x = fmaxf(side_max, own_ud_max), m8n = fminf(side_min, own_ud_min);
      mx9[k] = fmaxf(m8x, od[sm][k]);
      mn9[k] = fminf(m8n, od[sm][k]);
      if (k == 1 || k == 2) {
        mx8[k - 1] = m8x;
        mn8[k - 1] = m8n;
      }
    }
    const bool inside = y >= kBorder && y < rows - kBorder && xm >= kBorder && xm < cols - kBorder;
    bool f[2];
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      const float v = od[sm][1 + l];
      const float nmax = fmaxf(fmaxf(mx9[l], mx8[l]), mx9[l + 2]);
      const float nmin = fminf(fminf(mn9[l], mn8[l]), mn9[l + 2]);
      f[l] = inside && fabsf(v) > kDogThreshold && ((v > 0 && v >= nmax) || (v < 0 && v <= nmin));
    }
    const unsigned long long m1 = __ballot(f[0]), m2 = __ballot(f[1]);
    if (lane == 0 || lane == 32) {
      const int w = x0 / 32 + (lane >> 5);
      if (w < wpr) {
        const long long base = mbase + (long long)y * wpr + w;
        A.mask[base + A.M.start[2 * o]] = (unsigned)(m1 >> lane);
        A.mask[base + A.M.start[2 * o + 1]] = (unsigned)(m2 >> lane);
      }
    }
  };
  // rows y0-1 .. y1 enter the ring in order (row y0-1+i in slot i % 3); row y
  // is processed once row y+1 is in.  Three register sets rotate, so the
  // loads of the next two rows are in flight while a row is processed.
  float va[6], ha[6], vb[6], hb[6], vc[6], hc[6];
  load(y0 - 1, va, ha);
  load(y0, vb, hb);
  load(y0 + 1, vc, hc);
  // ring slot of row r: (r - y0 + 1) % 3, i.e. set a <-> slot 0, b <-> 1, c <-> 2
  auto step = [&](int r, float (&v)[6], float (&h)[6], int sr) {
    wave_sync();  // the previous process() read slot sr (row r - 3) at other lanes' columns
    put(sr, r, v, h);
    wave_sync();
    if (r + 3 <= y1) load(r + 3, v, h);
    if (r >= y0 + 1) process(r - 1, (sr + 1) % 3, (sr + 2) % 3, sr);
  };
  for (int r = y0 - 1; r <= y1; r += 3) {
    step(r, va, ha, 0);
    if (r + 1 > y1) break;
    step(r + 1, vb, hb, 1);
    if (r + 2 > y1) break;
    step(r + 2, vc, hc, 2);
  }
}

// ---- pass 2: ordered compaction of the bitmask ----------------------------
__global__ __launch_bounds__(256) void mask_count_kernel(const unsigned* __restrict__ mask, long long w_img,
                                                         int bpw, int* __restrict__ blk_counts) {
  __shared__ int wsum[4];
  const int b = blockIdx.y;
  const long long base = (long long)blockIdx.x * kWordChunk;
  const unsigned* m = mask + b * w_img;
  int cnt = 0;
#pragma unroll
  for (int it = 0; it < kWordChunk / 256; ++it) {
    const long long w = base + it * 256 + threadIdx.x;
    if (w < w_img) cnt += __popc(m[w]);
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) blk_counts[b * bpw + blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void mask_expand_kernel(MaskLayout M, const unsigned* __restrict__ mask,
                                                          const int* __restrict__ blk_off,
                                                          Cand* __restrict__ cands, int cap) {
  __shared__ int wcnt[4];
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long base = (long long)blockIdx.x * kWordChunk;
  const unsigned* m = mask + b * M.w_img;
  int run = blk_off[b * M.bpw + blockIdx.x];
  // every word of the chunk in flight at once (the loop below synchronises per step)
  unsigned words[kWordChunk / 256];
#pragma unroll
  for (int it = 0; it < kWordChunk / 256; ++it) {
    const long long w = base + it * 256 + threadIdx.x;
    words[it] = w < M.w_img ? m[w] : 0u;
  }
#pragma unroll
  for (int it = 0; it < kWordChunk / 256; ++it) {
    const long long w = base + it * 256 + threadIdx.x;
    unsigned bits = words[it];
    const int cnt = __popc(bits);
    int incl = cnt;
    for (int off = 1; off < 64; off <<= 1) {
      const int tt = __shfl_up(incl, off);
      if (lane >= off) incl += tt;
    }
    if (lane == 63) wcnt[wv] = incl;
    __syncthreads();
    int before = 0;
    for (int k = 0; k < wv; ++k) before += wcnt[k];
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (bits) {
      int s = 0;
      while (s + 1 < M.n && M.start[s + 1] <= w) ++s;
      const long long wi = w - M.start[s];
      const int r = (int)(wi / M.wpr[s]);
      const int c0 = (int)(wi % M.wpr[s]) * 32;
      int pos = run + before + incl - cnt;
      const int ol = M.o[s] | (M.layer[s] << 8);
      while (bits) {
        const int bit = __builtin_ctz(bits);
        bits &= bits - 1;
        if (pos < cap) cands[pos] = Cand{b, ol, r, c0 + bit};
        ++pos;
      }
    }
    run += tot;
    __syncthreads();
  }
}

// ---- exclusive scan (reduce / scan of tile sums / down-sweep) ---------------
// out[i] = sum(in[0..i)), out[n] = total (also *total_out if given).  n from
// n_dev (clamped to cap) if given, else n_host.  The grid is sized from cap on
// the host; tiles past n contribute 0 and write nothing.
constexpr int kScanT = 256, kScanPer = 16, kScanTile = kScanT * kScanPer;

__device__ __forceinline__ int scan_n(const int* n_dev, int n_host, int cap) {
  const int n = n_dev ? *n_dev : n_host;
  return n < cap ? n : cap;
}

__device__ __forceinline__ int block_sum(int v, int* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  int t = 0;
  for (int k = 0; k < kScanT / 64; ++k) t += red[k];
  return t;
}

__global__ __launch_bounds__(kScanT) void scan_reduce_kernel(const int* __restrict__ in, const int* n_dev,
                                                             int n_host, int cap, int* __restrict__ tsum) {
  __shared__ int red[kScanT / 64];
  const int n = scan_n(n_dev, n_host, cap);
  const long long base = (long long)blockIdx.x * kScanTile;
  int s = 0;
  if (base < n)
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      const long long i = base + k * kScanT + threadIdx.x;
      s += i < n ? in[i] : 0;
    }
  s = block_sum(s, red);
  if (threadIdx.x == 0) tsum[blockIdx.x] = s;
}

// exclusive scan of the tile sums in place (one workgroup); out[n] = total
__global__ __launch_bounds__(1024) void scan_tiles_kernel(int* __restrict__ tsum, int ntiles, const int* n_dev,
                                                          int n_host, int cap, int* __restrict__ out,
                                                          int* total_out) {
  __shared__ int wsum[16];
  __shared__ int carry_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < ntiles; base += 1024) {
    const int i = base + tid;
    const int v = i < ntiles ? tsum[i] : 0;
    int incl = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(incl, off);
      if (lane >= off) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int wbefore = 0, tot = 0;
    for (int k = 0; k < 16; ++k) {
      wbefore += k < wv ? wsum[k] : 0;
      tot += wsum[k];
    }
    if (i < ntiles) tsum[i] = carry_s + wbefore + incl - v;
    __syncthreads();
    if (tid == 0) carry_s += tot;
    __syncthreads();
  }
  if (tid == 0) {
    out[scan_n(n_dev, n_host, cap)] = carry_s;
    if (total_out) *total_out = carry_s;
  }
}

__global__ __launch_bounds__(kScanT) void scan_down_kernel(const int* __restrict__ in, const int* n_dev,
                                                           int n_host, int cap, const int* __restrict__ tsum,
                                                           int* __restrict__ out) {
  __shared__ int wsum[kScanT / 64];
  const int n = scan_n(n_dev, n_host, cap);
  const long long base = (long long)blockIdx.x * kScanTile;
  if (base >= n) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // thread tid owns the kScanPer consecutive elements [base + tid*kScanPer, ...)
  int v[kScanPer];
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const long long i = base + (long long)tid * kScanPer + k;
    v[k] = i < n ? in[i] : 0;
    s += v[k];
  }
  int incl = s;
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off);
    if (lane >= off) incl += t;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int run = tsum[blockIdx.x] + incl - s;
  for (int k = 0; k < wv; ++k) run += wsum[k];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const long long i = base + (long long)tid * kScanPer + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
}

// The same exclusive scan in one workgroup for short lists (one image's
// candidate blocks and orientation peaks): one launch instead of three, on a
// path whose launches are latency-bound.  Thread t owns the `per` consecutive
// elements [t * per, t * per + per) (per <= 64, in registers); out[n] = total.
// Per-image offsets from a scan: gout[b] = out[b * stride] (idx == nullptr) or
// out[min(idx[b], n)], b = 0..batch (gather_offsets_kernel's contract).
struct ScanGather {
  const int* idx;
  int stride, batch;
  int* gout;  // nullptr: no gather
};

constexpr int kScanSmallMax = 1024 * 64;  // one 1080p image: 64,800 candidates
__global__ __launch_bounds__(1024) void scan_small_kernel(const int* __restrict__ in, const int* n_dev, int n_host,
                                                          int cap, int* __restrict__ out, int* total_out,
                                                          ScanGather g) {
  __shared__ int wsum[16];
  const int n = scan_n(n_dev, n_host, cap);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // a multiple of 4 (<= kScanSmallMax / 1024): the chunk is read as int4s, all
  // in flight at once -- a loop of dependent loads cost ~13 us for a 1080p
  // image's ~50 K candidates (round 6)
  const int per = ((n + 1023) / 1024 + 3) & ~3;
  const int i0 = tid * per;
  const bool vec = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  int v[kScanSmallMax / 1024];
#pragma unroll
  for (int k = 0; k < kScanSmallMax / 1024; k += 4) {
    if (k < per && vec && i0 + k + 3 < n) {
      const int4 q = *reinterpret_cast<const int4*>(in + i0 + k);
      v[k] = q.x;
      v[k + 1] = q.y;
      v[k + 2] = q.z;
      v[k + 3] = q.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[k + u] = k < per && i0 + k + u < n ? in[i0 + k + u] : 0;
    }
  }
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanSmallMax / 1024; ++k) s += v[k];
  int incl = s;
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off);
    if (lane >= off) incl += t;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int run = incl - s, tot = 0;
  for (int k = 0; k < 16; ++k) {
    run += k < wv ? wsum[k] : 0;
    tot += wsum[k];
  }
#pragma unroll
  for (int k = 0; k < kScanSmallMax / 1024; ++k)
    if (k < per && i0 + k < n) {
      out[i0 + k] = run;
      run += v[k];
    }
  if (tid == 0) {
    out[n] = tot;
    if (total_out) *total_out = tot;
  }
  if (g.gout) {  // the gather of the per-image offsets, after the whole scan is written
    __syncthreads();
    for (int b = tid; b <= g.batch; b += 1024) {
      int i = b * g.stride;
      if (g.idx) i = g.idx[b] < n ? g.idx[b] : n;
      g.gout[b] = out[i];
    }
  }
}

int scan_tiles_for(long long cap) { return (int)((cap + kScanTile - 1) / kScanTile); }

__global__ void gather_offsets_kernel(const int* __restrict__ scan, const int* __restrict__ idx,
                                      int stride, int batch, const int* n_dev, int cap,
                                      int* __restrict__ out);

void launch_scan(hipStream_t st, const int* in, int* out, const int* n_dev, int n_host, int cap, int* total_out,
                 int* tsum, ScanGather g = ScanGather{nullptr, 0, 0, nullptr}) {
  if (cap <= kScanSmallMax) {
    hipLaunchKernelGGL(scan_small_kernel, dim3(1), dim3(1024), 0, st, in, n_dev, n_host, cap, out, total_out, g);
    return;
  }
  struct Tail {  // the three-kernel scan, then the gather as its own launch
    hipStream_t st;
    const int* out;
    const int* n_dev;
    int cap;
    ScanGather g;
    ~Tail() {
      if (g.gout)
        hipLaunchKernelGGL(gather_offsets_kernel, dim3(1), dim3(256), 0, st, out, g.idx, g.stride, g.batch,
                           g.idx ? n_dev : nullptr, cap, g.gout);
    }
  } tail{st, out, n_dev, cap, g};
  const int nt = scan_tiles_for(cap) > 0 ? scan_tiles_for(cap) : 1;
  hipLaunchKernelGGL(scan_reduce_kernel, dim3(nt), dim3(kScanT), 0, st, in, n_dev, n_host, cap, tsum);
  hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, st, tsum, nt, n_dev, n_host, cap, out, total_out);
  hipLaunchKernelGGL(scan_down_kernel, dim3(nt), dim3(kScanT), 0, st, in, n_dev, n_host, cap, tsum, out);
}

// out[b] = scan[b*stride] (idx == nullptr) or scan[min(idx[b], n)] with n the
// clamped length of the scanned list, for b = 0..batch (any batch: the block
// strides over it).
__global__ void gather_offsets_kernel(const int* __restrict__ scan, const int* __restrict__ idx,
                                      int stride, int batch, const int* n_dev, int cap,
                                      int* __restrict__ out) {
  int n = 0;
  if (idx) {
    n = *n_dev;
    n = n < cap ? n : cap;
  }
  for (int b = threadIdx.x; b <= batch; b += blockDim.x) {
    if (!idx) {
      out[b] = scan[(long long)b * stride];
    } else {
      const int i = idx[b];
      out[b] = scan[i < n ? i : n];
    }
  }
}

// Standalone gradient planes for scales [s_lo, s_hi] (sub-module entry points
// whose pyramids come from the caller).
__global__ __launch_bounds__(256) void grad_kernel(const float* __restrict__ gpyr, float2* __restrict__ grad,
                                                   long long g_img, long long g_off, int pitch, int rows,
                                                   int cols, int nscale, long long plane,
                                                   const MathConsts* __restrict__ mc) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z / nscale, s = blockIdx.z % nscale;
  if (!(y > 0 && y < rows - 1 && x > 0 && x < cols - 1)) return;
  const long long off = b * g_img + g_off + s * plane + (long long)y * pitch + x;
  const float* p = gpyr + off;
  const float dx = (float)(p[1] - p[-1]);
  const float dy = (float)(p[-pitch] - p[pitch]);
  grad[off] = make_float2(magnitude(dx, dy), fast_atan2(dy, dx, mc->t));
}

void launch_grad(hipStream_t st, const Layout& L, const float* gpyr, float2* grad, int batch, int s_lo,
                 int s_hi, const MathConsts* mc) {
  for (int o = 0; o < L.n_oct; ++o) {
    const Octave& O = L.oct[o];
    const int ns = s_hi - s_lo + 1;
    dim3 grid((O.cols + 63) / 64, (O.rows + 3) / 4, batch * ns);
    hipLaunchKernelGGL(grad_kernel, grid, dim3(256), 0, st, gpyr, grad, L.g_img, O.g_off[s_lo], O.pitch,
                       O.rows, O.cols, ns, (long long)O.rows * O.pitch, mc);
  }
}

void launch_extrema(hipStream_t st, const Layout& L, const float* gpyr, float* dog, bool write_dog,
                    float2* grad, const MathConsts* mc, int batch, DetectBufs& D) {
  WalkArgs W;
  W.L = L;
  W.M = make_mask(L);
  W.gpyr = gpyr;
  W.dog = dog;
  W.grad = grad;
  W.mc = mc;
  W.mask = D.mask;
  // rows per wave: about 64 K waves over the launch (measured on the
  // 64 x 1080p batch: 16 K 1.70 ms, 32 K 1.60, 64 K 1.56), at least
  // SIFT_EXTREMA_MIN_CHUNK rows (a chunk re-reads 2 rows)
  long long strip_rows = 0;
  for (int o = 0; o < L.n_oct; ++o) strip_rows += (long long)((L.oct[o].cols + 63) / 64) * L.oct[o].rows;
  constexpr long long target = 65536;  // waves per launch (16 K / 32 K / 64 K measured in round 2)
#ifndef SIFT_EXTREMA_MIN_CHUNK
#define SIFT_EXTREMA_MIN_CHUNK 4  // A/B builds only (tools/build_var.sh); one 1080p image: 4 rows 28.9 us, 8 30.7 (round 6)
#endif
  W.chunk = (int)std::min<long long>(512, std::max<long long>(SIFT_EXTREMA_MIN_CHUNK, strip_rows * batch / target));
  int w = 0;
  for (int o = 0; o < L.n_oct; ++o) {
    W.wave_start[o] = w;
    W.strips[o] = (L.oct[o].cols + 63) / 64;
    w += W.strips[o] * ((L.oct[o].rows + W.chunk - 1) / W.chunk);
  }
  W.wave_start[L.n_oct] = w;
  const int wg = (w + 7) / 8 * 8;  // whole XCD runs (extra waves exit)
  if (write_dog)
    hipLaunchKernelGGL(extrema_walk_kernel<true>, dim3(wg, batch), dim3(64), 0, st, W);
  else
    hipLaunchKernelGGL(extrema_walk_kernel<false>, dim3(wg, batch), dim3(64), 0, st, W);
  const MaskLayout& M = W.M;
  hipLaunchKernelGGL(mask_count_kernel, dim3(M.bpw, batch), dim3(256), 0, st, D.mask, M.w_img, M.bpw,
                     D.blk_counts);
  const int nblk = M.bpw * batch;
  launch_scan(st, D.blk_counts, D.scan_tmp, nullptr, nblk, nblk, D.cand_total, D.scan_tiles,
              ScanGather{nullptr, M.bpw, batch, D.img_cand_off});
  hipLaunchKernelGGL(mask_expand_kernel, dim3(M.bpw, batch), dim3(256), 0, st, M, D.mask, D.scan_tmp,
                     D.cands, D.cand_cap);
}

// ---- adjustLocalExtrema + calcOrientationHist + peaks ----------------------
struct RefArgs {
  Layout L;
  const float* gpyr;
  const float2* grad;
  const float* dog;
  int dog_from_g;  // 1: DoG values are Gaussian-plane differences (no DoG planes stored)
  const MathConsts* mc;
  const Cand* cands;
  const int* cand_total;
  int cand_cap;
  CandOut* couts;
  int* npeaks;
};

// adjustLocalExtrema (src/sift.cpp:287-388) for one candidate.
struct Refined {
  bool ok;
  int layer, r, c, octave;
  float x, y, size, response;
};

// DoG value of layer l at (yy, xx): the stored DoG plane, or -- FROM_G -- the
// difference of the Gaussian planes l+1 and l that buildDoGPyramid stores
// (src/sift.cpp:276; the same float subtraction, so bit-identical).
template <bool FROM_G>
__device__ __forceinline__ Refined refine_candidate(const Layout& Lay, const float* __restrict__ dimg,
                                                    const float* __restrict__ gimg, int o, int layer, int r,
                                                    int c) {
  const Octave& O = Lay.oct[o];
  const long long pitch = O.pitch;
  const float img_scale = 1. / 255;
  const float deriv_scale = img_scale * 0.5f;
  const float second_scale = img_scale;
  const float cross_scale = img_scale * 0.25f;
  float xi = 0, xr = 0, xc = 0, contr = 0;
  Refined R{};
  R.ok = true;
  int it = 0;
  // The 3x3 neighbourhood of (r, c) in DoG layers layer-1 .. layer+1, loaded
  // once per Newton step as one 12-byte row per plane and row (FROM_G: four
  // Gaussian planes, DoG = g[l+1] - g[l], src/sift.cpp:276 -- the same float
  // subtraction as the stored DoG, bit-identical).  (r, c) stays >= 5 from
  // the border and layer in [1, 2], so every row lies inside its plane.
  struct Row3 {
    float a, b, c;
  };
  float cube[3][3][3];  // [layer - (cur - 1)][dy + 1][dx + 1]
  int cube_layer = -1, cube_r = -1, cube_c = -1;
  auto load_cube = [&](int cur, int rr_, int cc_) {
    if (cur == cube_layer && rr_ == cube_r && cc_ == cube_c) return;
    cube_layer = cur;
    cube_r = rr_;
    cube_c = cc_;
    const long long base = (long long)(rr_ - 1) * pitch + (cc_ - 1);
    if (FROM_G) {
      Row3 gv[4][3];
#pragma unroll
      for (int pl = 0; pl < 4; ++pl)
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
          gv[pl][dy] = *reinterpret_cast<const Row3*>(gimg + O.g_off[cur - 1 + pl] + base + dy * pitch);
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          cube[l][dy][0] = gv[l + 1][dy].a - gv[l][dy].a;
          cube[l][dy][1] = gv[l + 1][dy].b - gv[l][dy].b;
          cube[l][dy][2] = gv[l + 1][dy].c - gv[l][dy].c;
        }
    } else {
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const Row3 v = *reinterpret_cast<const Row3*>(dimg + O.d_off[cur - 1 + l] + base + dy * pitch);
          cube[l][dy][0] = v.a;
          cube[l][dy][1] = v.b;
          cube[l][dy][2] = v.c;
        }
    }
  };
// DoG value of layer pl at (yy, xx): every use is within one of (layer, r, c),
// so the cube indices fold to constants
#define AT(pl, yy, xx) cube[(pl) - (layer - 1)][(yy) - r + 1][(xx) - c + 1]
  for (; it < kMaxInterp; ++it) {
    load_cube(layer, r, c);
    const int cur = layer, lo = layer - 1, hi = layer + 1;
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
      R.ok = false;
      return R;
    }
    c += cv_round(xc);
    r += cv_round(xr);
    layer += cv_round(xi);
    if (layer < 1 || layer > kLayers || c < kBorder || c >= O.cols - kBorder || r < kBorder ||
        r >= O.rows - kBorder) {
      R.ok = false;
      return R;
    }
  }
  if (it >= kMaxInterp) {
    R.ok = false;
    return R;
  }
  {
    load_cube(layer, r, c);  // unchanged since the last step's load (the loop left without moving)
    const int cur = layer, lo = layer - 1, hi = layer + 1;
    const float g0 = (AT(cur, r, c + 1) - AT(cur, r, c - 1)) * deriv_scale;
    const float g1 = (AT(cur, r + 1, c) - AT(cur, r - 1, c)) * deriv_scale;
    const float g2 = (AT(hi, r, c) - AT(lo, r, c)) * deriv_scale;
    float t = 0;  // Matx::dot: s = 0; s += a_i * b_i
    t = t + g0 * xc;
    t = t + g1 * xr;
    t = t + g2 * xi;
    contr = AT(cur, r, c) * img_scale + t * 0.5f;
    if (fabsf(contr) * kLayers < (float)0.04) {
      R.ok = false;
      return R;
    }
    const float v2 = AT(cur, r, c) * 2.f;
    const float dxx = (AT(cur, r, c + 1) + AT(cur, r, c - 1) - v2) * second_scale;
    const float dyy = (AT(cur, r + 1, c) + AT(cur, r - 1, c) - v2) * second_scale;
    const float dxy = (AT(cur, r + 1, c + 1) - AT(cur, r + 1, c - 1) - AT(cur, r - 1, c + 1) +
                       AT(cur, r - 1, c - 1)) * cross_scale;
    const float tr = dxx + dyy;
    const float det = dxx * dyy - dxy * dxy;
    const float et = 10.f;
    if (det <= 0 || tr * tr * et >= (et + 1) * (et + 1) * det) {
      R.ok = false;
      return R;
    }
  }
#undef AT
  R.layer = layer;
  R.r = r;
  R.c = c;
  R.x = (c + xc) * (1 << o);
  R.y = (r + xr) * (1 << o);
  R.octave = o + (layer << 8) + (cv_round_d((xi + 0.5) * 255) << 16);
  R.size = (float)kSigma * pow2f_cr((layer + xi) / kLayers) * (1 << o) * 2;
  R.response = fabsf(contr);
  return R;
}

// Refinement: one lane per candidate.  Writes the refined keypoint fields and
// the orientation pass's inputs (refined r, c, layer; npeaks = 1 if kept).
__global__ __launch_bounds__(256) void refine_kernel(RefArgs A) {
  int n = *A.cand_total;
  if (n > A.cand_cap) n = A.cand_cap;
  for (int ci = blockIdx.x * 256 + threadIdx.x; ci < n; ci += gridDim.x * 256) {
    const Cand cd = A.cands[ci];
    const Refined R = A.dog_from_g ? refine_candidate<true>(A.L, nullptr, A.gpyr + cd.b * A.L.g_img, cd.ol & 255,
                                                            cd.ol >> 8, cd.r, cd.c)
                                   : refine_candidate<false>(A.L, A.dog + cd.b * A.L.d_img, nullptr, cd.ol & 255,
                                                             cd.ol >> 8, cd.r, cd.c);
    CandOut* co = A.couts + ci;
    co->x = R.x;
    co->y = R.y;
    co->size = R.size;
    co->response = R.response;
    co->octave = R.octave;
    co->img = cd.b;
    co->npeaks = R.ok ? 1 : 0;
    co->ref_r = R.r;
    co->ref_c = R.c;
    co->ref_layer = R.layer;
  }
}

// Orientation: the batch kernel (orient_slots_kernel below) gives each 8-lane
// group candidates; lanes 8g..8g+7 of a group add their samples to the
// group's 36-bin histograms in raster order, lane q at step q.
constexpr int kOGrp = 8;

__device__ __forceinline__ int ori_radius(float size, int o) {
  const float scl = size * 0.5f / (1 << o);
  return cv_round(3 * 1.5f * scl);
}

// Orientation histograms, one wave per candidate, bins bucketed (round 4;
// the one-image path).
//
// The reference's only ordering constraint (src/sift.cpp:429-437) is that each
// bin receives its terms in window raster order; different bins are
// independent chains.  The batch kernel walks a window one sample per step
// (8 samples per batch, each added after the previous one's LDS round trip),
// so a radius-17 window is a 1,225-step chain and one image's launch is as
// long as its longest such walk.  Here a wave takes a candidate and 64
// consecutive raster samples per batch: every lane forms its sample's bin and
// value, the wave ranks each sample among the earlier samples of the same bin
// (a 6-bit match over ballots), scatters the value to [rank][bin] in LDS, and
// lane b (b < 36) then adds its bin's values in rank order into a register
// accumulator that runs across the batches.  The chain is now the largest
// per-batch bin count, summed over the batches, and every bin still gets
// exactly the reference's adds in the reference's order.  Invalid samples
// (outside the image interior, src/sift.cpp:405,410) join no bin; the masked
// reads past a bin's count add +0.0 to a sum that is >= +0 (exact no-op).
// (A per-XCD dynamic candidate fetch was bit-exact and 16 % slower: each
// draw is a returning atomic that sits in vmcnt order ahead of the
// candidate's gathers; tools/patches/r5_variants.patch.)
[[maybe_unused]] constexpr int kOBWaves = 4;  // waves per workgroup (persistent form, SIFT_ORIENT_PERSIST)

// PERSIST = false (the shipped form, round 6): one wave per candidate slot
// over a grid of the candidate capacity, one wave per workgroup -- the
// dispatcher hands the next candidate to whichever slot frees, instead of a
// fixed stride per resident wave (PERSIST = true, kOBW waves per workgroup:
// round 4's form, an A/B build, SIFT_ORIENT_PERSIST).
template <int kOBW, bool PERSIST>
__global__ __launch_bounds__(64 * kOBW) void orient_bin_kernel(RefArgs A) {
  __shared__ float vals[kOBW][64][kOriBins];  // [wave][rank][bin]: owner reads are conflict free
  __shared__ int cnt[kOBW][64];
  __shared__ float hist[kOBW][kOriBins + 4], sm[kOBW][kOriBins + 4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int n = *A.cand_total;
  if (n > A.cand_cap) n = A.cand_cap;
  const ExpConsts ek = A.mc->e;
  const float etab_lane = A.mc->exptab[lane];
  const unsigned long long below = (1ull << lane) - 1ull;
  cnt[w][lane] = 0;
  // (PERSIST) XCD-aware contiguous split of the raster-ordered candidates
  // (speed only): XCD x takes [x per, (x + 1) per), its waves interleaved
  // over them
  const int nw = PERSIST ? (int)(gridDim.x >> 3) * kOBW : 1;
  const int per = (n + 7) / 8;
  const int xcd = blockIdx.x & 7, wid = (int)(blockIdx.x >> 3) * kOBW + w;
  const int c0 = PERSIST ? xcd * per : (int)blockIdx.x * kOBW + w;
  const int cend = PERSIST ? min(n, c0 + per) : min(n, c0 + 1);
  for (int ci = PERSIST ? c0 + wid : c0; ci < cend; ci += nw) {
    const CandOut& co = A.couts[ci];
    if (co.npeaks == 0) {  // refinement rejected it
      if (lane == 0) A.npeaks[ci] = 0;
      continue;
    }
    const int o = A.cands[ci].ol & 255;
    const Octave& O = A.L.oct[o];
    const int pitch = O.pitch, rr = co.ref_r, rc = co.ref_c;
    // ---- calcOrientationHist, src/sift.cpp:389-437 ----
    const float scl = co.size * 0.5f / (1 << o);
    const int radius = cv_round(3 * 1.5f * scl);
    const float sigma = 1.5f * scl;
    const float escale = -1.f / (2.f * sigma * sigma);
    const float2* gwin = A.grad + co.img * A.L.g_img + O.g_off[co.ref_layer];
    const int D = 2 * radius + 1;
    // the window's valid rectangle (y in [1, rows - 2], x in [1, cols - 2],
    // src/sift.cpp:405,410): the pixels the reference skips are not
    // enumerated, so the rest keep their raster order and a sample needs no
    // range test (a kept candidate lies >= 5 px inside, so the rectangle is
    // >= min(rad + 5, cols - 2) >= 9 columns wide)
    const int i0 = max(0, 1 - rr + radius), i1 = min(D - 1, O.rows - 2 - rr + radius);
    const int j0 = max(0, 1 - rc + radius), j1 = min(D - 1, O.cols - 2 - rc + radius);
    const int W = max(j1 - j0 + 1, 1), ns = max(j1 - j0 + 1, 0) * max(i1 - i0 + 1, 0);
    // lane's sample index base + lane as (si, sj) of the window, moved on by
    // 64 = q W + rem per batch
    int si = i0 + lane / W, sj = j0 + lane - (lane / W) * W;
    const int q64 = 64 / W, r64 = 64 - q64 * W, jend = j0 + W;
    float acc = 0.f;  // lane b < 36: bin b's running sum
    // the batch at (si, sj): validity and the gather (issued one batch ahead,
    // so its latency runs under the previous batch's bucketing)
    auto gather = [&](int base_, bool& ok_, float2& mo_) {
      const int y = rr + si - radius, x = rc + sj - radius;
      ok_ = base_ + lane < ns;
      mo_ = gwin[ok_ ? (long long)y * pitch + x : (long long)rr * pitch + rc];  // (Mag, Ori)
    };
    auto step64 = [&]() {
      si += q64;
      sj += r64;
      if (sj >= jend) {
        sj -= W;
        ++si;
      }
    };
    bool ok_n;
    float2 mo_n;
    gather(0, ok_n, mo_n);
    for (int base = 0; base < ns; base += 64) {
      const int i = si - radius, j = sj - radius;
      const bool ok = ok_n;
      const float2 mo = mo_n;
      step64();
      if (base + 64 < ns) gather(base + 64, ok_n, mo_n);
      // |argument| <= 2 * 17^2 / (2 * 2.85^2) < 36: exp32f's input clamp never acts
      const float wgt = exp32f_v<false>((i * i + j * j) * escale, etab_lane, ek);
      // Ori in [0, 360]: bin in [0, 36], the reference's wraps reduce to 36 -> 0
      const int bin = cv_round((kOriBins / 360.f) * mo.y);
      const float val = wgt * mo.x;
      const int key = ok ? (bin != kOriBins ? bin : 0) : 63;
      // lanes with the same key: match over the key's 6 bits
      unsigned long long m = ~0ull;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const unsigned long long bk = __ballot((key >> k) & 1);
        m &= ((key >> k) & 1) ? bk : ~bk;
      }
      const int rank = __popcll(m & below), total = __popcll(m);
      if (ok) {
        vals[w][rank][key] = val;
        if (rank == total - 1) cnt[w][key] = total;
      }
      wave_sync();
      int c = 0;
      if (lane < kOriBins) {
        c = cnt[w][lane];
        cnt[w][lane] = 0;
      }
      // bin lane's values in rank (= raster) order, 4 reads in flight
      for (int r = 0; __ballot(r < c); r += 4) {
        float v4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v4[u] = (r + u < c) ? vals[w][r + u][lane] : 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = acc + v4[u];
      }
      wave_sync();
    }
    // ---- smoothing (src/sift.cpp:440-451), max, peaks (src/sift.cpp:524-541) ----
    if (lane < kOriBins) hist[w][lane] = acc;
    wave_sync();
    float h = -1.f;
    if (lane < kOriBins) {
      const float* th = hist[w];
      const int t = lane;
      const int jm2 = (t + kOriBins - 2) % kOriBins, jp2 = (t + 2) % kOriBins;
      const int jm1 = (t + kOriBins - 1) % kOriBins, jp1 = (t + 1) % kOriBins;
      h = (th[jm2] + th[jp2]) * (1.f / 16.f) + (th[jm1] + th[jp1]) * (4.f / 16.f) + th[t] * (6.f / 16.f);
      sm[w][t] = h;
    }
    float mx = h;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) mx = fmaxf(mx, __shfl_xor(mx, k));
    wave_sync();
    const float mag_thr = (float)(mx * 0.8f);
    bool pk = false;
    float ang = 0.f;
    if (lane < kOriBins) {
      const int t = lane;
      const int l = t > 0 ? t - 1 : kOriBins - 1;
      const int r2 = t < kOriBins - 1 ? t + 1 : 0;
      const float hl = sm[w][l], hr = sm[w][r2];
      if (h > hl && h > hr && h >= mag_thr) {
        float bn = t + 0.5f * (hl - hr) / (hl - 2 * h + hr);
        bn = bn < 0 ? kOriBins + bn : bn >= kOriBins ? bn - kOriBins : bn;
        float a = 360.f - (float)((360.f / kOriBins) * bn);
        if (fabsf(a - 360.f) < FLT_EPSILON) a = 0.f;
        ang = a;
        pk = true;
      }
    }
    const unsigned long long pmask = __ballot(pk);
    CandOut* cw = A.couts + ci;
    if (pk) cw->angle[__popcll(pmask & below)] = ang;
    if (lane == 0) A.npeaks[ci] = __popcll(pmask);
    wave_sync();
  }
}

// Orientation histograms, kOSlots candidates per lane group (default kernel).
//
// One candidate per group (round 1's orient_kernel) is bound by its histogram
// chain: a group's 8 samples of a batch are applied one after the other (each read-modify-write waits for the
// previous one's LDS round trip, ~100 cycles), and a wave's run time is the
// sum of its chains, which more resident waves cannot shorten.  Here each
// group carries kOSlots candidates at once -- 8 x kOSlots per wave -- with one
// histogram each, so every step of the chain issues kOSlots independent reads,
// one wait, kOSlots adds and kOSlots writes: the same ordered sums, kOSlots
// chains in flight per wave.  The gathers of the next batch are issued before
// the current batch's chain (software pipeline).  Lane q of a group adds its
// sample at step q, as before, so every bin receives its terms in the
// reference's raster order (src/sift.cpp:429-437); an invalid sample adds +0.0
// to bin 0 (exact no-op: every bin is >= +0).
template <int kOSlots>
#ifndef SIFT_ORIENT_WPE
#define SIFT_ORIENT_WPE 6  // A/B builds only (tools/build_var.sh): waves per SIMD orient_slots_kernel<2> is budgeted for
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kOSlots == 2 ? SIFT_ORIENT_WPE : 1))) void orient_slots_kernel(
    RefArgs A) {
  constexpr int SB = kOGrp * kOSlots;   // candidates per sub-batch
  constexpr int NSB = 64 / SB;          // sub-batches per ranked chunk
  constexpr int CH = NSB * SB;          // candidates per ranked chunk (<= 64: one per lane)
  __shared__ float oh[kOSlots][kOGrp][kOriBins + 4];
  __shared__ float sm[kOGrp][kOriBins + 4];
  __shared__ int sord[SB];
  __shared__ float etab[64];  // exp32f table, LDS-resident (gathered per sample)
  const int lane = threadIdx.x & 63;
  const int g = lane >> 3, q = lane & 7;
  int n = *A.cand_total;
  if (n > A.cand_cap) n = A.cand_cap;
  const ExpConsts ek = A.mc->e;
  etab[lane] = A.mc->exptab[lane];
  wave_sync();

  // XCD-aware contiguous split of the raster-ordered candidates (speed only)
  const int xcd = blockIdx.x & 7, nslot = gridDim.x >> 3, wslot = blockIdx.x >> 3;
  const int per = ((n + 7) / 8 + CH - 1) / CH * CH;
  const int c0 = xcd * per;
  const int cend = min(n, (xcd + 1) * per);
  const int chend = c0 + (max(cend - c0, 0) + CH - 1) / CH * CH;
  for (int cb = c0 + wslot * SB; cb < chend; cb += nslot * SB) {
    // lane balance: the chunk's CH candidates ranked by window radius, this
    // sub-batch takes SB consecutive ranks (XOR with the pass index: no wave
    // always draws the largest)
    const int rel = (cb - c0) / SB, pass = rel / nslot;
    const int kc = c0 + (rel / NSB) * CH, win = ((rel % NSB) ^ (pass % NSB)) * SB;
    {
      const int kk = kc + lane;
      int key = 0x1ffffff;  // past the end: ranked last
      if (lane < CH && kk < cend) {
        const CandOut& co = A.couts[kk];
        key = co.npeaks ? min(max(ori_radius(co.size, A.cands[kk].ol & 255), 0), 0xffffff) : 0;
      }
      key = (key << 6) | lane;
      int rank = 0;
#pragma unroll
      for (int m = 0; m < 64; ++m) rank += __builtin_amdgcn_readlane(key, m) < key ? 1 : 0;
      if (rank >= win && rank < win + SB) sord[rank - win] = kk;
      wave_sync();
    }
    // per slot: the window's top-left gradient address (gwin, pitch) and the
    // sample walk (si, sj) over the window's valid rectangle -- interior
    // pixels only, src/sift.cpp:405,410, the pixels the reference skips are
    // never enumerated, so the raster order of the rest is unchanged and a
    // sample needs no per-pixel range test: [j0, jend) x rows from si
    int radius[kOSlots], ns[kOSlots], Dw[kOSlots], si[kOSlots], sj[kOSlots], pitch[kOSlots], jend[kOSlots];
    float escale[kOSlots];
    const float2* gwin[kOSlots];
    int nmax = 0;
#pragma unroll
    for (int u = 0; u < kOSlots; ++u) {
      const int ci = sord[u * kOGrp + g];
      bool ok = false;
      int o = 0, rl = 0, b = 0, rr = 0, rc = 0;
      float size = 0.f;
      if (ci < cend) {
        const CandOut& co = A.couts[ci];
        ok = co.npeaks != 0;
        o = A.cands[ci].ol & 255;
        size = co.size;
        rr = co.ref_r;
        rc = co.ref_c;
        rl = co.ref_layer;
        b = co.img;
      }
      const Octave& O = A.L.oct[o];
      pitch[u] = (int)O.pitch;
      // ---- calcOrientationHist setup, src/sift.cpp:389-402 ----
      const float scl = size * 0.5f / (1 << o);
      const int rad = ok ? cv_round(3 * 1.5f * scl) : 0;
      radius[u] = rad;
      const float sigma = 1.5f * scl;
      escale[u] = -1.f / (2.f * sigma * sigma);
      // (rr, rc) is an interior pixel (refinement keeps it >= 5 from the
      // border), so the window centre is a valid address for every slot
      gwin[u] = A.grad + b * A.L.g_img + O.g_off[ok ? rl : 0] + (long long)(rr - rad) * pitch[u] + (rc - rad);
      const int D = 2 * rad + 1;
      // y = rr + si - rad in [1, rows - 2], x = rc + sj - rad in [1, cols - 2]
      const int i0 = max(0, 1 - rr + rad), i1 = min(D - 1, O.rows - 2 - rr + rad);
      const int j0 = max(0, 1 - rc + rad), j1 = min(D - 1, O.cols - 2 - rc + rad);
      const int wv = j1 - j0 + 1, hv = i1 - i0 + 1;
      ns[u] = ok && wv > 0 && hv > 0 ? wv * hv : 0;
      // a kept candidate lies >= 5 px inside its octave (cols >= 11) and
      // rad = cvRound(4.5 scl) >= 8, so wv >= min(rad + 5, cols - 2) >= 9 > 8:
      // one advance wraps at most once; rejected: never wraps
      Dw[u] = ns[u] ? wv : 0x40000000;
      jend[u] = ns[u] ? j1 + 1 : 0x40000000;
      // lane q walks samples s = q, q+8, ... as (row si, column sj) of the rectangle
      si[u] = i0;
      sj[u] = j0 + q;
      while (sj[u] >= jend[u]) {
        sj[u] -= Dw[u];
        ++si[u];
      }
      nmax = max(nmax, ns[u]);
      for (int t = q; t < kOriBins; t += 8) oh[u][g][t] = 0.f;
    }
    int okbits = 0;  // slot u's candidate is kept (bit u): read by the epilogue's rolled loop
#pragma unroll
    for (int u = 0; u < kOSlots; ++u) okbits |= ns[u] > 0 ? 1 << u : 0;
    nmax = max(nmax, __shfl_xor(nmax, 8));
    nmax = max(nmax, __shfl_xor(nmax, 16));
    nmax = max(nmax, __shfl_xor(nmax, 32));
    wave_sync();
    // one batch (one sample per lane and slot): the gather, branch-free (the
    // window centre for an invalid sample), and the weight W = exp32f, which
    // depends on the position only (src/sift.cpp:424); w = -1 marks an invalid
    // sample (exp32f > 0 for every window position)
    float2 mo[kOSlots];
    float wt[kOSlots];
    auto fetch = [&](int base) {
#pragma unroll
      for (int u = 0; u < kOSlots; ++u) {
        const int i = si[u] - radius[u], j = sj[u] - radius[u];
        const bool okv = base + q < ns[u];
        // 24-bit products, 32-bit offsets (full-rate VALU; a window's offsets are < 2^31)
        mo[u] = gwin[u][(unsigned)(okv ? __mul24(si[u], pitch[u]) + sj[u] : __mul24(radius[u], pitch[u] + 1))];  // (Mag, Ori)
        // |argument| <= 2 * 17^2 / (2 * 2.85^2) < 36: exp32f's input clamp never acts
        const float w = exp32f<false>((__mul24(i, i) + __mul24(j, j)) * escale[u], etab, ek);
        wt[u] = okv ? w : -1.f;
        sj[u] += 8;  // at most one wrap (above)
        if (sj[u] >= jend[u]) {
          sj[u] -= Dw[u];
          ++si[u];
        }
      }
    };
    if (nmax > 0) fetch(0);
    for (int base = 0; base < nmax; base += 8) {
      int bin[kOSlots];
      float val[kOSlots];
#pragma unroll
      for (int u = 0; u < kOSlots; ++u) {
        // src/sift.cpp:426-432: Ori = fastAtan2 (precomputed), bin, W * Mag
        // Ori in [0, 360] (fastAtan2 of this library's gradients) puts bn in
        // [0, 36]: the reference's two wraps reduce to 36 -> 0, folded into
        // the validity select
        const int bn = cv_round((kOriBins / 360.f) * mo[u].y);
        const bool okv = wt[u] > 0.f;
        bin[u] = okv && bn != kOriBins ? bn : 0;
        val[u] = okv ? wt[u] * mo[u].x : 0.f;
      }
      if (base + 8 < nmax) fetch(base + 8);  // next batch's gathers fly during this chain
      // step jj: lane jj of every group adds its kOSlots samples into the
      // slots' histograms (kOSlots independent rows: reads, one wait, adds,
      // writes); the wave's LDS operations stay in program order, so step
      // jj + 1 reads what step jj wrote.  Each step tests a fresh opaque copy
      // of q behind a compiler barrier: with plain q == jj guards -- eight
      // mutually exclusive blocks for one thread -- hipcc rebuilt the steps as
      // a switch on q and ran them out of order (measured: 3 % of the angles
      // a few ulps off).  (A branch-free form, the other lanes updating a
      // scratch word, measured 1.54 ms against 1.42: its scratch accesses
      // share banks with the histogram rows.)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        int qv = q;
        asm volatile("; orient step %1" : "+v"(qv) : "n"(jj) : "memory");
        if (qv == jj) {
          float h[kOSlots];
#pragma unroll
          for (int u = 0; u < kOSlots; ++u) h[u] = oh[u][g][bin[u]];
#pragma unroll
          for (int u = 0; u < kOSlots; ++u) oh[u][g][bin[u]] = h[u] + val[u];
        }
      }
    }
    wave_sync();
#pragma unroll 1
    for (int u = 0; u < kOSlots; ++u) {
      // smoothing (src/sift.cpp:440-451), max, peaks (src/sift.cpp:524-541)
      float mx = -1.f;
      for (int t = q; t < kOriBins; t += 8) {
        const float* th = oh[u][g];
        const int jm2 = (t + kOriBins - 2) % kOriBins, jp2 = (t + 2) % kOriBins;
        const int jm1 = (t + kOriBins - 1) % kOriBins, jp1 = (t + 1) % kOriBins;
        const float h = (th[jm2] + th[jp2]) * (1.f / 16.f) + (th[jm1] + th[jp1]) * (4.f / 16.f) +
                        th[t] * (6.f / 16.f);
        sm[g][t] = h;
        mx = fmaxf(mx, h);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 1));
      mx = fmaxf(mx, __shfl_xor(mx, 2));
      mx = fmaxf(mx, __shfl_xor(mx, 4));
      wave_sync();
      const float mag_thr = (float)(mx * 0.8f);
      unsigned long long pmask = 0;
      float ang[5];
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const int t = q + 8 * m;
        ang[m] = 0.f;
        if (t < kOriBins && ((okbits >> u) & 1)) {
          const int l = t > 0 ? t - 1 : kOriBins - 1;
          const int r2 = t < kOriBins - 1 ? t + 1 : 0;
          const float h = sm[g][t], hl = sm[g][l], hr = sm[g][r2];
          if (h > hl && h > hr && h >= mag_thr) {
            float bn = t + 0.5f * (hl - hr) / (hl - 2 * h + hr);
            bn = bn < 0 ? kOriBins + bn : bn >= kOriBins ? bn - kOriBins : bn;
            float a = 360.f - (float)((360.f / kOriBins) * bn);
            if (fabsf(a - 360.f) < FLT_EPSILON) a = 0.f;
            ang[m] = a;
            pmask |= 1ull << t;
          }
        }
      }
      pmask |= __shfl_xor(pmask, 1);
      pmask |= __shfl_xor(pmask, 2);
      pmask |= __shfl_xor(pmask, 4);
      const int ci = sord[u * kOGrp + g];
      if (ci < cend) {
        CandOut* co = A.couts + ci;
#pragma unroll
        for (int m = 0; m < 5; ++m) {
          const int t = q + 8 * m;
          if (t < kOriBins && ((pmask >> t) & 1ull))
            co->angle[__popcll(pmask & ((1ull << t) - 1ull))] = ang[m];
        }
        // co->npeaks keeps the refine pass's kept flag (other waves rank
        // their chunk from it); the peak count goes to A.npeaks only
        const int np = ((okbits >> u) & 1) ? __popcll(pmask) : 0;
        if (q == 0) A.npeaks[ci] = np;
      }
      wave_sync();
    }
  }
}

bool one_image_variants(const Layout& L, int batch) {
  static const long long lim = [] {
    const char* e = getenv("SIFT_HIP_ONE_IMAGE_PX");
    return e ? atoll(e) : kOneImagePx;
  }();
  return batch == 1 && (long long)L.rows * L.cols <= lim;
}

void launch_refine_orient(hipStream_t st, const Layout& L, const float* gpyr, const float2* grad,
                          const float* dog, const MathConsts* mc, DetectBufs& D, int batch) {
  RefArgs A;
  A.L = L;
  A.gpyr = gpyr;
  A.grad = grad;
  A.dog = dog;
  A.dog_from_g = dog == nullptr;
  A.mc = mc;
  A.cands = D.cands;
  A.cand_total = D.cand_total;
  A.cand_cap = D.cand_cap;
  A.couts = D.couts;
  A.npeaks = D.npeaks;
  hipLaunchKernelGGL(refine_kernel, dim3(resident_grid((const void*)refine_kernel, 256, 0, 2048)), dim3(256), 0, st, A);
  // batches: two candidates per lane group (orient_slots_kernel<2>; three
  // slots 1.65, four 1.53-1.57 vs 1.48-1.50 ms, round 5); one image: one wave
  // per candidate with bucketed bins (orient_bin_kernel, round 4), whose chain
  // is a window's largest per-batch bin counts instead of its whole sample
  // walk.  Every variant is bit-identical (the losers are kept as
  // tools/patches/r5_variants.patch).
  // One image: a workgroup (one wave) per candidate slot, so the dispatcher
  // gives the next candidate to whichever wave slot frees first -- a fixed
  // stride per resident wave left the waves alive 40 % of the launch on
  // average (61.6 vs 41.8 us for one 1080p image, round 6; rejected
  // candidates exit after one load).
#ifndef SIFT_ORIENT_PERSIST
#define SIFT_ORIENT_PERSIST 0  // A/B builds only (tools/build_var.sh): 1 = the round-4 resident grid
#endif
  if (one_image_variants(L, batch)) {
#if SIFT_ORIENT_PERSIST
    hipLaunchKernelGGL((orient_bin_kernel<kOBWaves, true>),
                       dim3(resident_grid((const void*)orient_bin_kernel<kOBWaves, true>, 64 * kOBWaves, 0, 2048)),
                       dim3(64 * kOBWaves), 0, st, A);
#else
    hipLaunchKernelGGL((orient_bin_kernel<1, false>), dim3(std::max(1, D.cand_cap)), dim3(64), 0, st, A);
#endif
  } else {
    // (one 8K image: 4 resident grids were 457 -> 520 us here, unlike the
    // descriptor's; profiles/r6_one_image_grids_ab.txt)
    hipLaunchKernelGGL(orient_slots_kernel<2>,
                       dim3(resident_grid((const void*)orient_slots_kernel<2>, 64, 0, 8192)), dim3(64), 0, st, A);
  }
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

// End-of-call status (one lane).  err[0..2] are sticky words (assertion,
// candidate workspace overflow, keypoint capacity exceeded); this call's own
// overflows are added to them.  stat = {candidates, keypoints, this call's
// bits, all sticky bits} (bit i <-> err[i]), copied by the host to pinned
// memory in the same stream, so it arrives with the stream synchronisation.
__global__ void status_kernel(const int* __restrict__ cand_total, int cand_cap, const int* __restrict__ img_off,
                              int batch, int kp_cap, int* __restrict__ err, int* __restrict__ stat) {
  if (threadIdx.x != 0) return;
  const int ct = cand_total ? *cand_total : 0;
  const int n = img_off ? img_off[batch] : 0;
  const int fresh = (err[0] ? kErrAssert : 0) | (ct > cand_cap ? kErrWorkspace : 0) | (n > kp_cap ? kErrKpCapacity : 0) |
                    (err[3] ? kErrStall : 0);
  if (fresh & kErrWorkspace) err[1] = 1;
  if (fresh & kErrKpCapacity) err[2] = 1;
  stat[0] = ct;
  stat[1] = n;
  stat[2] = fresh;
  stat[3] = (err[0] ? kErrAssert : 0) | (err[1] ? kErrWorkspace : 0) | (err[2] ? kErrKpCapacity : 0) |
            (err[3] ? kErrStall : 0);
}

void launch_status(hipStream_t st, const int* cand_total, int cand_cap, const int* img_off, int batch, int kp_cap,
                   int* err, int* stat) {
  hipLaunchKernelGGL(status_kernel, dim3(1), dim3(64), 0, st, cand_total, cand_cap, img_off, batch, kp_cap, err,
                     stat);
}

void launch_emit(hipStream_t st, DetectBufs& D, int batch, sift_keypoint* kpts, int kp_cap,
                 int* img_kp_off) {
  // kp_scan = exclusive scan of npeaks over the (clamped) candidate list
  launch_scan(st, D.npeaks, D.kp_scan, D.cand_total, 0, D.cand_cap, D.kp_total, D.scan_tiles,
              ScanGather{D.img_cand_off, 0, batch, img_kp_off});
  hipLaunchKernelGGL(emit_kernel, dim3(1024), dim3(256), 0, st, D.couts, D.kp_scan, D.cand_total,
                     D.cand_cap, kpts, kp_cap);
}

}  // namespace sift
