// descriptor.hip -- 128-D descriptor (reference src/sift.cpp:579-753) for gfx950.
//
// The reference builds a 6x6x10 trilinear histogram by adding window samples
// in raster order; every bin's float sum must keep that order to be
// bit-exact.  Design (one wave = 8 keypoints, lanes 8g..8g+7 own keypoint g):
//
//  * Samples: only the (i, j) that can pass the rotated-square test
//    rbin, cbin in (-1, d) are enumerated -- per window row the candidate
//    j-range is derived from the two slabs |r_rot|, |c_rot| < 2.5 (plus a
//    margin), so about half of the (2r+1)^2 window is skipped; the exact float
//    predicate of src/sift.cpp:620-621 still decides each sample.  Gradient
//    magnitude / orientation per pixel come precomputed (detect.hip), so a
//    sample is one 8-byte gather + exp32f + the trilinear weights.
//  * Accumulation by bin ownership: a sample's 8 corners (r0+dr, c0+dc, o0+do)
//    always have 8 distinct parities (R&1, C&1, O&1).  Lane q of a group owns
//    every bin of parity q, so each sample hands exactly one corner to each
//    lane and every bin is updated by one lane only, in sample order -- plain
//    per-lane LDS read-modify-writes, no atomics, no cross-lane hazards.  The
//    histogram lives at [qidx][lane] (qidx = (R'>>1)*10 + (C'>>1)*5 + (O>>1)
//    over the interior rows / columns R' = R-1, C' = C-1 in [0, 4) -- the only
//    bins the fold reads; a border-bin update carries +0.0 into an interior
//    bin), so all 64 lanes of an update hit distinct banks and a wave needs
//    5.1 KB, not 11.5 KB.
//  * One image (round 6): a keypoint's window is split over 4 groups by the
//    half of the interior rows and the half of the interior columns its bins
//    lie in (window parts, PARTS); each group walks only the samples that
//    reach its bins, in raster order, so a keypoint's longest owner chain is
//    ~0.36 of its window.  (Plain LDS
//    read-modify-writes: ds_add_f32 is bit-exact here but took the batch
//    descriptor from 5.6 to 50.9 ms; profiles/r6_desc_one_image_ab.txt.)
//  * Fold, 0.2 clamp, uchar quantisation, RootSIFT (src/sift.cpp:676-721)
//    keep the reference's sequential sums (lane 0 of the group).
#include "common.hpp"

#include <float.h>
#include <stdlib.h>

#include <type_traits>

// waves per SIMD the batch descriptor kernel is compiled for (register budget;
// 3 with no spills measured 8.4-8.5 vs 7.6 ms, round 3; 5 -- 96 VGPRs, spills
// outside the sample loop -- 8.34 vs 6.42-6.46 ms, round 4,
// profiles/r4_desc_wpe5_ab.txt)
constexpr int kDescWpe = 4;

namespace sift {

__device__ __forceinline__ void wave_sync_d() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kGrp = 8;            // keypoints per wave
#ifndef SIFT_DESC_RANK_CHUNK
#define SIFT_DESC_RANK_CHUNK 256  // A/B builds (tools/build_var.sh): 128, 256, 512
#endif
constexpr int kRankChunk = SIFT_DESC_RANK_CHUNK;  // keypoints ranked together by window size (desc_rank_kernel)
constexpr int kSubPerChunk = kRankChunk / kGrp;
constexpr int kSubBits = kSubPerChunk == 16 ? 4 : kSubPerChunk == 32 ? 5 : 6;
static_assert(kSubPerChunk == 1 << kSubBits, "the sub-batch position hash yields kSubBits bits");
constexpr int kQBins = 20;         // bins per parity class: 2 x 2 x 5 interior
constexpr int kMaxWinRows = 81;    // window rows with a row table (radius <= 40)
constexpr int kRowsTab = kMaxWinRows + 2;  // + the entries D, D + 1 the walk reads past its last row (unused values)

struct DescArgs {
  Layout L;
  const float2* grad;     // per-pixel (magnitude, orientation) planes, gpyr layout
  const MathConsts* mc;
  const sift_keypoint* kpts;
  const int* perm;        // [n] keypoint indices ranked by window size within chunks of kRankChunk
                          // (null: one image, last keypoint first -- see the sub-batch loop)
  const int* img_kp_off;  // [batch+1]
  int batch;
  int kp_cap;
  float* desc;
  int first_octave;
  int* err_flag;
};

// Narrow [lo, hi] to the j with |j*a + b| < 2.5 (+ margin).
// inv_a = 1 / a (per keypoint): the bounds only have to enclose the samples
// the exact predicate keeps, and the margin (>= 0.057 in j for |a| <= 1/5.7)
// dwarfs the rounding of a multiply by the reciprocal.
// A window part (PARTS > 1, below) narrows |.| < 2.5 to (lim_lo, lim_hi).
__device__ __forceinline__ void slab(float a, float inv_a, float b, int& lo, int& hi, float lim_lo = -2.5f,
                                     float lim_hi = 2.5f) {
  const float m = 1e-2f;  // margin >> float rounding of r_rot / c_rot
  const float l0 = lim_lo - m, l1 = lim_hi + m;
  if (fabsf(a) < 1e-12f) {
    if (!(b > l0 && b < l1)) hi = lo - 1;
    return;
  }
  float x0 = (l0 - b) * inv_a, x1 = (l1 - b) * inv_a;
  if (x0 > x1) {
    const float t = x0;
    x0 = x1;
    x1 = t;
  }
  lo = max(lo, (int)fmaxf(ceilf(x0), -1e6f));
  hi = min(hi, (int)fminf(floorf(x1), 1e6f));
}

// Record hand-off (packed, round 2): values in a 2 KB array laid out so that
// the eight ds_write_b32 of a batch are bank-conflict free whatever the
// samples' parities (round 6, see the store), each store address one XOR, the
// owner's two ds_read_b128 at most 2-way; the bin bytes handed to their owners in
// registers (round 4), a 16-bit row table for caller keypoints (1.3 KB; DET:
// 32-bit cumulative entries, 2.7 KB), and the in-flight records packed as 8
// values + 2 words of bin bytes, so four waves per SIMD fit.  (Round 1's
// float2 (qidx, value) records at [sample][group][owner] with a trash row,
// 12.4 KB per wave and three waves per SIMD, were 8.71 vs 8.39 ms per step:
// tools/patches/r5_variants.patch.)
constexpr int kRecG = 64;  // value words per group (8 owners x 8 samples, see the store)

struct RecT {  // one lane's 8 corner records
  float v[8];
  unsigned qb[2];  // byte s (word s >> 2): qidx of corner s ^ odd, the one owner slot s takes
};

// DET: the keypoints come from this library's detection, so every window has
// radius <= 40 (scl < 1.6 * 2^1.25, src/sift.cpp:588) and a row table: the
// whole-window walk and its interior tests compile away.
// PF: sample batches in flight.  1: the next batch's gather is issued in the
// step that runs this batch's chain and used right after it.  2 (default for
// detected keypoints): its gather is issued a step earlier, so it flies for a
// whole step -- a wave that is alone on its SIMD (one image) no longer waits a
// full memory latency per batch, and at four waves per SIMD (batches) the
// descriptor took 6.36-6.38 vs 6.49-6.54 ms per 64 x 1080p step
// (profiles/r4_desc_pf2_ab.txt; three batches ahead, 38 spills: 5.56-5.58 vs
// 5.50-5.51, round 5).  WPE: waves per SIMD the registers are budgeted for
// (PF = 2 at 4: 128 VGPRs, the spills outside the sample loop).
// PARTS = 4 (one image, round 6; 2 and 8 for A/B builds): a keypoint's window
// is split over PARTS groups of one wave by the part of the interior rows (and
// columns) its bins lie in; see "Window parts" below.
template <bool DET, int PF, int WPE, int PARTS = 1>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void
descriptor_kernel(DescArgs A) {
  static_assert(PF == 1 || PF == 2, "one or two sample batches in flight");
  static_assert(PARTS == 1 || ((PARTS == 2 || PARTS == 4 || PARTS == 8) && DET), "window parts: detected keypoints (row table) only");
  constexpr int kKpw = kGrp / PARTS;  // keypoints per wave
  // [qidx][group*8 + parity]
  constexpr int kHistRows = kQBins;
  __shared__ float hist[kHistRows * 64];
  // per-sample hand-off records (see RecT); outside the sample loop the same
  // words hold the sub-batch's keypoint indices and the normalisation scalars
  __shared__ __attribute__((aligned(16))) float rec[kGrp * kRecG];
  // per row: (jlo + 64) | len << 8 (16 bits); DET: (jb << 16) | cum (see the
  // walk below)
  __shared__ typename std::conditional<!DET, unsigned short, int>::type rows_tab[kGrp][kRowsTab];
  constexpr int kLenSh = 8, kLoMask = 0xff;
  int* const sord = reinterpret_cast<int*>(rec);                 // [kGrp] keypoint indices
  float(*const bc)[4] = reinterpret_cast<float(*)[4]>(rec + kGrp);  // [kGrp][4] normalisation scalars
  const int lane = threadIdx.x & 63;
  const int g = lane >> 3, q = lane & 7;
  const int d = kDescW, nb = kDescBins;
  int n = A.img_kp_off[A.batch];
  if (n > A.kp_cap) n = A.kp_cap;
  const ExpConsts ek = A.mc->e;
  const float etab_lane = A.mc->exptab[lane];  // lane j holds 2^(j/64) * A0 (exp32f_v)

  // XCD-aware split (speed only): blocks b and b+8 share an XCD, so XCD x takes
  // one contiguous eighth of the raster-ordered keypoints and its L2 sees the
  // overlapping windows of neighbouring keypoints.
  const int xcd = blockIdx.x & 7, nslot = gridDim.x >> 3, slot = blockIdx.x >> 3;
  //
  // Lane balance (speed only): a wave's sample loop runs to the largest window
  // of its 8 keypoints, so desc_rank_kernel ranks each chunk of kRankChunk
  // consecutive keypoints by window size (perm) and a sub-batch takes 8
  // consecutive ranks of one chunk.  Chunks are aligned to the XCD ranges;
  // sub-batch position p of chunk c is read as p ^ h(c), h a multiplicative
  // hash, so a wave's fixed stride does not keep drawing the same ranks (a
  // per-chunk XOR by c itself repeats every two passes at 16 chunks a pass:
  // 6.31 vs 5.85 ms, the waves alive 72 % of the launch instead of 79 %).
  // Keypoints are independent; only the processing order changes.
  // (PARTS > 1: one image, kKpw keypoints per wave, last first or ranked)
  const int per = ((n + 7) / 8 + kRankChunk - 1) / kRankChunk * kRankChunk;
  const int k0 = PARTS > 1 ? 0 : xcd * per;
  const int kend = PARTS > 1 ? n : min(n, (xcd + 1) * per);
  const int nch = (n + kRankChunk - 1) / kRankChunk;
  const int nsb = PARTS > 1 ? (A.perm ? nch * (kRankChunk / kKpw) : (n + kKpw - 1) / kKpw)
                            : (max(kend - k0, 0) + kRankChunk - 1) / kRankChunk * kSubPerChunk;
  for (int sb = PARTS > 1 ? (int)blockIdx.x : slot; sb < nsb; sb += PARTS > 1 ? (int)gridDim.x : nslot) {
    if constexpr (PARTS > 1) {
      if (A.perm) {
        // largest windows first over the whole launch: sub-batch sb takes ranks
        // kKpw j .. from the top of chunk sb % nch (j = sb / nch)
        const int c = sb % nch, j = sb / nch;
        const int clen = min(kRankChunk, n - c * kRankChunk), r = clen - 1 - (j * kKpw + lane);
        if (lane < kKpw) sord[lane] = r >= 0 ? A.perm[c * kRankChunk + r] : kend;
      } else {
        // unranked: last keypoint first -- within an octave the keypoints come
        // in layer order and a layer's windows are larger than the one before
        const int i = sb * kKpw + lane;
        if (lane < kKpw) sord[lane] = i < kend ? kend - 1 - i : kend;
      }
      wave_sync_d();
    } else {
      const int ch = sb / kSubPerChunk;
      const int pos = (sb % kSubPerChunk) ^ (int)(((unsigned)ch * 0x9E3779B1u) >> (32 - kSubBits));
      const int i = k0 + ch * kRankChunk + pos * kGrp + lane;
      if (lane < kGrp) sord[lane] = i < kend ? (A.perm ? A.perm[i] : i) : kend;
      wave_sync_d();
    }
    const int kslot = g / PARTS;            // this group's keypoint among the wave's kKpw
    const bool lead = g % PARTS == 0;       // the group that normalises and stores it
    // Window parts (PARTS = 2): part hr of a keypoint owns the interior bins
    // with R >> 1 == hr.  A sample reaches them only from base corners Rm in
    // [2 hr - 1, 2 hr + 1] -- rbin in [2 hr - 1, 2 hr + 2), r_rot in
    // [2 hr - 2.5, 2 hr + 0.5) -- so the part walks the samples of that band
    // (slab limits below, ~60 % of the window), in raster order, and masks the
    // corners outside its bins like those outside the interior: each of its
    // bins sums the same samples in the same order as a whole-window walk,
    // and a keypoint's longest chain is ~0.6 of the window's.
    // (PARTS = 4, shipped: part (hr, hc) also halves the columns the same way,
    // ~36 % of the window, chain ~0.36;
    // PARTS = 8: part (rq, hc) owns the row R == rq alone: Rm in {rq - 1, rq},
    // r_rot in [rq - 2.5, rq - 0.5).)
    const int hr = PARTS == 4 ? (g >> 1) & 1 : PARTS == 2 ? g & 1 : 0, hc = PARTS >= 4 ? g & 1 : 0;
    const int rq = PARTS == 8 ? g >> 1 : 0;
    const float rlim_lo = PARTS == 8 ? rq - 2.5f : PARTS > 1 ? 2.f * hr - 2.5f : -2.5f;
    const float rlim_hi = PARTS == 8 ? rq - 0.5f : PARTS > 1 ? 2.f * hr + 0.5f : 2.5f;
    const float clim_lo = PARTS >= 4 ? 2.f * hc - 2.5f : -2.5f, clim_hi = PARTS >= 4 ? 2.f * hc + 0.5f : 2.5f;
    const int k = sord[kslot];
    bool active = k < kend;
    int b = 0, oi = 0, layer = 0;
    sift_keypoint kp{};
    if (active) {
      while (b + 1 < A.batch && A.img_kp_off[b + 1] <= k) ++b;
      kp = A.kpts[k];
      int octave = kp.octave & 255;
      layer = (kp.octave >> 8) & 255;
      octave = octave < 128 ? octave : (-128 | octave);
      oi = octave - A.first_octave;
      if (oi < 0 || oi >= A.L.n_oct || layer > kLayers + 2) {  // CV_Assert, src/sift.cpp:744
        if (q == 0) atomicOr(A.err_flag, 1);
        for (int t = q; t < kDescLen; t += 8) A.desc[(long long)k * kDescLen + t] = 0.f;
        active = false;
      }
    }
    // ---- unpackOctave + calcSIFTDescriptor setup (src/sift.cpp:724-751, 582-592) ----
    int octave = kp.octave & 255;
    octave = octave < 128 ? octave : (-128 | octave);
    const float scale = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
    const float size = kp.size * scale;
    const float ptx = kp.x * scale, pty = kp.y * scale;
    float ori = 360.f - kp.angle;
    if (fabsf(ori - 360.f) < FLT_EPSILON) ori = 0.f;
    const float scl = size * 0.5f;
    const Octave& O = A.L.oct[active ? oi : 0];
    const long long pitch = O.pitch;
    const float2* gimg = A.grad + b * A.L.g_img + O.g_off[active ? layer : 0];
    const int rows = O.rows, cols = O.cols;
    const int px = cv_round(ptx), py = cv_round(pty);
    const int pitch32 = (int)pitch;
    const int ctr_off = min(max(py, 0), rows - 1) * pitch32 + min(max(px, 0), cols - 1);
    float cos_t = cosf_cr(ori * (float)(kCvPi / 180));
    float sin_t = sinf_cr(ori * (float)(kCvPi / 180));
    const float bins_per_rad = nb / 360.f;
    const float exp_scale = -1.f / (d * d * 0.5f);
    const float hist_width = 3.f * scl;
    int radius = cv_round(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    const int diag = (int)sqrt(((double)cols) * cols + ((double)rows) * rows);
    radius = radius < diag ? radius : diag;
    if (DET) radius = min(radius, (kMaxWinRows - 1) / 2);  // a no-op for detected keypoints (<= 40); keeps the table in bounds
    cos_t /= hist_width;
    sin_t /= hist_width;
    const float inv_sin = fabsf(sin_t) < 1e-12f ? 0.f : 1.f / sin_t;
    const float inv_cos = fabsf(cos_t) < 1e-12f ? 0.f : 1.f / cos_t;
    const int D = active ? 2 * radius + 1 : 0;
    const bool table = DET || D <= kMaxWinRows;
    // ---- per-row candidate j-ranges and the sample count ----
    int nsamp = 0;
    if constexpr (DET) {
      // Lane q takes the contiguous rows [r0, r1) (ceil(D / 8) each): per row
      // its candidate j-range [lo, lo + len), then, after a prefix sum of the
      // counts over the group, the entry (jb << 16) | cum with cum = the
      // candidates before the row and jb = lo - cum, so candidate t of the
      // group's raster-ordered list lies in the row whose cum <= t < next cum,
      // at j = t + jb.  Two sentinel entries (cum = 0xffff) follow row D - 1.
      const int rb = (D + 7) >> 3;
      const int r0 = min(q * rb, D), r1 = min(r0 + rb, D);
      int cnt = 0;
      for (int ri = r0; ri < r1; ++ri) {
        const int i = ri - radius;
        int lo = max(-radius, 1 - px), hi = min(radius, cols - 2 - px);  // 0 < px + j < cols-1
        if (!(py + i > 0 && py + i < rows - 1)) hi = lo - 1;
        slab(sin_t, inv_sin, i * cos_t, lo, hi, rlim_lo, rlim_hi);     // r_rot = j*sin_t + i*cos_t
        slab(cos_t, inv_cos, -(i * sin_t), lo, hi, clim_lo, clim_hi);  // c_rot = j*cos_t - i*sin_t
        const int len = hi >= lo ? hi - lo + 1 : 0;
        rows_tab[g][ri] = (int)(((unsigned)lo << 16) | (unsigned)len);  // |lo| <= 40
        cnt += len;
      }
      int incl = cnt;
#pragma unroll
      for (int sh = 1; sh < 8; sh <<= 1) {
        const int y = __shfl_up(incl, sh, 8);
        if (q >= sh) incl += y;
      }
      nsamp = __shfl(incl, 7, 8);  // <= 81 * 81
      int cum = incl - cnt;
      for (int ri = r0; ri < r1; ++ri) {
        const int e = rows_tab[g][ri];
        rows_tab[g][ri] = (int)(((unsigned)((e >> 16) - cum) << 16) | (unsigned)cum);
        cum += e & 0xffff;
      }
      if (q == 7) {
        rows_tab[g][D] = 0xffff;
        rows_tab[g][D + 1] = 0xffff;
      }
    } else if (table) {
      for (int ri = q; ri < D; ri += 8) {
        const int i = ri - radius;
        int lo = max(-radius, 1 - px), hi = min(radius, cols - 2 - px);  // 0 < px + j < cols-1
        if (!(py + i > 0 && py + i < rows - 1)) hi = lo - 1;
        slab(sin_t, inv_sin, i * cos_t, lo, hi);     // r_rot = j*sin_t + i*cos_t
        slab(cos_t, inv_cos, -(i * sin_t), lo, hi);  // c_rot = j*cos_t - i*sin_t
        const int len = hi >= lo ? hi - lo + 1 : 0;
        rows_tab[g][ri] = len ? (lo + 64) | (len << kLenSh) : 0;  // lo in [-40, 40] when len > 0
        nsamp += len;
      }
      nsamp += __shfl_xor(nsamp, 1);
      nsamp += __shfl_xor(nsamp, 2);
      nsamp += __shfl_xor(nsamp, 4);
    } else {
      nsamp = D * D;  // radius > 40 (caller-supplied keypoints): the whole window
    }
    for (int t = 0; t < kHistRows; ++t) hist[t * 64 + lane] = 0.f;
    const int nsq = nsamp - q;  // sample base + q is in range iff base < nsq
    int nmax = nsamp;
    nmax = max(nmax, __shfl_xor(nmax, 8));
    nmax = max(nmax, __shfl_xor(nmax, 16));
    nmax = max(nmax, __shfl_xor(nmax, 32));
    nmax = __builtin_amdgcn_readfirstlane(nmax);  // wave-uniform: scalar loop control
    wave_sync_d();
    // lane q walks candidate samples t = q, q+8, ... in raster order (row ri, offset u)
    int ri = 0, u = q, rlo = -radius, rlen = D;
    // DET: the walk holds t and the table entries of rows ri, ri + 1, ri + 2
    int t = q, e0 = 0, e1 = 0, e2 = 0;
    if constexpr (DET) {
      e0 = rows_tab[g][0];
      e1 = rows_tab[g][1];
      while (t >= (e1 & 0xffff)) {  // stops at the sentinel (row D) at the latest
        ++ri;
        e0 = e1;
        e1 = rows_tab[g][ri + 1];
      }
      e2 = rows_tab[g][ri + 2];
      rlen = 0;  // unused
    } else if (table && D > 0) {
      const int e = rows_tab[g][0];
      rlo = (e & kLoMask) - 64;
      rlen = e >> kLenSh;
    }
    while (!DET && ri < D && u >= rlen) {
      u -= rlen;
      if (++ri < D && table) {
        const int e = rows_tab[g][ri];
        rlo = (e & kLoMask) - 64;
        rlen = e >> kLenSh;
      }
    }
    // Software pipeline: each step stashes batch k, then computes batch k+1
    // (independent VALU + one gather) in the same basic block as batch k's
    // ordered LDS read-modify-write chain, so the scheduler fills the chain's
    // LDS latency with the next batch's arithmetic.  Both halves are
    // branch-free: an invalid sample hands every owner "+0.0f into your bin 0"
    // (exact no-op, every bin is >= +0) and gathers from a clamped address.
    //
    // The sample's lane resolves ownership for all 8 owners: with
    // (Rm, Cm, O0) = (r0, c0, o0) (interior coordinates, R' = R - 1) and odd =
    // their parity bits, corner k = dr*4 + dc*2 + do lands in interior bin
    // (Rm+dr, Cm+dc, O0+do), whose parity -- its owner -- is k ^ odd, at
    //   qidx_k = qi0 + [dr and Rm odd]*10 + [dc and Cm odd]*5 + [do and O0 odd],
    // or outside the interior when Rm+dr or Cm+dc leaves [0, 4) (value +0.0).
    // The record (qidx_k, value_k) is stored straight into owner slot k ^ odd;
    // the owner adds its lane to form the [qidx][lane] address.
    RecT rc_cur;  // (qidx, val) x 8 corners of this lane's sample
    // locate: the sample at the walk position, its gather (in flight until
    // finish uses it) and the parts of its record that do not need the pixel
    // (weight, spatial bins); finish: the rest.
    struct Loc {
      float w, rbin, cbin;  // Gaussian weight; fractional spatial bin parts
      int X, Y;             // base corner + 1: X = Rm + 1 = cvFloor(rbin) + 1 in [0, d] (1 for an invalid sample)
      float2 mo_raw;
      bool ok;
    };
    auto locate = [&](bool in_range, Loc& L) {
      const int i = ri - radius, j = DET ? t + (e0 >> 16) : rlo + u;
      const float c_rot = j * cos_t - i * sin_t;
      const float r_rot = j * sin_t + i * cos_t;
      float rbin = r_rot + d / 2 - 0.5f;
      float cbin = c_rot + d / 2 - 0.5f;
      const int r = py + i, c = px + j;
      // cvFloor: |rbin|, |cbin| < 10, so floorf is exact and (int)floorf ==
      // cvFloor; rbin - floorf(rbin) == rbin - (float)r0
      const float fr = floorf(rbin), fc = floorf(cbin);
      const int xr = (int)fr + 1, yc = (int)fc + 1;
      // the row table enumerates interior pixels only (src/sift.cpp:620-621's
      // 0 < r < rows-1, 0 < c < cols-1), so only the whole-window walk tests them.
      // DET tests rbin, cbin in (-1, d) as cvFloor in [-1, d - 1]: that admits
      // rbin (cbin) == -1.0 exactly, a sample whose every corner value is +0.0
      // (the R = -1 corners are masked, the R = 0 ones carry mag * 0), an
      // exact no-op; two integer compares instead of four float ones
      if constexpr (DET)
        L.ok = in_range && (unsigned)xr <= (unsigned)d && (unsigned)yc <= (unsigned)d;
      else
        L.ok = in_range && rbin > -1 && rbin < d && cbin > -1 && cbin < d &&
               (table || (r > 0 && r < rows - 1 && c > 0 && c < cols - 1));
      // an invalid sample gathers from the clamped keypoint centre (any valid
      // address: its value is replaced below); plane offsets fit 32 bits
      int pix = __mul24(r, pitch32) + c;
      if constexpr (DET) asm volatile("" : "+v"(pix));  // computed on every lane: a select, not a branch
      L.mo_raw = gimg[(unsigned)(L.ok ? pix : ctr_off)];  // (Mag, Ori) of the pixel
      L.w = exp32f_v<false>((c_rot * c_rot + r_rot * r_rot) * exp_scale, etab_lane, ek);
      L.rbin = rbin - fr;
      L.cbin = cbin - fc;
      // the base corner R0 = r0 + 1 = X in [0, d] (interior coordinate Rm =
      // X - 1 in [-1, 3]); an invalid sample's values are all +0.0, so any
      // base corner serves it: DET clamps, which keeps the perm-table
      // selectors in range without waiting for ok
      L.X = DET ? min(max(xr, 0), d) : L.ok ? xr : 1;
      L.Y = DET ? min(max(yc, 0), d) : L.ok ? yc : 1;
    };
    auto finish = [&](const Loc& L, RecT& out, int& odd_out) {
      const float rbin = L.rbin, cbin = L.cbin;
      const bool ok = L.ok;
      // An invalid sample must add +0.0 everywhere.  Caller keypoints: its
      // pixel is (0, 0) -- it gathered the clamped centre, and border
      // gradients are never written and may hold NaN.  Detected keypoints
      // (DET) lie >= SIFT_IMG_BORDER inside the image, so the centre's
      // gradient is finite and a zero weight alone makes mag = +0 (one select
      // instead of two); lanes of an inactive group may sum NaN into their
      // own histogram, which is never stored.
      const float2 mo = DET || ok ? L.mo_raw : make_float2(0.f, 0.f);
      float obin = (mo.y - ori) * bins_per_rad;
      const float mag = mo.x * (!DET || ok ? L.w : 0.f);
      const float fo = floorf(obin);  // |obin| < 10: exact, as above
      int o0 = (int)fo;
      obin -= fo;
      int O0;
      if constexpr (DET) {
        // Ori in [0, 360] and ori in [0, 360) put obin in (-8, 8], so o0 in
        // [-8, 8], where the two wraps below are o0 & 7 (nb = 8); an invalid
        // sample's o0 is any bin (its values are +0.0)
        static_assert(kDescBins == 8, "o0 & 7 is the wrap for 8 bins");
        O0 = o0 & 7;
      } else {
        if (o0 < 0) o0 += nb;
        if (o0 >= nb) o0 -= nb;
        O0 = ok ? o0 : 0;
      }
      const int X = L.X, Y = L.Y, Rm = X - 1, Cm = Y - 1;  // Rm, Cm: the unpacked form only
      const int odd = ((Rm & 1) << 2) | ((Cm & 1) << 1) | (O0 & 1);
      float v_r1 = mag * rbin, v_r0 = mag - v_r1;
      // corners outside the interior rows carry +0.0 (added to some interior
      // bin: an exact no-op, every bin is >= +0) instead of going to a trash
      // bin; each weight is masked after every product that uses its
      // unmasked value, so the interior corners' values are unchanged
      // (PARTS > 1: outside the part's rows R in {2 hr, 2 hr + 1} -- the corner
      // R = Rm = X - 1 for dr = 0, R = X for dr = 1 -- and columns likewise)
      const bool r0_in = PARTS == 8 ? X == rq + 1 : PARTS > 1 ? (unsigned)(X - 2 * hr - 1) <= 1u : X >= 1;  // Rm >= 0
      const bool r1_in = PARTS == 8 ? X == rq : PARTS > 1 ? (unsigned)(X - 2 * hr) <= 1u : X <= 3;          // Rm <= 2
      const bool c0_in = PARTS >= 4 ? (unsigned)(Y - 2 * hc - 1) <= 1u : Y >= 1;
      const bool c1_in = PARTS >= 4 ? (unsigned)(Y - 2 * hc) <= 1u : Y <= 3;
      v_r0 = r0_in ? v_r0 : 0.f;
      v_r1 = r1_in ? v_r1 : 0.f;
      float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
      float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
      // and outside the interior columns
      v_rc00 = c0_in ? v_rc00 : 0.f;
      v_rc10 = c0_in ? v_rc10 : 0.f;
      v_rc01 = c1_in ? v_rc01 : 0.f;
      v_rc11 = c1_in ? v_rc11 : 0.f;
      float v[8];
      v[7] = v_rc11 * obin;  // corner index = dr*4 + dc*2 + do, src/sift.cpp:659-672
      v[6] = v_rc11 - v[7];
      v[5] = v_rc10 * obin;
      v[4] = v_rc10 - v[5];
      v[3] = v_rc01 * obin;
      v[2] = v_rc01 - v[3];
      v[1] = v_rc00 * obin;
      v[0] = v_rc00 - v[1];
      {
#pragma unroll
        for (int k = 0; k < 8; ++k) out.v[k] = v[k];
        // bin bytes in owner-slot order: byte s (word s >> 2) is the qidx of
        // corner k = s ^ odd, whose R = Rm + (s2 ^ (Rm & 1)) is even for s2 = 0
        // and odd for s2 = 1 (likewise C with s1, O with s0), so
        //   qidx = Rpart[s2] + Cpart[s1] + Opart[s0]
        // with (x = Rm + 1, y = Cm + 1 in [0, 4]) Rpart[0] = T_R[x + 1],
        // Rpart[1] = T_R[x], T_R = {0, 0, 0, 10, 10, 10}; Cpart likewise from
        // T_C = {0, 0, 0, 5, 5, 5}; Opart[0] = (O0 + 1) >> 1, Opart[1] = O0 >> 1.
        // The tables are byte lookups (v_perm_b32 over the 8-byte table);
        // their entries for a row / column outside the interior are arbitrary
        // interior bins (those corners carry +0.0, above).
        // (byte replication by v_perm_b32 with selector 0)
        const unsigned x = (unsigned)X, y = (unsigned)Y;
        const unsigned selR1 = __builtin_amdgcn_perm(0u, x, 0u), selR0 = selR1 + 0x01010101u;
        const unsigned selC = __builtin_amdgcn_perm(0u, y, 0u) + 0x00000101u;
        const unsigned po = (unsigned)(O0 & 1);
        const unsigned o4 = __builtin_amdgcn_perm(0u, (unsigned)(O0 >> 1), 0u) + (po | (po << 16));
        const unsigned c4 = __builtin_amdgcn_perm(0x00000505u, 0x05000000u, selC) + o4;
        out.qb[0] = __builtin_amdgcn_perm(0x00000a0au, 0x0a000000u, selR0) + c4;
        out.qb[1] = __builtin_amdgcn_perm(0x00000a0au, 0x0a000000u, selR1) + c4;
      }
      // the slot bits of the hand-off store address from the parities of X =
      // Rm + 1 and Y = Cm + 1 -- (odd ^ 6) << 7, i.e. slot s is stored at
      // position s ^ 6 (the owner reads there) -- by shift-and-or steps
      (void)odd;
      odd_out = ((X << 9) & 0x200) | ((Y << 8) & 0x100) | ((O0 & 1) << 7);
    };
    auto sample = [&](bool in_range, RecT& out, int& odd_out) {
      Loc L;
      locate(in_range, L);
      finish(L, out, odd_out);
    };
    // Entry ri+1 of the row table rides in a register (loaded one advance
    // ahead), so the common advance -- at most one row change -- is
    // branch-free selects with no LDS round trip; short or empty rows fall
    // back to the row walk under a wave-uniform branch.
    // Caller keypoints may have D > kMaxWinRows (no table, the value is
    // unused): clamped.
    auto next_entry = [&]() { return rows_tab[g][min(ri + 1, kRowsTab - 1)]; };
    int enext = DET ? 0 : next_entry();
    auto advance = [&]() {  // to candidate sample t + 8
      if constexpr (DET) {
        // entries e1, e2 of rows ri + 1, ri + 2 were loaded an advance ahead:
        // a move by one row is compares and selects; rows shorter than 8 take
        // the loop (the sentinel after row D - 1 ends it)
        t += 8;
        const bool mv = t >= (e1 & 0xffff);
        ri += mv ? 1 : 0;
        e0 = mv ? e1 : e0;
        e1 = mv ? e2 : e1;
        while (t >= (e1 & 0xffff)) {
          ++ri;
          e0 = e1;
          e1 = rows_tab[g][ri + 1];
        }
        e2 = rows_tab[g][ri + 2];  // ri <= D - 1: within the table
      } else {
        u += 8;
        const bool mv = ri < D && u >= rlen;
        u = mv ? u - rlen : u;
        ri = mv ? ri + 1 : ri;
        if (table) {
          rlo = mv ? (enext & kLoMask) - 64 : rlo;
          rlen = mv ? enext >> kLenSh : rlen;
        }
        while (ri < D && u >= rlen) {  // skipped by exec when no lane needs it
          u -= rlen;
          if (++ri < D && table) {
            const int e = rows_tab[g][ri];
            rlo = (e & kLoMask) - 64;
            rlen = e >> kLenSh;
          }
        }
        enext = next_entry();
      }
    };
    int odd_cur = 0;
    uint2 qq_cur = make_uint2(0u, 0u);  // this owner's 8 bin bytes of the batch
    Loc loc_nxt, loc_alt;  // PF = 2: batches k + 1 and k + 2, located and gathering (two buffers)
    if (nmax > 0) {
      if constexpr (PF == 2) {
        Loc l0;
        locate(0 < nsq, l0);
        advance();
        locate(8 < nsq, loc_nxt);
        advance();
        finish(l0, rc_cur, odd_cur);
      } else {
        sample(0 < nsq, rc_cur, odd_cur);
        advance();
      }
    }
    // one batch: ln = batch k + 1 (PF = 2; located a step ago), l2 = the batch
    // located in this step
    auto step = [&](int base, Loc& ln, Loc& l2) {
      {
        // corner k to owner slot s = k ^ odd: value at byte
        //   ((g >> 2) << 10) | ((s ^ 6) << 7) | ((g & 3) << 5) | (q << 2).
        // A ds_write_b32 banks on (a / 4) mod 32 per 32-lane half (MI355X:
        // LDS table), i.e. on byte bits 2-6 = (q, g & 3): one store
        // instruction's 64 lanes hit 32 distinct banks per half whatever the
        // data-dependent slots -- conflict free.  (Round 2-5's layout, with the
        // slot bits at 5-7, left two of them in the store's bank and put 4
        // lanes of random slots on each bank column: 47.4 instead of 16
        // LDS-array cycles per batch's eight stores, simulated; the 0.34 of
        // SQ_LDS_IDX_ACTIVE that SQ_LDS_BANK_CONFLICT measured.)  The owner's
        // ds_read_b128 (16-lane groups, (a / 4) mod 64) see bits 4-7 = (half,
        // g & 3, s & 1): 2-way, 16 instead of 8 cycles per batch.  No layout
        // makes both conflict free: data-independent store banks leave the
        // reads only bit 7 for the slot.  Slot bits are clear in the base, so
        // each store address is one XOR with k's slot bits, as before.
        char* rb = reinterpret_cast<char*>(rec);
        const int wv = (((g >> 2) << 10) | ((g & 3) << 5) | (q << 2)) | odd_cur;  // odd_cur = (odd ^ 6) << 7
#pragma unroll
        for (int k = 0; k < 8; ++k) *reinterpret_cast<float*>(rb + (wv ^ (k << 7))) = rc_cur.v[k];
        // bin bytes to their owners in registers (round 4; were eight
        // ds_write_b8 per lane and one ds_read_b64): byte s of this lane's
        // pair is corner s ^ odd's (finish), then an 8 x 8 byte transpose over the group's
        // lanes (lane bit b <-> byte bit b: DPP row shifts by 4, quad perms,
        // v_perm_b32), so owner s holds sample q's bin byte at byte q
        {
          unsigned w0 = rc_cur.qb[0], w1 = rc_cur.qb[1];
          const unsigned a = (unsigned)__builtin_amdgcn_mov_dpp((int)w0, 0x104, 0xf, 0xf, true);  // lane + 4
          const unsigned c = (unsigned)__builtin_amdgcn_mov_dpp((int)w1, 0x114, 0xf, 0xf, true);  // lane - 4
          if (q & 4)
            w0 = c;
          else
            w1 = a;
          const unsigned s2 = (q & 2) ? 0x03020706u : 0x05040100u;
          unsigned p0 = (unsigned)__builtin_amdgcn_mov_dpp((int)w0, 0x4E, 0xf, 0xf, true);  // lane ^ 2
          unsigned p1 = (unsigned)__builtin_amdgcn_mov_dpp((int)w1, 0x4E, 0xf, 0xf, true);
          w0 = __builtin_amdgcn_perm(p0, w0, s2);
          w1 = __builtin_amdgcn_perm(p1, w1, s2);
          const unsigned s1 = (q & 1) ? 0x03070105u : 0x06020400u;
          p0 = (unsigned)__builtin_amdgcn_mov_dpp((int)w0, 0xB1, 0xf, 0xf, true);  // lane ^ 1
          p1 = (unsigned)__builtin_amdgcn_mov_dpp((int)w1, 0xB1, 0xf, 0xf, true);
          qq_cur = make_uint2(__builtin_amdgcn_perm(p0, w0, s1), __builtin_amdgcn_perm(p1, w1, s1));
        }
      }
      wave_sync_d();
      RecT rc_nxt;
      int odd_nxt = 0;
      if constexpr (PF == 2) {
        locate(base + 16 < nsq, l2);  // batch k + 2: its gather flies for two steps
        advance();
        finish(ln, rc_nxt, odd_nxt);
      } else {
        locate(base + 8 < nsq, l2);  // batch k + 1: finished after this batch's chain
      }
      // ordered accumulation of batch k: lane q applies its record of each sample
      {
        const char* rb = reinterpret_cast<const char*>(rec);
        // slot q at position q ^ 6 (finish's odd_out); samples 0-3, then 4-7 (bit 4)
        const int rv = ((g >> 2) << 10) | ((q ^ 6) << 7) | ((g & 3) << 5);
        const float4 va = *reinterpret_cast<const float4*>(rb + rv);
        const float4 vb = *reinterpret_cast<const float4*>(rb + (rv | 16));
        const uint2 qq = qq_cur;
        const float vals[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
        // byte address qidx * 256 + lane * 4 in one v_perm_b32: byte 0 <- lane * 4
        // (< 256), byte 1 <- the bin byte, bytes 2-3 <- 0 (selector 12)
        const unsigned lane4 = (unsigned)lane << 2;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const unsigned ab = __builtin_amdgcn_perm(lane4, jj < 4 ? qq.x : qq.y, 0x0c0c0004u | ((unsigned)(jj & 3) << 8));
          float* hp = reinterpret_cast<float*>(reinterpret_cast<char*>(hist) + ab);
          *hp = *hp + vals[jj];
        }
      }
      if constexpr (PF == 1) {
        // batch k + 1's gathered pixel is first used after the chain (an
        // opaque copy behind the chain's LDS operations): its memory latency
        // overlaps the chain whatever order the scheduler picks
        asm volatile("" : "+v"(l2.mo_raw.x), "+v"(l2.mo_raw.y) : : "memory");
        finish(l2, rc_nxt, odd_nxt);
      }
      wave_sync_d();
      if constexpr (PF == 1) advance();
      rc_cur = rc_nxt;
      odd_cur = odd_nxt;
    };
    if constexpr (PF == 2) {
      // unrolled by two so the two Loc buffers swap roles instead of being
      // copied (a copy of the gathered pixel would wait for its load)
      for (int base = 0; base < nmax; base += 16) {
        step(base, loc_nxt, loc_alt);
        if (base + 8 >= nmax) break;
        step(base + 8, loc_alt, loc_nxt);
      }
    } else {
      for (int base = 0; base < nmax; base += 8) step(base, loc_nxt, loc_alt);
    }
    // ---- fold (src/sift.cpp:676-684): read the 16 cells' bins, then write the 128 ----
    float* dv = hist + kslot * (kDescLen + 4);  // the 128-vector reuses histogram storage
    if constexpr (PARTS > 1) {
      // a part's 4 (PARTS = 8: 2) cells: lane q takes one cell and NO = 4 (2)
      // of its orientations, the first of them adding the two wrap bins
      // (PARTS = 2: 8 cells, lane q takes cell q whole)
      constexpr int NO = PARTS == 8 ? 2 : PARTS == 4 ? 4 : 8;
      const int R = PARTS == 8 ? rq : PARTS == 4 ? 2 * hr + ((q >> 2) & 1) : 2 * hr + (q >> 2);
      const int C = PARTS == 8 ? 2 * hc + ((q >> 2) & 1) : PARTS == 4 ? 2 * hc + ((q >> 1) & 1) : q & 3;
      const int oh = PARTS == 8 ? q & 3 : PARTS == 4 ? q & 1 : 0;
      float cl[NO];
#pragma unroll
      for (int u = 0; u < NO; ++u) {
        const int o = NO * oh + u;
        const int par = ((R & 1) << 2) | ((C & 1) << 1) | (o & 1);
        cl[u] = hist[((R >> 1) * 10 + (C >> 1) * 5 + (o >> 1)) * 64 + g * 8 + par];
      }
      if (oh == 0) {
#pragma unroll
        for (int o = nb; o < nb + 2; ++o) {
          const int par = ((R & 1) << 2) | ((C & 1) << 1) | (o & 1);
          cl[o - nb] = cl[o - nb] + hist[((R >> 1) * 10 + (C >> 1) * 5 + (o >> 1)) * 64 + g * 8 + par];
        }
      }
      wave_sync_d();
#pragma unroll
      for (int u = 0; u < NO; ++u) dv[(R * d + C) * nb + NO * oh + u] = cl[u];
    } else {
      float cell[2][8];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int cidx = q + 8 * h2;
        const int R = cidx / d, C = cidx % d;  // interior coordinates R' = R-1, C' = C-1
#pragma unroll
        for (int o = 0; o < nb + 2; ++o) {
          const int par = ((R & 1) << 2) | ((C & 1) << 1) | (o & 1);
          const float hv = hist[((R >> 1) * 10 + (C >> 1) * 5 + (o >> 1)) * 64 + g * 8 + par];
          if (o < nb)
            cell[h2][o] = hv;
          else
            cell[h2][o - nb] = cell[h2][o - nb] + hv;
        }
      }
      wave_sync_d();
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
        for (int t = 0; t < nb; ++t) dv[(q + 8 * h2) * nb + t] = cell[h2][t];
    }
    wave_sync_d();
    // ---- hysteresis + quantisation + RootSIFT (src/sift.cpp:689-721) ----
    if (q == 0 && lead) {
      float nrm2 = 0;
      for (int t = 0; t < kDescLen; ++t) nrm2 = nrm2 + dv[t] * dv[t];
      bc[kslot][0] = sqrtf(nrm2) * 0.2f;
    }
    wave_sync_d();
    const float thr = bc[kslot][0];
    if (lead)
      for (int t = q; t < kDescLen; t += 8) dv[t] = dv[t] < thr ? dv[t] : thr;
    wave_sync_d();
    if (q == 0 && lead) {
      float nrm2 = 0;
      for (int t = 0; t < kDescLen; ++t) nrm2 = nrm2 + dv[t] * dv[t];
      const float sq = sqrtf(nrm2);
      bc[kslot][1] = 512.f / (sq < FLT_EPSILON ? FLT_EPSILON : sq);
    }
    wave_sync_d();
    const float nrm2s = bc[kslot][1];
    if (lead)
      for (int t = q; t < kDescLen; t += 8) dv[t] = sat_u8(dv[t] * nrm2s) * nrm2s;
    wave_sync_d();
    if (q == 0 && lead) {
      float nrm1 = 0;
      for (int t = 0; t < kDescLen; ++t) nrm1 = nrm1 + dv[t];
      bc[kslot][2] = 1.f / (nrm1 < FLT_EPSILON ? FLT_EPSILON : nrm1);
    }
    wave_sync_d();
    const float nrm1 = bc[kslot][2];
    if (active && lead) {
      float4* out = reinterpret_cast<float4*>(A.desc + (long long)k * kDescLen) + q * 4;
      const float4* src = reinterpret_cast<const float4*>(dv) + q * 4;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 x = src[t];
        out[t] = make_float4(sqrtf(x.x * nrm1), sqrtf(x.y * nrm1), sqrtf(x.z * nrm1), sqrtf(x.w * nrm1));
      }
    }
    wave_sync_d();
  }
}

// Lane-balance ranking for descriptor_kernel (speed only): chunk c of
// kRankChunk consecutive keypoints -> perm[c kRankChunk + rank] = index, ranked
// by the window size size * 2^-octave (positive floats order as their bits;
// ties by index).
__global__ __launch_bounds__(kRankChunk) void desc_rank_kernel(const sift_keypoint* __restrict__ kpts,
                                                               const int* __restrict__ img_kp_off, int batch,
                                                               int kp_cap, int* __restrict__ perm) {
  __shared__ __attribute__((aligned(16))) int keys[kRankChunk];
  int n = img_kp_off[batch];
  if (n > kp_cap) n = kp_cap;
  const int t = threadIdx.x;
  for (int c0 = blockIdx.x * kRankChunk; c0 < n; c0 += gridDim.x * kRankChunk) {
    const int i = c0 + t;
    int key = 0x7fffffff;
    if (i < n) {
      int oc = kpts[i].octave & 255;
      oc = oc < 128 ? oc : (-128 | oc);
      const float sc = oc >= 0 ? 1.f / (1 << (oc & 31)) : (float)(1 << ((-oc) & 31));
#ifdef SIFT_DESC_RANK_RADIUS
      key = min(max(cv_round(kpts[i].size * sc * 1.5f * 1.4142135623730951f * (kDescW + 1) * 0.5f), 0), 0xffffff);
#else
      key = __float_as_int(fabsf(kpts[i].size * sc));
#endif
    }
    __syncthreads();
    keys[t] = key;
    __syncthreads();
    // four keys per (broadcast) LDS read, unrolled so the reads pipeline
    int rank = 0;
#pragma unroll 8
    for (int u = 0; u < kRankChunk; u += 4) {
      const int4 k4 = *reinterpret_cast<const int4*>(&keys[u]);
      rank += k4.x < key || (k4.x == key && u < t) ? 1 : 0;
      rank += k4.y < key || (k4.y == key && u + 1 < t) ? 1 : 0;
      rank += k4.z < key || (k4.z == key && u + 2 < t) ? 1 : 0;
      rank += k4.w < key || (k4.w == key && u + 3 < t) ? 1 : 0;
    }
    if (i < n) perm[c0 + rank] = i;
  }
}

// Element-wise evaluation of the device helpers (sift_selftest_math).
__global__ __launch_bounds__(256) void math_selftest_kernel(int op, const float* __restrict__ a,
                                                            const float* __restrict__ b,
                                                            float* __restrict__ out, int n,
                                                            const MathConsts* __restrict__ mc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = a[i];
  float r = 0.f;
  switch (op) {
    case 0: r = exp32f(x, mc->exptab, mc->e); break;
    case 1: r = fast_atan2(x, b[i], mc->t); break;
    case 2: r = magnitude(x, b[i]); break;
    case 3: r = cosf_cr(x); break;
    case 4: r = sinf_cr(x); break;
    case 5: r = pow2f_cr(x); break;
    case 6: r = (float)cv_round(x); break;
    default: r = (float)cv_floor(x); break;
  }
  out[i] = r;
}

void launch_math_selftest(hipStream_t st, int op, const float* a, const float* b, float* out, int n,
                          const MathConsts* mc) {
  hipLaunchKernelGGL(math_selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, st, op, a, b, out, n,
                     mc);
}

void launch_descriptors(hipStream_t st, const Layout& L, const float2* grad, const MathConsts* mc,
                        const sift_keypoint* kpts, const int* img_kp_off, int batch, int kp_cap,
                        float* desc, int first_octave, int* err_flag, bool detected, int* perm) {
  if (kp_cap <= 0) return;
  // One image of up to kOneImagePx splits each window over PARTS groups (row
  // and column halves) and takes its keypoints last first (a layer's windows
  // are larger than the previous layer's), no ranking pass (8.4 us per 1080p
  // image): round 6, configs[1]'s descriptor 281 us whole-window (groups of 8,
  // own order); resident grids: 207 with 4 parts, 197 + 8 ranked largest
  // first, 182-192 + 8 with 2 parts ranked, 194 with 2 parts last first (217
  // first first), 8 parts 238-262 (1.9 x the samples); capacity grids (below):
  // 2 parts 191, 4 parts 184, 8 parts 220; profiles/r6_desc_one_image_ab.txt.
#ifndef SIFT_DESC_ONE_RANK
#define SIFT_DESC_ONE_RANK 0  // A/B builds only: 1 = rank one image too (largest first)
#endif
  const bool rank = !(detected && one_image_variants(L, batch)) || SIFT_DESC_ONE_RANK;
  if (rank)
    hipLaunchKernelGGL(desc_rank_kernel, dim3(std::min((kp_cap + kRankChunk - 1) / kRankChunk, 4096)),
                       dim3(kRankChunk), 0, st, kpts, img_kp_off, batch, kp_cap, perm);
  DescArgs A;
  A.perm = rank ? perm : nullptr;
  A.L = L;
  A.grad = grad;
  A.mc = mc;
  A.kpts = kpts;
  A.img_kp_off = img_kp_off;
  A.batch = batch;
  A.kp_cap = kp_cap;
  A.desc = desc;
  A.first_octave = first_octave;
  A.err_flag = err_flag;
  // detected keypoints gather two batches ahead (PF = 2): one image of up to
  // kOneImagePx (one_image_variants) in window parts at 4 waves per SIMD
  // (2: 223 vs 197 us ranked with 4 parts), batches and larger images whole
  // at kDescWpe;
  // caller keypoints (calDescriptor: any radius, the whole-window walk) run
  // the general form one batch ahead
#ifndef SIFT_DESC_GRID_PCT
#define SIFT_DESC_GRID_PCT 100  // A/B builds only (tools/build_var.sh): the grid as a share of the resident one
#endif
#define SIFT_DESC_LAUNCH(...)                                                                                       \
  hipLaunchKernelGGL((descriptor_kernel<__VA_ARGS__>),                                                              \
                     dim3(std::max(8, resident_grid((const void*)descriptor_kernel<__VA_ARGS__>, 64, 0, 8192) *     \
                                          SIFT_DESC_GRID_PCT / 800 * 8)),                                           \
                     dim3(64), 0, st, A)
#ifndef SIFT_ONE_BIG_GRIDS
#define SIFT_ONE_BIG_GRIDS 4  // A/B builds only (tools/build_var.sh); one 8K image: 1 1994 us, 4 1850, 16 1877 (round 6)
#endif
#ifndef SIFT_DESC_ONE_GRID
#define SIFT_DESC_ONE_GRID 1  // A/B builds only (tools/build_var.sh): 0 = the resident grid
#endif
#ifndef SIFT_DESC_ONE_PARTS
#define SIFT_DESC_ONE_PARTS 4  // A/B builds only (tools/build_var.sh): 1 = whole windows, 2, 4, 8 parts
#endif
  if (detected && one_image_variants(L, batch) && SIFT_DESC_ONE_GRID)
    // a workgroup per sub-batch of the capacity (waves past the keypoint count
    // exit at once): the dispatcher hands the next sub-batch to whichever wave
    // slot frees first, as for the one-image orientation (192 vs 201 us per
    // 1080p image, round 6)
    // (at most 4 resident grids: a large capacity does not launch empty waves
    // without bound; the kernel strides past its grid)
    hipLaunchKernelGGL((descriptor_kernel<true, 2, kDescWpe, SIFT_DESC_ONE_PARTS>),
                       dim3(std::min((kp_cap + kGrp / SIFT_DESC_ONE_PARTS - 1) / (kGrp / SIFT_DESC_ONE_PARTS),
                                     4 * resident_grid((const void*)descriptor_kernel<true, 2, kDescWpe, SIFT_DESC_ONE_PARTS>,
                                                       64, 0, 8192))),
                       dim3(64), 0, st, A);
  else if (detected && one_image_variants(L, batch))
    SIFT_DESC_LAUNCH(true, 2, kDescWpe, SIFT_DESC_ONE_PARTS);
  else if (detected && batch == 1)
    // one image above kOneImagePx: several resident grids, so that the slots
    // that finish early take the remaining strides (the XCD mapping above
    // works for any grid of whole XCD runs)
    hipLaunchKernelGGL((descriptor_kernel<true, 2, kDescWpe>),
                       dim3(resident_grid((const void*)descriptor_kernel<true, 2, kDescWpe>, 64, 0, 8192) *
                            SIFT_ONE_BIG_GRIDS),
                       dim3(64), 0, st, A);
  else if (detected)
    SIFT_DESC_LAUNCH(true, 2, kDescWpe);
  else
    SIFT_DESC_LAUNCH(false, 1, kDescWpe);
#undef SIFT_DESC_LAUNCH
}

}  // namespace sift
