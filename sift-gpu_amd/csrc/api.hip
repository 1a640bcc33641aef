// api.hip -- the C ABI (include/sift_hip.h): context, device workspace,
// pipeline orchestration on one HIP stream, sub-module entry points and
// per-stage HIP-event profiling.  Host code only; kernels live in blur.hip,
// detect.hip and descriptor.hip.
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"

namespace sift {

Layout make_layout(int rows, int cols, int n_oct) {
  Layout L;
  memset(&L, 0, sizeof(L));
  L.n_oct = n_oct;
  L.rows = rows;
  L.cols = cols;
  long long g = 0, d = 0;
  int r = rows, c = cols;
  for (int o = 0; o < n_oct; ++o) {
    Octave& O = L.oct[o];
    O.rows = r;
    O.cols = c;
    O.pitch = round_up(c > 0 ? c : 1, kPitchAlign);
    const long long plane = (long long)O.rows * O.pitch;
    for (int s = 0; s < kScales; ++s) O.g_off[s] = g + s * plane;
    for (int s = 0; s < kDogPer; ++s) O.d_off[s] = d + s * plane;
    g += kScales * plane;
    d += kDogPer * plane;
    r /= 2;  // Size(src.cols/2, src.rows/2), src/sift.cpp:254
    c /= 2;
  }
  L.g_img = g;
  L.d_img = d;
  return L;
}

int resident_grid(const void* kernel, int block, size_t lds, int fixed_grid) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fixed_grid;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(kernel, dev);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1 ||
      cus < 1)
    return fixed_grid;
  const int g = std::max(8, per_cu * cus / 8 * 8);
  cache[key] = g;
  return g;
}

void host_math_consts(MathConsts* mc) {
  const double A0 = .9670371139572337719125840413672004409288e-2;
  const double prescale = 1.4426950408889634073599246810019 * 64;
  const double maxval = 3000. * 64;
  mc->e.A4 = (float)(1.000000000000002438532970795181890933776 / A0);
  mc->e.A3 = (float)(.6931471805521448196800669615864773144641 / A0);
  mc->e.A2 = (float)(.2402265109513301490103372422686535526573 / A0);
  mc->e.A1 = (float)(.5550339366753125211915322047004666939128e-1 / A0);
  mc->e.lo = (float)(-maxval / prescale);
  mc->e.hi = (float)(maxval / prescale);
  mc->e.post = (float)(1. / 64);
  mc->e.prescale = (float)prescale;
  for (int j = 0; j < 64; ++j) mc->exptab[j] = (float)((double)exp2l((long double)j / 64.0L) * A0);
  const float deg = (float)(180 / kCvPi);
  mc->t.p1 = 0.9997878412794807f * deg;
  mc->t.p3 = -0.3258083974640975f * deg;
  mc->t.p5 = 0.1555786518463281f * deg;
  mc->t.p7 = -0.04432655554792128f * deg;
  mc->t.eps = (float)DBL_EPSILON;
}

}  // namespace sift

using namespace sift;

namespace {

struct StageRec {
  int stage;
  hipEvent_t a, b;
  double flops, bytes;
};

const char* const kStageNames[] = {"blur_base", "blur_octave", "decimate", "dog", "extrema",
                                   "refine_orient", "emit", "descriptor", "upload", "download",
                                   "blur_1d", "pyramid_fast", "match", "blur_octave_sym"};
enum Stage { ST_BLUR_BASE, ST_BLUR_OCT, ST_DECIMATE, ST_DOG, ST_EXTREMA, ST_REFINE, ST_EMIT,
             ST_DESC, ST_UPLOAD, ST_DOWNLOAD, ST_BLUR1D, ST_PYR_FAST, ST_MATCH, ST_BLUR_SYM, ST_N };

template <typename T>
hipError_t dmalloc(T** p, size_t count) {
  return hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (count ? count : 1));
}

}  // namespace

struct sift_ctx {
  int device = 0;
  unsigned flags = 0;
  int n_oct = 5;
  int max_rows = 0, max_cols = 0, max_batch = 0, max_oct = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  // workspace
  float* d_in = nullptr;
  long long in_pitch = 0, in_img = 0;
  float* d_gpyr = nullptr;
  float* d_dog = nullptr;
  float* d_tmp = nullptr;
  float2* d_grad = nullptr;       // per-pixel (magnitude, orientation), gpyr layout
  long long gpyr_elems = 0, dog_elems = 0;
  float* d_coef = nullptr;        // base (w=4) then the 4 octave scales
  float* d_coef_gen = nullptr;    // per-call coefficients (Gaussian_Blur / _1D)
  bool fast_ok = false;           // SIFT_FLAG_FAST: pyramid_pc.hip's compiled-in taps equal the host's
  // test hooks (SIFT_HIP_TEST_HOOKS, a comma list read at context creation; tests only):
  bool poison_pad = false;        // "poison_pad": NaN into every plane's pitch padding after the pyramid
  bool stall_once = false;        // "pc_stall_once": the next pyr_pc_kernel launch gets an expired wait bound
  // exact blur: launches with fewer 8-pixel tile workgroups than this use the
  // 2-output-per-lane tiles (blur_small_kernel); SIFT_HIP_SMALL_MAX overrides
  long long small_max = 2048;
  size_t coef_gen_cap = 0;
  int wsz[4] = {0, 0, 0, 0};
  int w_base = 0;
  bool sym_blur = false;          // symmetric scatter blur (blur.hip) for the base and octave scales
  int sym_min = 256;              // ... for launches of >= sym_min 64-column strips x images
  int sym_rows = 0;               //     of >= sym_rows rows (A/B knob, SIFT_HIP_SYM_ROWS_MIN)
  size_t coef_base_off = 0, coef_oct_off = 0;
  MathConsts* d_mc = nullptr;
  DetectBufs D{};
  int blk_cap = 0;
  int* d_img_off = nullptr;       // [max_batch+1] for the host entry points
  sift_keypoint* d_kpts = nullptr;
  float* d_desc = nullptr;
  int kp_cap = 0;
  int* d_perm = nullptr;          // descriptor lane-balance ranking scratch (desc_rank_kernel)
  int perm_cap = 0;
  int last_n = -1;                // keypoints held from the last host call
  bool last_has_desc = false;
  int* d_err = nullptr;           // sticky error words [assert, workspace, kp capacity] (common.hpp)
  int* d_stat = nullptr;          // status_kernel output: {candidates, keypoints, error word, 0}
  int* h_stat = nullptr;          // pinned copy of d_stat, written at the end of every compute call
  void* d_match = nullptr;        // knn-match scratch (grown on demand)
  // hipGraph cache of compute sequences (one per argument set; SIFT_FLAG_NO_GRAPH,
  // _PROFILE and _VERBOSE run the launches directly)
  struct GraphEntry {
    std::vector<char> key;   // everything that shapes the sequence (dims, batch, flags, ...)
    std::vector<char> ptrs;  // the caller's buffers baked into the kernel arguments
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
  };
  std::vector<GraphEntry> graphs;
  long long graph_captures = 0, graph_updates = 0, graph_instantiations = 0;  // sift_graph_stats
  size_t match_cap = 0;
  // profiling
  std::vector<StageRec> recs;
  std::vector<hipEvent_t> pool;
  double acc_ms[ST_N] = {0}, acc_flops[ST_N] = {0}, acc_bytes[ST_N] = {0};
  int acc_n[ST_N] = {0};
};

namespace {

int fail(sift_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_fail(sift_ctx* c, hipError_t e, const char* what) {
  return fail(c, SIFT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(ctx, expr)                                   \
  do {                                                       \
    hipError_t e_ = (expr);                                  \
    if (e_ != hipSuccess) return hip_fail((ctx), e_, #expr); \
  } while (0)

hipEvent_t get_event(sift_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

struct StageScope {
  sift_ctx* c;
  int stage;
  double flops, bytes;
  hipEvent_t a = nullptr;
  StageScope(sift_ctx* c_, int st, double f = 0, double b = 0) : c(c_), stage(st), flops(f), bytes(b) {
    if (c->flags & SIFT_FLAG_PROFILE) {
      a = get_event(c);
      (void)hipEventRecord(a, c->stream);
    }
  }
  ~StageScope() {
    if (a) {
      hipEvent_t b = get_event(c);
      (void)hipEventRecord(b, c->stream);
      c->recs.push_back(StageRec{stage, a, b, flops, bytes});
    }
  }
};

void drain_profile(sift_ctx* c) {
  if (c->recs.empty()) return;
  (void)hipStreamSynchronize(c->stream);
  for (auto& r : c->recs) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    c->acc_ms[r.stage] += ms;
    c->acc_flops[r.stage] += r.flops;
    c->acc_bytes[r.stage] += r.bytes;
    c->acc_n[r.stage] += 1;
    c->pool.push_back(r.a);
    c->pool.push_back(r.b);
  }
  c->recs.clear();
}

int max_octaves_for(int rows, int cols) {
  int n = 0;
  while (n < kMaxOctaves && (rows >> n) >= 1 && (cols >> n) >= 1) ++n;
  return n;
}

int check_dims(sift_ctx* c, int rows, int cols, int n_oct, int batch) {
  if (rows <= 0 || cols <= 0) return fail(c, SIFT_E_INVALID, "image dimensions must be positive");
  if (n_oct < 1 || n_oct > kMaxOctaves) return fail(c, SIFT_E_INVALID, "n_octaves out of range");
  if ((rows >> (n_oct - 1)) < 1 || (cols >> (n_oct - 1)) < 1)
    return fail(c, SIFT_E_INVALID,
                "image too small: every octave must keep at least one row and column "
                "(the reference's resize to an empty Size throws)");
  if (rows > c->max_rows || cols > c->max_cols || batch > c->max_batch || n_oct > c->max_oct)
    return fail(c, SIFT_E_SIZE, "image/batch exceeds the context's creation limits");
  if (batch < 1) return fail(c, SIFT_E_INVALID, "batch must be >= 1");
  return SIFT_OK;
}

// SIFT_FLAG_FAST preconditions: pyramid_pc.hip's literal taps equal the host
// formula, and every plane and the input rows stay below the buffer offset
// its dropped loads and stores use (without the size check a plane
// of ~530 M pixels would read real pixels as padding and write inside itself).
int check_fast(sift_ctx* c, const Layout& L, long long src_row_stride) {
  if (!(c->flags & SIFT_FLAG_FAST)) return SIFT_OK;
  if (!c->fast_ok) return fail(c, SIFT_E_INVALID, "SIFT_FLAG_FAST: compiled-in separable taps differ from the host's");
  if (!pyramid_fast_fits(L, src_row_stride))
    return fail(c, SIFT_E_SIZE,
                "SIFT_FLAG_FAST: the octave-0 plane or the input rows exceed the separable pyramid's "
                "2,130,706,432-byte buffer-offset range");
  return SIFT_OK;
}

// coefficient scratch for arbitrary sigma
int ensure_coef_gen(sift_ctx* c, size_t n) {
  if (n <= c->coef_gen_cap) return SIFT_OK;
  if (c->d_coef_gen) (void)hipFree(c->d_coef_gen);
  c->d_coef_gen = nullptr;
  HIP_TRY(c, dmalloc(&c->d_coef_gen, n));
  c->coef_gen_cap = n;
  return SIFT_OK;
}

void drop_graphs(sift_ctx* c);

int ensure_kp(sift_ctx* c, int need) {
  if (need <= c->kp_cap) return SIFT_OK;
  drop_graphs(c);  // captured sequences name the old buffers
  if (c->d_kpts) (void)hipFree(c->d_kpts);
  if (c->d_desc) (void)hipFree(c->d_desc);
  c->d_kpts = nullptr;
  c->d_desc = nullptr;
  c->kp_cap = 0;
  HIP_TRY(c, dmalloc(&c->d_kpts, (size_t)need));
  HIP_TRY(c, dmalloc(&c->d_desc, (size_t)need * kDescLen));
  c->kp_cap = need;
  return SIFT_OK;
}

// The descriptor's ranking scratch (one int per keypoint the descriptor pass
// can see); grown before any capture (captured sequences name the buffer).
int ensure_perm(sift_ctx* c, int need) {
  if (need <= c->perm_cap) return SIFT_OK;
  drop_graphs(c);
  if (c->d_perm) (void)hipFree(c->d_perm);
  c->d_perm = nullptr;
  c->perm_cap = 0;
  HIP_TRY(c, dmalloc(&c->d_perm, (size_t)need));
  c->perm_cap = need;
  return SIFT_OK;
}

// Candidate-list workspace for cap extrema (all images of a batch), plus the
// internal keypoint buffer at 2 keypoints per candidate slot.
int alloc_candidates(sift_ctx* c, int cap) {
  drop_graphs(c);
  void* old[] = {c->D.cands, c->D.couts, c->D.kp_scan, c->D.npeaks, c->D.scan_tmp, c->D.scan_tiles};
  for (void* p : old)
    if (p) (void)hipFree(p);
  c->D.cands = nullptr;
  c->D.couts = nullptr;
  c->D.kp_scan = c->D.npeaks = c->D.scan_tmp = c->D.scan_tiles = nullptr;
  c->D.cand_cap = 0;
  const size_t scan_n = (size_t)std::max<long long>(c->blk_cap, cap) + 1;
  if (dmalloc(&c->D.cands, (size_t)cap) != hipSuccess || dmalloc(&c->D.couts, (size_t)cap) != hipSuccess ||
      dmalloc(&c->D.kp_scan, (size_t)cap + 1) != hipSuccess || dmalloc(&c->D.npeaks, (size_t)cap) != hipSuccess ||
      dmalloc(&c->D.scan_tmp, scan_n) != hipSuccess ||
      dmalloc(&c->D.scan_tiles, (size_t)scan_tiles_for((long long)scan_n) + 1) != hipSuccess)
    return fail(c, SIFT_E_NOMEM, "candidate workspace allocation failed");
  c->D.cand_cap = cap;
  return ensure_kp(c, (int)std::min<long long>((long long)cap * 2, 1 << 28));
}

double plane_px(const Layout& L, int o) { return (double)L.oct[o].rows * L.oct[o].cols; }

bool use_sym_blur(const sift_ctx* c, int rows, int cols, int batch) {
  return c->sym_blur && rows >= c->sym_rows && (long long)((cols + 63) / 64) * batch >= c->sym_min;
}

// Test switch for the pitch-padding invariant (common.hpp, kPitchAlign):
// overwrite columns [cols, pitch) of every Gaussian plane of the batch with a
// NaN once the pyramid is built, so a later kernel that read them would change
// its output (tests/test_gpu_fast.py::test_pitch_padding_is_never_read).
struct PadArgs {
  float* gpyr;
  long long g_img;
  int n_planes;
  long long off[kMaxOctaves * kScales];
  int rows[kMaxOctaves * kScales], cols[kMaxOctaves * kScales], pitch[kMaxOctaves * kScales];
};
__global__ __launch_bounds__(64) void poison_pad_kernel(PadArgs A) {
  int r = blockIdx.x, p = 0;
  while (p < A.n_planes && r >= A.rows[p]) r -= A.rows[p++];
  if (p >= A.n_planes) return;
  const int x = A.cols[p] + (int)threadIdx.x;
  if (x < A.pitch[p])
    A.gpyr[(long long)blockIdx.y * A.g_img + A.off[p] + (long long)r * A.pitch[p] + x] = __builtin_nanf("");
}
void enqueue_poison_pad(sift_ctx* c, const Layout& L, int batch) {
  PadArgs A{};
  A.gpyr = c->d_gpyr;
  A.g_img = L.g_img;
  int total = 0;
  for (int o = 0; o < L.n_oct; ++o)
    for (int s = 0; s < kScales; ++s) {
      const int p = A.n_planes++;
      A.off[p] = L.oct[o].g_off[s];
      A.rows[p] = L.oct[o].rows;
      A.cols[p] = L.oct[o].cols;
      A.pitch[p] = L.oct[o].pitch;
      total += L.oct[o].rows;
    }
  static_assert(kPitchAlign <= 64, "one lane per padding column");
  hipLaunchKernelGGL(poison_pad_kernel, dim3(total, batch), dim3(64), 0, c->stream, A);
}

// Gaussian pyramid (src/sift.cpp:229-263) + DoG (:265-283) for a batch whose
// input planes are described by src.  Async on c->stream.
void enqueue_pyramid(sift_ctx* c, const Layout& L, Plane src, int batch, bool with_dog) {
  hipStream_t st = c->stream;
  if (c->flags & SIFT_FLAG_FAST) {
    // separable pyramid: 24 algorithmic bytes per pixel (1 read + 5 plane
    // writes); 2 x (row + column taps) flops per pixel
    for (int o = 0; o < L.n_oct; ++o) {
      const double px = plane_px(L, o) * batch;
      const double taps = 2.0 * (9 + 17 + 25 + 37) + (o == 0 ? 2.0 * 9 : 0.0);
      // pyramid_pc.hip: octave o-1's launch wrote plane 0 of octave o when
      // it is an exact half; otherwise decimate first (plane 0
      // is one of the five plane writes, the decimation's read is not
      // algorithmic, so it is outside the pyramid stage's bytes)
      if (o > 0 && !pyramid_fuses_decimation(L, o)) {
        StageScope s(c, ST_DECIMATE, 0, 8.0 * px);
        launch_decimate(st, L, o, c->d_gpyr, batch);
      }
      StageScope s(c, ST_PYR_FAST, 2.0 * taps * px, 24.0 * px);
      launch_pyramid_pc(st, L, o, c->d_gpyr, src, batch, c->d_err + 3, c->stall_once);
      c->stall_once = false;
    }
    if (c->poison_pad) enqueue_poison_pad(c, L, batch);
    if (with_dog)
      for (int o = 0; o < L.n_oct; ++o) {
        StageScope s(c, ST_DOG, 4.0 * plane_px(L, o) * batch, 36.0 * plane_px(L, o) * batch);
        launch_dog(st, L, o, c->d_gpyr, c->d_dog, batch);
      }
    return;
  }
  {
    const double px = plane_px(L, 0) * batch;
    const int k = 2 * c->w_base + 1;
    StageScope s(c, ST_BLUR_BASE, 2.0 * k * k * px, 8.0 * px);
    if (use_sym_blur(c, L.oct[0].rows, L.oct[0].cols, batch))
      launch_blur_base_sym(st, src, c->d_gpyr + L.oct[0].g_off[0], L.oct[0].pitch, L.g_img, L.rows, L.cols, batch);
    else
      launch_blur_plane(st, c->w_base, c->d_coef + c->coef_base_off, src, c->d_gpyr + L.oct[0].g_off[0],
                        L.oct[0].pitch, L.g_img, L.rows, L.cols, batch);
  }
  // Every octave blur also writes the next octave's plane 0 when it is an
  // exact half of plane 2 (no decimation launch; the launches of one image are
  // latency-bound, and the batch's decimation was a full extra read of plane 2).
  bool fused = false;  // this octave's plane 0 came out of the previous launch
  for (int o = 0; o < L.n_oct; ++o) {
    const double px = plane_px(L, o) * batch;
    if (o > 0 && !fused) {
      StageScope s(c, ST_DECIMATE, 0, 8.0 * px);
      launch_decimate(st, L, o, c->d_gpyr, batch);
    }
    {
      double taps = 0;
      for (int q = 0; q < 4; ++q) taps += (double)(2 * c->wsz[q] + 1) * (2 * c->wsz[q] + 1);
      const bool sym = use_sym_blur(c, L.oct[o].rows, L.oct[o].cols, batch);
      const bool fuse = o + 1 < L.n_oct && blur_fuses_decimation(L, o + 1);
      StageScope s(c, sym ? ST_BLUR_SYM : ST_BLUR_OCT, 2.0 * taps * px, 20.0 * px);
      if (sym)
        launch_blur_octave_sym(st, L, o, c->d_gpyr, batch, fuse);
      else if (blur_octave_tiles(L, o, batch) < c->small_max)
        launch_blur_octave_small(st, L, o, c->d_gpyr, c->d_coef + c->coef_oct_off, c->wsz, batch, fuse);
      else
        launch_blur_octave(st, L, o, c->d_gpyr, c->d_coef + c->coef_oct_off, c->wsz, batch, fuse);
      fused = fuse;
    }
    if (with_dog) {
      StageScope s(c, ST_DOG, 4.0 * px, 36.0 * px);
      launch_dog(st, L, o, c->d_gpyr, c->d_dog, batch);
    }
  }
  if (c->poison_pad) enqueue_poison_pad(c, L, batch);
}

// dog_from_gpyr: the fused extrema pass forms the DoG values from the Gaussian
// pyramid and refinement re-forms the few it needs, so no DoG plane is written
// (SIFT_NCL never returns them); otherwise the DoG planes are already resident
// (sift_find_scale_space_extrema uploads both pyramids).
void enqueue_detect(sift_ctx* c, const Layout& L, int batch, sift_keypoint* kpts, int kp_cap,
                    int* img_off, bool dog_from_gpyr) {
  hipStream_t st = c->stream;
  {
    StageScope s(c, ST_EXTREMA);
    launch_extrema(st, L, c->d_gpyr, c->d_dog, dog_from_gpyr, c->d_grad, c->d_mc, batch, c->D);
  }
  {
    StageScope s(c, ST_REFINE);
    launch_refine_orient(st, L, c->d_gpyr, c->d_grad, dog_from_gpyr ? nullptr : c->d_dog, c->d_mc, c->D, batch);
  }
  {
    StageScope s(c, ST_EMIT);
    launch_emit(st, c->D, batch, kpts, kp_cap, img_off);
  }
}

void enqueue_desc(sift_ctx* c, const Layout& L, const sift_keypoint* kpts, const int* img_off,
                  int batch, int kp_cap, float* desc, int first_octave, bool detected) {
  StageScope s(c, ST_DESC);
  launch_descriptors(c->stream, L, c->d_grad, c->d_mc, kpts, img_off, batch, std::min(kp_cap, c->perm_cap), desc,
                     first_octave, c->d_err, detected, c->d_perm);
}

// End of every compute sequence: status_kernel folds the candidate and
// keypoint capacity checks into the sticky error word and the status block is
// copied to pinned host memory on the same stream, so the host learns the
// counts from the one stream synchronisation it already does.
// img_off == nullptr: no keypoint count (calDescriptor); check_cand false: no
// candidate check (no detection ran).
void enqueue_status(sift_ctx* c, bool check_cand, const int* img_off, int batch, int kp_cap) {
  launch_status(c->stream, check_cand ? c->D.cand_total : nullptr, c->D.cand_cap, img_off, batch, kp_cap, c->d_err,
                c->d_stat);
  (void)hipMemcpyAsync(c->h_stat, c->d_stat, 4 * sizeof(int), hipMemcpyDeviceToHost, c->stream);
}

// After a stream sync: interprets the pinned status block of the last
// compute call -- its own bits (sticky = false: host entry points) or every
// bit not yet reported (sticky = true: sift_sync) -- restricted to mask, and
// clears the device words of the bits it consumes.  kp_internal: keypoint
// overflow of the context's own buffer is the caller's growth case.
int take_status(sift_ctx* c, bool sticky, int mask, bool kp_internal = false) {
  const int ct = c->h_stat[0], n = c->h_stat[1];
  int e = (sticky ? c->h_stat[3] : c->h_stat[2]) & mask;
  for (int i = 0; i < 4; ++i)
    if (e & (1 << i)) HIP_TRY(c, hipMemsetAsync(c->d_err + i, 0, sizeof(int), c->stream));
  c->h_stat[2] &= ~e;
  c->h_stat[3] &= ~e;
  if (kp_internal) e &= ~kErrKpCapacity;
  if (!e) return SIFT_OK;
  if (e & kErrWorkspace)
    return fail(c, SIFT_E_WORKSPACE,
                "candidate workspace overflow: capacity " + std::to_string(c->D.cand_cap) + " < " +
                    std::to_string(ct) + " extrema (sift_set_candidate_capacity, or a larger context)");
  if (e & kErrStall)
    return fail(c, SIFT_E_HIP, "an in-kernel pipeline wait expired (pyramid_pc.hip): the SIFT_FLAG_FAST planes are invalid");
  if (e & kErrAssert)
    return fail(c, SIFT_E_INVALID,
                "keypoint octave/layer outside the pyramid (CV_Assert at src/sift.cpp:744)");
  return fail(c, SIFT_E_CAPACITY, "keypoint total " + std::to_string(n) +
                                      " exceeds the output capacity (see d_img_offsets[batch])");
}

constexpr int kAllErr = kErrAssert | kErrWorkspace | kErrKpCapacity | kErrStall;

// ---- hipGraph cache --------------------------------------------------------
template <typename T>
void key_put(std::vector<char>& k, const T& v) {
  const char* p = reinterpret_cast<const char*>(&v);
  k.insert(k.end(), p, p + sizeof(T));
}

void drop_graphs(sift_ctx* c) {
  for (auto& g : c->graphs) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (g.graph) (void)hipGraphDestroy(g.graph);
  }
  c->graphs.clear();
}

bool graphs_enabled(const sift_ctx* c) {
  return !(c->flags & (SIFT_FLAG_PROFILE | SIFT_FLAG_VERBOSE | SIFT_FLAG_NO_GRAPH));
}

// Runs body() on the context stream: replayed from a cached hipGraph when one
// was captured for the same key and buffers; captured now otherwise (direct
// launches if graphs are off or capture fails).  A caller whose buffers move
// between calls (a caching allocator, a ring of output slots) with the same
// shape gets the new capture patched into the cached executable with
// hipGraphExecUpdate -- no re-instantiation -- so a rotating set of buffers
// does not thrash the 4-entry cache.
template <typename F>
int run_graphed(sift_ctx* c, const std::vector<char>& key, const std::vector<char>& ptrs, F&& body) {
  if (!graphs_enabled(c)) {
    body();
    HIP_TRY(c, hipGetLastError());
    return SIFT_OK;
  }
  for (size_t i = 0; i < c->graphs.size(); ++i)
    if (c->graphs[i].key == key && c->graphs[i].ptrs == ptrs) {
      HIP_TRY(c, hipGraphLaunch(c->graphs[i].exec, c->stream));
      return SIFT_OK;
    }
  hipGraph_t g = nullptr;
  if (hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    body();
    HIP_TRY(c, hipGetLastError());
    return SIFT_OK;
  }
  body();
  const hipError_t le = hipGetLastError();
  const hipError_t ce = hipStreamEndCapture(c->stream, &g);
  if (le != hipSuccess || ce != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    body();  // capture failed: nothing ran, launch directly
    HIP_TRY(c, hipGetLastError());
    return SIFT_OK;
  }
  c->graph_captures++;
  // same shape, other buffers: update the cached executable in place
  for (size_t i = 0; i < c->graphs.size(); ++i) {
    sift_ctx::GraphEntry& e = c->graphs[i];
    if (e.key != key) continue;
    hipGraphNode_t err_node = nullptr;
    hipGraphExecUpdateResult res;
    if (hipGraphExecUpdate(e.exec, g, &err_node, &res) == hipSuccess && res == hipGraphExecUpdateSuccess) {
      (void)hipGraphDestroy(e.graph);
      e.graph = g;
      e.ptrs = ptrs;
      c->graph_updates++;
      HIP_TRY(c, hipGraphLaunch(e.exec, c->stream));
      return SIFT_OK;
    }
    // not updatable: the update may have patched some nodes before it
    // failed, so this executable no longer matches its recorded buffers --
    // drop the entry and instantiate a new executable below
    (void)hipGetLastError();
    (void)hipGraphExecDestroy(e.exec);
    (void)hipGraphDestroy(e.graph);
    c->graphs.erase(c->graphs.begin() + (long)i);
    break;
  }
  sift_ctx::GraphEntry e;
  e.key = key;
  e.ptrs = ptrs;
  e.graph = g;
  if (hipGraphInstantiate(&e.exec, e.graph, nullptr, nullptr, 0) != hipSuccess) {
    (void)hipGraphDestroy(e.graph);
    (void)hipGetLastError();
    body();
    HIP_TRY(c, hipGetLastError());
    return SIFT_OK;
  }
  c->graph_instantiations++;
  if (c->graphs.size() >= 4) {
    (void)hipGraphExecDestroy(c->graphs.front().exec);
    (void)hipGraphDestroy(c->graphs.front().graph);
    c->graphs.erase(c->graphs.begin());
  }
  c->graphs.push_back(e);
  HIP_TRY(c, hipGraphLaunch(e.exec, c->stream));
  return SIFT_OK;
}

int upload_image(sift_ctx* c, const float* img, int rows, int cols, size_t row_stride_bytes) {
  StageScope s(c, ST_UPLOAD, 0, 4.0 * rows * cols);
  HIP_TRY(c, hipMemcpy2DAsync(c->d_in, c->in_pitch * sizeof(float), img, row_stride_bytes,
                              (size_t)cols * sizeof(float), rows, hipMemcpyHostToDevice, c->stream));
  return SIFT_OK;
}

// packed host pyramid <-> pitched device pyramid (image 0)
int copy_pyramid(sift_ctx* c, const Layout& L, float* dev, const float* host_in, float* host_out,
                 int per) {
  size_t off = 0;
  for (int o = 0; o < L.n_oct; ++o) {
    const Octave& O = L.oct[o];
    for (int s = 0; s < per; ++s) {
      float* d = dev + (per == kScales ? O.g_off[s] : O.d_off[s]);
      const size_t w = (size_t)O.cols * sizeof(float);
      if (host_in)
        HIP_TRY(c, hipMemcpy2DAsync(d, O.pitch * sizeof(float), host_in + off, w, w, O.rows,
                                    hipMemcpyHostToDevice, c->stream));
      if (host_out)
        HIP_TRY(c, hipMemcpy2DAsync(host_out + off, w, d, O.pitch * sizeof(float), w, O.rows,
                                    hipMemcpyDeviceToHost, c->stream));
      off += (size_t)O.rows * O.cols;
    }
  }
  return SIFT_OK;
}

void verbose_phase(sift_ctx* c, const char* what, hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(&ms, a, b);
  printf("%s: %g\n", what, (double)ms);
}

}  // namespace

extern "C" {

int sift_graph_stats(const sift_ctx* c, long long* captures, long long* updates, long long* instantiations) {
  if (!c || !captures || !updates || !instantiations) return SIFT_E_INVALID;
  *captures = c->graph_captures;
  *updates = c->graph_updates;
  *instantiations = c->graph_instantiations;
  return SIFT_OK;
}

const char* sift_version(void) { return "sift-hip 0.2 (gfx950; exact + SIFT_FLAG_FAST separable pyramid)"; }

int sift_octave_shapes(int rows, int cols, int n_octaves, int* orows, int* ocols) {
  if (n_octaves < 1 || n_octaves > kMaxOctaves || !orows || !ocols) return SIFT_E_INVALID;
  int r = rows, c = cols;
  for (int o = 0; o < n_octaves; ++o) {
    orows[o] = r;
    ocols[o] = c;
    r /= 2;
    c /= 2;
  }
  return SIFT_OK;
}

size_t sift_packed_size(int rows, int cols, int n_octaves, int per) {
  size_t t = 0;
  int r = rows, c = cols;
  for (int o = 0; o < n_octaves; ++o) {
    t += (size_t)per * r * c;
    r /= 2;
    c /= 2;
  }
  return t;
}

int sift_ctx_create(int device, int max_rows, int max_cols, int max_batch, unsigned flags,
                    sift_ctx** out) {
  if (!out || max_rows < 1 || max_cols < 1 || max_batch < 1) return SIFT_E_INVALID;
  *out = nullptr;
  // descriptor.hip gathers with 32-bit element offsets inside one plane
  // (row * pitch + col): an octave-0 plane must stay below 2^31 elements
  if ((long long)max_rows * round_up(max_cols, kPitchAlign) >= (1ll << 31)) return SIFT_E_SIZE;
  if (hipSetDevice(device) != hipSuccess) return SIFT_E_HIP;
  sift_ctx* c = new sift_ctx();
  c->device = device;
  c->flags = flags;
  c->max_rows = max_rows;
  c->max_cols = max_cols;
  c->max_batch = max_batch;
  c->max_oct = max_octaves_for(max_rows, max_cols);
  auto bail = [&](int code) {
    sift_ctx_destroy(c);
    return code;
  };
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail(SIFT_E_HIP);
  c->own_stream = true;
  const Layout L = make_layout(max_rows, max_cols, c->max_oct);
  c->in_pitch = round_up(max_cols, kPitchAlign);
  c->in_img = c->in_pitch * max_rows;
  c->gpyr_elems = L.g_img * max_batch;
  c->dog_elems = L.d_img * max_batch;
  if (dmalloc(&c->d_in, (size_t)c->in_img * max_batch) != hipSuccess ||
      dmalloc(&c->d_gpyr, (size_t)c->gpyr_elems) != hipSuccess ||
      dmalloc(&c->d_dog, (size_t)c->dog_elems) != hipSuccess ||
      dmalloc(&c->d_tmp, (size_t)c->in_img) != hipSuccess ||
      dmalloc(&c->d_grad, (size_t)c->gpyr_elems) != hipSuccess)
    return bail(SIFT_E_NOMEM);
  // Gaussian coefficients: base sigma sqrt(1.6^2 + 0.2^2) (src/sift.cpp:237)
  // and sig[1..4] (src/sift.cpp:240-245), each through getGaussianKernel(float).
  std::vector<float> coefs;
  float sig_f[4] = {0, 0, 0, 0};
  float sb = 0;
  sift_sigmas(&sb, sig_f);
  {
    const int ks = gaussian_kernel_host(sb, nullptr);
    c->w_base = ks / 2;
    c->coef_base_off = 0;
    coefs.resize(ks * ks);
    gaussian_kernel_host(sb, coefs.data());
    c->coef_oct_off = coefs.size();
    for (int i = 1; i < kScales; ++i) {
      const float sg = sig_f[i - 1];
      const int kk = gaussian_kernel_host(sg, nullptr);
      c->wsz[i - 1] = kk / 2;
      const size_t at = coefs.size();
      coefs.resize(at + kk * kk);
      gaussian_kernel_host(sg, coefs.data() + at);
    }
  }
  if (c->w_base != 4 || c->wsz[0] != 4 || c->wsz[1] != 8 || c->wsz[2] != 12 || c->wsz[3] != 18)
    return bail(SIFT_E_INVALID);  // the octave kernel is unrolled for these widths
  {
    // the scatter-form blur carries these tables as literals; the gather-form
    // kernels (same chain, twice the multiplies) stay as the path for any
    // mismatch and for A/B runs (SIFT_HIP_BLUR_GATHER=1)
    const char* e = getenv("SIFT_HIP_BLUR_GATHER");
    c->sym_blur = sym_tables_match(coefs.data()) && !(e && atoi(e) != 0);
    // a scatter walk is a tall column strip (its halo is recomputed per
    // chunk), so it needs many strips to fill the chip; small launches (one
    // 1080p or 8K image, the last octaves of a batch) keep the 2-D tiles.
    // SIFT_HIP_SYM_MIN=0 forces it (tests).
    const char* m = getenv("SIFT_HIP_SYM_MIN");
    if (m) c->sym_min = atoi(m);
    const char* r = getenv("SIFT_HIP_SYM_ROWS_MIN");
    if (r) c->sym_rows = atoi(r);
    const char* sm = getenv("SIFT_HIP_SMALL_MAX");
    if (sm) c->small_max = atoll(sm);
  }
  // SIFT_FLAG_FAST: pyramid_pc.hip carries its 1-D taps as literals; a
  // mismatch with the host formula makes the flag an error (enqueue-time check)
  c->fast_ok = fast_taps_match(sb, sig_f);
  {
    const char* th = getenv("SIFT_HIP_TEST_HOOKS");
    const std::string hooks = "," + std::string(th ? th : "") + ",";
    c->poison_pad = hooks.find(",poison_pad,") != std::string::npos;
    c->stall_once = hooks.find(",pc_stall_once,") != std::string::npos;
  }
  MathConsts mc;
  host_math_consts(&mc);
  if (dmalloc(&c->d_coef, coefs.size()) != hipSuccess || dmalloc(&c->d_mc, 1) != hipSuccess ||
      dmalloc(&c->d_err, 4) != hipSuccess || dmalloc(&c->d_stat, 4) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_stat), 4 * sizeof(int), hipHostMallocDefault) != hipSuccess)
    return bail(SIFT_E_NOMEM);
  memset(c->h_stat, 0, 4 * sizeof(int));
  if (hipMemcpy(c->d_coef, coefs.data(), coefs.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_mc, &mc, sizeof(mc), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->d_err, 0, 4 * sizeof(int)) != hipSuccess)
    return bail(SIFT_E_HIP);
  // detection workspace
  const long long px = (long long)max_rows * max_cols;
  const long long per_img = std::max<long long>(16384, px / 32);
  const long long cap = per_img * max_batch;
  if (cap > (1ll << 30)) return bail(SIFT_E_NOMEM);
  c->blk_cap = mask_blocks_per_image(L) * max_batch;
  if (dmalloc(&c->D.mask, (size_t)mask_words_per_image(L) * max_batch) != hipSuccess ||
      dmalloc(&c->D.blk_counts, c->blk_cap) != hipSuccess ||
      dmalloc(&c->D.cand_total, 1) != hipSuccess ||
      dmalloc(&c->D.img_cand_off, max_batch + 1) != hipSuccess ||
      dmalloc(&c->D.kp_total, 1) != hipSuccess || dmalloc(&c->d_img_off, max_batch + 1) != hipSuccess ||
      alloc_candidates(c, (int)cap) != SIFT_OK)
    return bail(SIFT_E_NOMEM);
  if (hipMemset(c->D.cand_total, 0, sizeof(int)) != hipSuccess) return bail(SIFT_E_HIP);
  *out = c;
  return SIFT_OK;
}

int sift_ctx_destroy(sift_ctx* c) {
  if (!c) return SIFT_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& r : c->recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : c->pool) (void)hipEventDestroy(e);
  drop_graphs(c);
  if (c->h_stat) (void)hipHostFree(c->h_stat);
  void* bufs[] = {c->d_stat, c->d_in, c->d_gpyr, c->d_dog, c->d_tmp, c->d_grad, c->d_coef, c->d_coef_gen, c->d_mc,
                  c->D.mask, c->D.blk_counts, c->D.cand_total, c->D.img_cand_off, c->D.cands, c->D.couts,
                  c->D.kp_scan, c->D.kp_total, c->D.npeaks, c->D.scan_tmp, c->D.scan_tiles,
                  c->d_img_off, c->d_kpts, c->d_desc, c->d_perm, c->d_err, c->d_match};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return SIFT_OK;
}

const char* sift_last_error(const sift_ctx* c) { return c ? c->err.c_str() : "null context"; }

int sift_set_stream(sift_ctx* c, void* s) {
  if (!c) return SIFT_E_INVALID;
  if (c->own_stream && c->stream) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
  }
  drop_graphs(c);  // captured on the old stream
  c->stream = (hipStream_t)s;
  c->own_stream = false;
  return SIFT_OK;
}

void* sift_get_stream(sift_ctx* c) { return c ? (void*)c->stream : nullptr; }

int sift_set_flags(sift_ctx* c, unsigned flags) {
  if (!c) return SIFT_E_INVALID;
  c->flags = flags;
  return SIFT_OK;
}

int sift_set_octaves(sift_ctx* c, int n) {
  if (!c) return SIFT_E_INVALID;
  if (n < 1 || n > c->max_oct) return fail(c, SIFT_E_INVALID, "n_octaves out of range");
  c->n_oct = n;
  return SIFT_OK;
}

int sift_set_candidate_capacity(sift_ctx* c, int per_image) {
  if (!c) return SIFT_E_INVALID;
  if (per_image < 1 || (long long)per_image * c->max_batch > (1ll << 30))
    return fail(c, SIFT_E_INVALID, "candidate capacity out of range");
  (void)hipSetDevice(c->device);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->last_n = -1;
  return alloc_candidates(c, per_image * c->max_batch);
}

int sift_sync(sift_ctx* c) {
  if (!c) return SIFT_E_INVALID;
  (void)hipSetDevice(c->device);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return take_status(c, true, kAllErr);
}

int sift_synth_images(sift_ctx* c, float* d_out, int batch, int rows, int cols, size_t row_stride,
                      size_t img_stride, int seed_base) {
  if (!c || !d_out || batch < 1 || rows < 1 || cols < 1 || row_stride < (size_t)cols)
    return fail(c, SIFT_E_INVALID, "bad synth arguments");
  (void)hipSetDevice(c->device);
  launch_synth(c->stream, d_out, batch, rows, cols, (long long)row_stride, (long long)img_stride,
               seed_base);
  HIP_TRY(c, hipGetLastError());
  return SIFT_OK;
}

int sift_copy_results(sift_ctx* c, sift_keypoint* kpts, float* desc, int cap, int* n_out) {
  if (!c) return SIFT_E_INVALID;
  if (!n_out) return fail(c, SIFT_E_INVALID, "null n_out");
  if (c->last_n < 0) return fail(c, SIFT_E_INVALID, "no results held: run a host detect call first");
  const int n = c->last_n;
  *n_out = n;
  if (n > cap) return fail(c, SIFT_E_CAPACITY, "keypoint capacity " + std::to_string(cap) +
                                                   " < required " + std::to_string(n));
  if (n == 0) return SIFT_OK;
  if (!kpts || (desc && !c->last_has_desc)) return fail(c, SIFT_E_INVALID, "nothing to copy into");
  (void)hipSetDevice(c->device);
  {
    StageScope s(c, ST_DOWNLOAD, 0, (28.0 + (desc ? 512.0 : 0.0)) * n);
    HIP_TRY(c, hipMemcpyAsync(kpts, c->d_kpts, sizeof(sift_keypoint) * n, hipMemcpyDeviceToHost, c->stream));
    if (desc)
      HIP_TRY(c, hipMemcpyAsync(desc, c->d_desc, sizeof(float) * kDescLen * n, hipMemcpyDeviceToHost,
                                c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SIFT_OK;
}

}  // extern "C"

namespace {

// The whole SIFT_NCL device sequence for a batch (pyramid -> detect ->
// descriptors -> status block), replayed from the context's hipGraph cache.
int enqueue_ncl(sift_ctx* c, const float* d_imgs, int batch, int rows, int cols, size_t row_stride,
                size_t img_stride, sift_keypoint* d_kpts, float* d_desc, int kp_cap, int* d_img_offsets) {
  const Layout L = make_layout(rows, cols, c->n_oct);
  const Plane src{d_imgs, (long long)row_stride, (long long)img_stride};
  if (int rc = check_fast(c, L, (long long)row_stride)) return rc;
  // detection yields at most kMaxPeaks keypoints per candidate slot, so the
  // ranking scratch never needs more than that, whatever kp_cap the caller gives
  if (int rc = ensure_perm(c, (int)std::min<long long>(kp_cap, (long long)kMaxPeaks * c->D.cand_cap))) return rc;
  if (c->flags & SIFT_FLAG_VERBOSE) {
    hipEvent_t v0 = get_event(c), v1 = get_event(c), v2 = get_event(c), v3 = get_event(c);
    (void)hipEventRecord(v0, c->stream);
    enqueue_pyramid(c, L, src, batch, false);
    (void)hipEventRecord(v1, c->stream);
    enqueue_detect(c, L, batch, d_kpts, kp_cap, d_img_offsets, true);
    (void)hipEventRecord(v2, c->stream);
    enqueue_desc(c, L, d_kpts, d_img_offsets, batch, kp_cap, d_desc, 0, true);
    (void)hipEventRecord(v3, c->stream);
    enqueue_status(c, true, d_img_offsets, batch, kp_cap);
    verbose_phase(c, "pyramid construction time", v0, v1);
    verbose_phase(c, "keypoint localization time", v1, v2);
    verbose_phase(c, "descriptor extraction time", v2, v3);
    c->pool.insert(c->pool.end(), {v0, v1, v2, v3});
    HIP_TRY(c, hipGetLastError());
    return SIFT_OK;
  }
  std::vector<char> key, ptrs;
  key_put(key, 1);  // sequence id
  key_put(key, batch);
  key_put(key, rows);
  key_put(key, cols);
  key_put(key, row_stride);
  key_put(key, img_stride);
  key_put(key, kp_cap);
  key_put(key, c->n_oct);
  key_put(key, c->flags);
  key_put(key, c->stall_once);  // test hook: a captured poll bound must not be replayed
  key_put(ptrs, d_imgs);
  key_put(ptrs, d_kpts);
  key_put(ptrs, d_desc);
  key_put(ptrs, d_img_offsets);
  return run_graphed(c, key, ptrs, [&]() {
    enqueue_pyramid(c, L, src, batch, false);
    enqueue_detect(c, L, batch, d_kpts, kp_cap, d_img_offsets, true);
    enqueue_desc(c, L, d_kpts, d_img_offsets, batch, kp_cap, d_desc, 0, true);
    enqueue_status(c, true, d_img_offsets, batch, kp_cap);
  });
}

}  // namespace

extern "C" {

int sift_detect_compute_batch(sift_ctx* c, const float* d_imgs, int batch, int rows, int cols,
                              size_t row_stride, size_t img_stride, sift_keypoint* d_kpts,
                              float* d_desc, int kp_cap, int* d_img_offsets) {
  if (!c) return SIFT_E_INVALID;
  int rc = check_dims(c, rows, cols, c->n_oct, batch);
  if (rc) return rc;
  if (!d_imgs || !d_kpts || !d_desc || !d_img_offsets || kp_cap < 0 || row_stride < (size_t)cols)
    return fail(c, SIFT_E_INVALID, "null buffer or bad stride");
  (void)hipSetDevice(c->device);
  c->last_n = -1;
  return enqueue_ncl(c, d_imgs, batch, rows, cols, row_stride, img_stride, d_kpts, d_desc, kp_cap,
                     d_img_offsets);
}

// SIFT_NCL from host memory: upload -> the graphed device sequence -> ONE
// stream synchronisation (the status block, with the keypoint count, arrives
// in pinned memory with it) -> one copy of exactly n results.  The internal
// keypoint buffer is sized at creation for 2 keypoints per candidate slot;
// a larger count (more than 2 orientation peaks per extremum on average)
// grows it and runs again.
int sift_detect_compute(sift_ctx* c, const float* img, int rows, int cols, size_t row_stride_bytes,
                        sift_keypoint* kpts, float* desc, int cap, int* n_out) {
  if (!c) return SIFT_E_INVALID;
  if (!img || !n_out) return fail(c, SIFT_E_INVALID, "null image or n_out");
  if (row_stride_bytes == 0) row_stride_bytes = (size_t)cols * sizeof(float);
  int rc = check_dims(c, rows, cols, c->n_oct, 1);
  if (rc) return rc;
  (void)hipSetDevice(c->device);
  c->last_n = -1;
  *n_out = -1;
  if ((rc = upload_image(c, img, rows, cols, row_stride_bytes))) return rc;
  for (int attempt = 0; attempt < 2; ++attempt) {
    rc = enqueue_ncl(c, c->d_in, 1, rows, cols, c->in_pitch, c->in_img, c->d_kpts, c->d_desc, c->kp_cap,
                     c->d_img_off);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if ((rc = take_status(c, false, kAllErr, true))) return rc;
    const int n = c->h_stat[1];
    if (n > c->kp_cap) {  // grow the internal buffer and run again
      if ((rc = ensure_kp(c, n))) return rc;
      continue;
    }
    *n_out = n;
    c->last_n = n;
    c->last_has_desc = true;
    if (n > cap || (n > 0 && (!kpts || !desc)))
      return fail(c, SIFT_E_CAPACITY, "keypoint capacity " + std::to_string(cap) +
                                          " < required " + std::to_string(n));
    if (n > 0) {
      StageScope s(c, ST_DOWNLOAD, 0, (28.0 + 512.0) * n);
      HIP_TRY(c, hipMemcpyAsync(kpts, c->d_kpts, sizeof(sift_keypoint) * n, hipMemcpyDeviceToHost,
                                c->stream));
      HIP_TRY(c, hipMemcpyAsync(desc, c->d_desc, sizeof(float) * kDescLen * n,
                                hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return SIFT_OK;
  }
  return fail(c, SIFT_E_CAPACITY, "keypoint buffer growth failed");
}

int sift_gaussian_blur(sift_ctx* c, const float* src, int rows, int cols, double sigma, float* dst) {
  if (!c) return SIFT_E_INVALID;
  if (!src || !dst) return fail(c, SIFT_E_INVALID, "null buffer");
  int rc = check_dims(c, rows, cols, 1, 1);
  if (rc) return rc;
  if (!(sigma > 0) || sigma > 100) return fail(c, SIFT_E_INVALID, "sigma out of range");
  (void)hipSetDevice(c->device);
  const int ks = gaussian_kernel_host((float)sigma, nullptr);
  std::vector<float> k((size_t)ks * ks);
  gaussian_kernel_host((float)sigma, k.data());
  if ((rc = ensure_coef_gen(c, k.size()))) return rc;
  HIP_TRY(c, hipMemcpyAsync(c->d_coef_gen, k.data(), k.size() * sizeof(float), hipMemcpyHostToDevice,
                            c->stream));
  if ((rc = upload_image(c, src, rows, cols, (size_t)cols * sizeof(float)))) return rc;
  {
    StageScope s(c, ST_BLUR_BASE, 2.0 * ks * ks * rows * cols, 8.0 * rows * cols);
    launch_blur_plane(c->stream, ks / 2, c->d_coef_gen, Plane{c->d_in, c->in_pitch, c->in_img},
                      c->d_tmp, c->in_pitch, c->in_img, rows, cols, 1);
  }
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipMemcpy2DAsync(dst, (size_t)cols * sizeof(float), c->d_tmp, c->in_pitch * sizeof(float),
                              (size_t)cols * sizeof(float), rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SIFT_OK;
}

int sift_gaussian_blur_1d(sift_ctx* c, const float* src, int rows, int cols, double sigma,
                          float* dst) {
  if (!c) return SIFT_E_INVALID;
  if (!src || !dst) return fail(c, SIFT_E_INVALID, "null buffer");
  int rc = check_dims(c, rows, cols, 1, 1);
  if (rc) return rc;
  if (!(sigma > 0) || sigma > 100) return fail(c, SIFT_E_INVALID, "sigma out of range");
  (void)hipSetDevice(c->device);
  // getGaussianKernel1D(double sigma), src/sift.cpp:157-168
  const int w = (int)floor(3 * sigma);
  std::vector<float> k(2 * w + 1);
  for (int i = -w; i <= w; ++i)
    k[i + w] = (float)(1. / sqrt(2 * kRefPi * sigma * sigma) *
                       exp(-((double)i * i) * 1. / (2 * sigma * sigma)));
  if ((rc = ensure_coef_gen(c, k.size()))) return rc;
  HIP_TRY(c, hipMemcpyAsync(c->d_coef_gen, k.data(), k.size() * sizeof(float), hipMemcpyHostToDevice,
                            c->stream));
  if ((rc = upload_image(c, src, rows, cols, (size_t)cols * sizeof(float)))) return rc;
  float* out = c->d_gpyr;  // scratch (>= one max-size plane)
  {
    StageScope s(c, ST_BLUR1D, 4.0 * (2 * w) * rows * cols, 16.0 * rows * cols);
    launch_blur_1d(c->stream, w, c->d_coef_gen, Plane{c->d_in, c->in_pitch, c->in_img}, c->d_tmp, out,
                   c->in_pitch, c->in_img, rows, cols, 1);
  }
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipMemcpy2DAsync(dst, (size_t)cols * sizeof(float), out, c->in_pitch * sizeof(float),
                              (size_t)cols * sizeof(float), rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SIFT_OK;
}

int sift_build_gaussian_pyramid(sift_ctx* c, const float* img, int rows, int cols, int n_octaves,
                                float* gpyr) {
  if (!c) return SIFT_E_INVALID;
  if (!img || !gpyr) return fail(c, SIFT_E_INVALID, "null buffer");
  int rc = check_dims(c, rows, cols, n_octaves, 1);
  if (rc) return rc;
  (void)hipSetDevice(c->device);
  const Layout L = make_layout(rows, cols, n_octaves);
  if ((rc = check_fast(c, L, c->in_pitch))) return rc;
  if ((rc = upload_image(c, img, rows, cols, (size_t)cols * sizeof(float)))) return rc;
  enqueue_pyramid(c, L, Plane{c->d_in, c->in_pitch, c->in_img}, 1, false);
  // SIFT_FLAG_FAST: an expired in-kernel wait of pyr_pc_kernel (err[3]) means
  // the planes are invalid -- reported by this call, and consumed so that it
  // cannot surface in a later one
  enqueue_status(c, false, nullptr, 1, c->kp_cap);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if ((rc = take_status(c, false, kErrStall))) return rc;
  if ((rc = copy_pyramid(c, L, c->d_gpyr, nullptr, gpyr, kScales))) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SIFT_OK;
}

int sift_build_dog_pyramid(sift_ctx* c, const float* gpyr, int rows, int cols, int n_octaves,
                           float* dog) {
  if (!c) return SIFT_E_INVALID;
  if (!gpyr || !dog) return fail(c, SIFT_E_INVALID, "null buffer");
  int rc = check_dims(c, rows, cols, n_octaves, 1);
  if (rc) return rc;
  (void)hipSetDevice(c->device);
  const Layout L = make_layout(rows, cols, n_octaves);
  if ((rc = copy_pyramid(c, L, c->d_gpyr, gpyr, nullptr, kScales))) return rc;
  for (int o = 0; o < L.n_oct; ++o) {
    StageScope s(c, ST_DOG, 4.0 * plane_px(L, o), 36.0 * plane_px(L, o));
    launch_dog(c->stream, L, o, c->d_gpyr, c->d_dog, 1);
  }
  HIP_TRY(c, hipGetLastError());
  if ((rc = copy_pyramid(c, L, c->d_dog, nullptr, dog, kDogPer))) return rc;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SIFT_OK;
}

int sift_find_scale_space_extrema(sift_ctx* c, const float* gpyr, const float* dog, int rows,
                                  int cols, int n_octaves, sift_keypoint* kpts, int cap, int* n_out) {
  if (!c) return SIFT_E_INVALID;
  if (!gpyr || !dog || !n_out) return fail(c, SIFT_E_INVALID, "null buffer");
  int rc = check_dims(c, rows, cols, n_octaves, 1);
  if (rc) return rc;
  (void)hipSetDevice(c->device);
  const Layout L = make_layout(rows, cols, n_octaves);
  if ((rc = copy_pyramid(c, L, c->d_gpyr, gpyr, nullptr, kScales))) return rc;
  if ((rc = copy_pyramid(c, L, c->d_dog, dog, nullptr, kDogPer))) return rc;
  c->last_n = -1;
  *n_out = -1;
  for (int attempt = 0; attempt < 2; ++attempt) {
    enqueue_detect(c, L, 1, c->d_kpts, c->kp_cap, c->d_img_off, false);
    enqueue_status(c, true, c->d_img_off, 1, c->kp_cap);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if ((rc = take_status(c, false, kAllErr, true))) return rc;
    const int n = c->h_stat[1];
    if (n > c->kp_cap) {
      if ((rc = ensure_kp(c, n))) return rc;
      continue;
    }
    *n_out = n;
    c->last_n = n;
    c->last_has_desc = false;
    if (n > cap || (n > 0 && !kpts))
      return fail(c, SIFT_E_CAPACITY, "keypoint capacity " + std::to_string(cap) +
                                          " < required " + std::to_string(n));
    if (n > 0)
      HIP_TRY(c, hipMemcpy(kpts, c->d_kpts, sizeof(sift_keypoint) * n, hipMemcpyDeviceToHost));
    return SIFT_OK;
  }
  return fail(c, SIFT_E_CAPACITY, "keypoint buffer growth failed");
}

int sift_calc_descriptors(sift_ctx* c, const float* gpyr, int rows, int cols, int n_octaves,
                          const sift_keypoint* kpts, int n, float* desc, int first_octave) {
  if (!c) return SIFT_E_INVALID;
  if (!gpyr || (n > 0 && (!kpts || !desc)) || n < 0) return fail(c, SIFT_E_INVALID, "null buffer");
  int rc = check_dims(c, rows, cols, n_octaves, 1);
  if (rc) return rc;
  if (n == 0) return SIFT_OK;
  (void)hipSetDevice(c->device);
  const Layout L = make_layout(rows, cols, n_octaves);
  if ((rc = ensure_kp(c, n))) return rc;
  c->last_n = -1;  // the internal keypoint buffer is reused below
  if ((rc = copy_pyramid(c, L, c->d_gpyr, gpyr, nullptr, kScales))) return rc;
  const int off[2] = {0, n};
  HIP_TRY(c, hipMemcpyAsync(c->d_img_off, off, sizeof(off), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->d_kpts, kpts, sizeof(sift_keypoint) * n, hipMemcpyHostToDevice,
                            c->stream));
  // keypoints may name any scale 0..4 (CV_Assert at src/sift.cpp:744): gradients of all five
  launch_grad(c->stream, L, c->d_gpyr, c->d_grad, 1, 0, kScales - 1, c->d_mc);
  if ((rc = ensure_perm(c, c->kp_cap))) return rc;
  enqueue_desc(c, L, c->d_kpts, c->d_img_off, 1, c->kp_cap, c->d_desc, first_octave, false);
  enqueue_status(c, false, nullptr, 1, c->kp_cap);  // no detection ran: assertion bit only
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if ((rc = take_status(c, false, kErrAssert))) return rc;
  HIP_TRY(c, hipMemcpy(desc, c->d_desc, sizeof(float) * kDescLen * n, hipMemcpyDeviceToHost));
  return SIFT_OK;
}

int sift_selftest_math(sift_ctx* c, int op, const float* a, const float* b, float* out, int n) {
  if (!c) return SIFT_E_INVALID;
  if (!a || !out || n < 0 || op < 0 || op > 7 || ((op == 1 || op == 2) && !b))
    return fail(c, SIFT_E_INVALID, "bad selftest arguments");
  if (n == 0) return SIFT_OK;
  (void)hipSetDevice(c->device);
  float *da = nullptr, *db = nullptr, *dout = nullptr;
  HIP_TRY(c, dmalloc(&da, (size_t)n));
  HIP_TRY(c, dmalloc(&db, (size_t)n));
  HIP_TRY(c, dmalloc(&dout, (size_t)n));
  hipError_t e = hipMemcpy(da, a, sizeof(float) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess && b) e = hipMemcpy(db, b, sizeof(float) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    launch_math_selftest(c->stream, op, da, db, dout, n, c->d_mc);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(float) * n, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  if (e != hipSuccess) return hip_fail(c, e, "sift_selftest_math");
  return SIFT_OK;
}

// ---- BFMatcher(NORM_L1).knnMatch, src/main.cpp:25-27 ----
namespace {

int ensure_match(sift_ctx* c, size_t bytes) {
  if (bytes <= c->match_cap) return SIFT_OK;
  if (c->d_match) {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    (void)hipFree(c->d_match);
    c->d_match = nullptr;
    c->match_cap = 0;
  }
  if (hipMalloc(&c->d_match, bytes) != hipSuccess) return fail(c, SIFT_E_NOMEM, "match scratch");
  c->match_cap = bytes;
  return SIFT_OK;
}

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

int check_match_args(sift_ctx* c, int n_query, int n_train, int k) {
  if (n_query < 0 || n_train < 0) return fail(c, SIFT_E_INVALID, "negative descriptor count");
  if (k != 1 && k != 2) return fail(c, SIFT_E_INVALID, "k must be 1 or 2");
  return SIFT_OK;
}

size_t match_part_bytes(int nq, int nt) {
  const size_t part = (size_t)knn_splits(nq, nt) * nq;
  return align256(part * sizeof(float2)) + align256(part * sizeof(int2));
}

// Partials at d_match + off (the scratch must already hold off + match_part_bytes).
int knn_device(sift_ctx* c, const float* q, int nq, const float* t, int nt, int k, int* idx, float* dist,
               size_t off) {
  const int splits = knn_splits(nq, nt);
  const size_t part = (size_t)splits * nq;
  char* base = static_cast<char*>(c->d_match) + off;
  float2* pd = reinterpret_cast<float2*>(base);
  int2* pi = reinterpret_cast<int2*>(base + align256(part * sizeof(float2)));
  {
    StageScope s(c, ST_MATCH, 2.0 * kDescLen * nq * (double)nt, 512.0 * (nq + (double)nt));
    launch_knn_l1(c->stream, q, nq, t, nt, k, splits, pd, pi, idx, dist);
  }
  HIP_TRY(c, hipGetLastError());
  return SIFT_OK;
}

}  // namespace

int sift_knn_match_l1_device(sift_ctx* c, const float* d_query, int n_query, const float* d_train, int n_train,
                             int k, int* d_idx, float* d_dist) {
  if (!c) return SIFT_E_INVALID;
  int rc = check_match_args(c, n_query, n_train, k);
  if (rc) return rc;
  if (n_query == 0) return SIFT_OK;
  if (!d_query || !d_idx || !d_dist || (n_train > 0 && !d_train)) return fail(c, SIFT_E_INVALID, "null buffer");
  if ((reinterpret_cast<uintptr_t>(d_query) | reinterpret_cast<uintptr_t>(d_train)) & 15)
    return fail(c, SIFT_E_INVALID, "descriptor rows must be 16-byte aligned");
  (void)hipSetDevice(c->device);
  if ((rc = ensure_match(c, match_part_bytes(n_query, n_train)))) return rc;
  return knn_device(c, d_query, n_query, d_train, n_train, k, d_idx, d_dist, 0);
}

int sift_knn_match_l1(sift_ctx* c, const float* query, int n_query, const float* train, int n_train, int k,
                      int* idx, float* dist) {
  if (!c) return SIFT_E_INVALID;
  int rc = check_match_args(c, n_query, n_train, k);
  if (rc) return rc;
  if (n_query == 0) return SIFT_OK;
  if (!query || !idx || !dist || (n_train > 0 && !train)) return fail(c, SIFT_E_INVALID, "null buffer");
  (void)hipSetDevice(c->device);
  const size_t qb = align256((size_t)n_query * kDescLen * sizeof(float));
  const size_t tb = align256((size_t)(n_train ? n_train : 1) * kDescLen * sizeof(float));
  const size_t ib = align256((size_t)n_query * k * sizeof(int)), db = align256((size_t)n_query * k * sizeof(float));
  const size_t off = qb + tb + ib + db;
  if ((rc = ensure_match(c, off + match_part_bytes(n_query, n_train)))) return rc;
  char* base = static_cast<char*>(c->d_match);
  float* dq = reinterpret_cast<float*>(base);
  float* dt = reinterpret_cast<float*>(base + qb);
  int* di = reinterpret_cast<int*>(base + qb + tb);
  float* dd = reinterpret_cast<float*>(base + qb + tb + ib);
  HIP_TRY(c, hipMemcpyAsync(dq, query, (size_t)n_query * kDescLen * sizeof(float), hipMemcpyHostToDevice,
                            c->stream));
  if (n_train)
    HIP_TRY(c, hipMemcpyAsync(dt, train, (size_t)n_train * kDescLen * sizeof(float), hipMemcpyHostToDevice,
                              c->stream));
  if ((rc = knn_device(c, dq, n_query, dt, n_train, k, di, dd, off))) return rc;
  HIP_TRY(c, hipMemcpyAsync(idx, di, (size_t)n_query * k * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(dist, dd, (size_t)n_query * k * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SIFT_OK;
}

// ---- readImage front end, src/main.cpp:79-87 ----
int sift_bgr8_to_gray_device(sift_ctx* c, const uint8_t* d_bgr, int batch, int rows, int cols, size_t row_stride,
                             size_t img_stride, int out_rows, int out_cols, float* d_gray, size_t out_row_stride,
                             size_t out_img_stride) {
  if (!c) return SIFT_E_INVALID;
  if (!d_bgr || !d_gray) return fail(c, SIFT_E_INVALID, "null buffer");
  if (batch < 1 || rows < 1 || cols < 1 || out_rows < 1 || out_cols < 1)
    return fail(c, SIFT_E_INVALID, "empty image");
  if (row_stride < (size_t)cols * 3 || (batch > 1 && img_stride < row_stride * rows))
    return fail(c, SIFT_E_INVALID, "source strides too small");
  if (out_row_stride % sizeof(float) || out_img_stride % sizeof(float) ||
      out_row_stride < (size_t)out_cols * sizeof(float) ||
      (batch > 1 && out_img_stride < out_row_stride * out_rows))
    return fail(c, SIFT_E_INVALID, "output strides");
  (void)hipSetDevice(c->device);
  {
    StageScope s(c, ST_UPLOAD, 0, (3.0 * rows * cols + 4.0 * out_rows * out_cols) * batch);
    launch_bgr8_gray(c->stream, d_bgr, (long long)row_stride, (long long)img_stride, rows, cols, d_gray,
                     (long long)(out_row_stride / sizeof(float)), (long long)(out_img_stride / sizeof(float)),
                     out_rows, out_cols, batch);
  }
  HIP_TRY(c, hipGetLastError());
  return SIFT_OK;
}

int sift_bgr8_to_gray(sift_ctx* c, const uint8_t* bgr, int rows, int cols, size_t row_stride, int out_rows,
                      int out_cols, float* gray) {
  if (!c) return SIFT_E_INVALID;
  if (!bgr || !gray) return fail(c, SIFT_E_INVALID, "null buffer");
  if (rows < 1 || cols < 1 || out_rows < 1 || out_cols < 1) return fail(c, SIFT_E_INVALID, "empty image");
  if (row_stride < (size_t)cols * 3) return fail(c, SIFT_E_INVALID, "row stride too small");
  (void)hipSetDevice(c->device);
  const size_t sb = align256((size_t)rows * row_stride), ob = (size_t)out_rows * out_cols * sizeof(float);
  int rc = ensure_match(c, sb + ob);  // the matcher's scratch doubles as staging here
  if (rc) return rc;
  uint8_t* d_src = static_cast<uint8_t*>(c->d_match);
  float* d_out = reinterpret_cast<float*>(static_cast<char*>(c->d_match) + sb);
  HIP_TRY(c, hipMemcpyAsync(d_src, bgr, (size_t)rows * row_stride, hipMemcpyHostToDevice, c->stream));
  if ((rc = sift_bgr8_to_gray_device(c, d_src, 1, rows, cols, row_stride, 0, out_rows, out_cols, d_out,
                                     (size_t)out_cols * sizeof(float), 0)))
    return rc;
  HIP_TRY(c, hipMemcpyAsync(gray, d_out, ob, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SIFT_OK;
}

// ---- findHomography(RANSAC) + perspectiveTransform, src/main.cpp:54-62 ----
int sift_find_homography(const float* src_xy, const float* dst_xy, int n, double ransac_thresh, int max_iters,
                         double confidence, double* H, unsigned char* inlier_mask) {
  if (!src_xy || !dst_xy || !H || n < 0) return SIFT_E_INVALID;
  if (!find_homography_ransac(src_xy, dst_xy, n, ransac_thresh, max_iters, confidence, H, inlier_mask)) {
    for (int i = 0; i < 9; ++i) H[i] = 0;  // OpenCV returns an empty Mat
    return SIFT_E_INVALID;
  }
  return SIFT_OK;
}

int sift_perspective_transform(const double* H, const float* xy, int n, float* out_xy) {
  if (!H || n < 0 || (n > 0 && (!xy || !out_xy))) return SIFT_E_INVALID;
  perspective_transform(H, xy, n, out_xy);
  return SIFT_OK;
}

int sift_get_stage_stats(sift_ctx* c, sift_stage_stat* out, int cap, int* n, int reset) {
  if (!c) return SIFT_E_INVALID;
  drain_profile(c);
  int k = 0;
  for (int s = 0; s < ST_N; ++s) {
    if (!c->acc_n[s]) continue;
    if (out && k < cap) {
      memset(&out[k], 0, sizeof(out[k]));
      strncpy(out[k].name, kStageNames[s], sizeof(out[k].name) - 1);
      out[k].launches = c->acc_n[s];
      out[k].ms = c->acc_ms[s];
      out[k].flops = c->acc_flops[s];
      out[k].bytes = c->acc_bytes[s];
    }
    ++k;
  }
  if (n) *n = k;
  if (reset)
    for (int s = 0; s < ST_N; ++s) c->acc_ms[s] = c->acc_flops[s] = c->acc_bytes[s] = c->acc_n[s] = 0;
  return SIFT_OK;
}

}  // extern "C"
