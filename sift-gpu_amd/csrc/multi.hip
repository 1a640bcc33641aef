// multi.hip -- multi-GPU batch mode behind the C ABI (SURVEY.md 8(e);
// BASELINE configs[3]: 512 x 1080p sharded over the 8 MI355X of one node).
//
// The reference's only parallelism is OpenMP over descriptors
// (src/sift.cpp:738); its images are independent, so the batch is sharded by
// contiguous image ranges and there is no data-path collective.  The one
// exchange step is the keypoint gather to device 0, and it runs one step
// behind the compute so it overlaps it:
//
//   step k (slot s = k & 1):
//     every device i runs its shard as S contiguous sub-batches, one context
//     and HIP stream each (bench.py's two-stream overlap: the sub-batches'
//     VALU-bound blur and latency-bound descriptor phases run beside each
//     other); each sub-batch's stream waits until the gather of step k - 2
//     has read slot s, runs sift_detect_compute_batch into slot s (graph
//     replay), copies its per-image offsets to pinned host memory and records
//     cdone[unit][s];
//     then the gather of step k - 1 (slot p = s ^ 1): the host waits for
//       cdone[*][p] (normally complete: step k is queued behind it), reads the
//       record counts, and one ncclGroupStart / ncclGroupEnd posts, on a
//       separate gather stream per device (waiting on cdone[i][p] on the
//       device), ncclSend of device i's records (28 B each, optionally the
//       512 B descriptors) and the matching ncclRecv on device 0 at exact
//       sizes -- point-to-point, so the xGMI links of all peers run at once
//       rather than as a ring (device 0's own pieces: a DMA copy); gdone[i][p]
//       marks slot p free again.
//   flush: the gather of the last step, then every stream is drained and the
//     contexts' sticky status reported.
//
// One process, S contexts + HIP streams per device (sift_ctx; a "unit" is one
// of them), a gather stream per device, communicators from ncclCommInitAll
// (RCCL over xGMI).  Layered on the public C ABI only.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/sift_hip.h"

struct sift_multi {
  int n = 0;   // devices
  int S = 1;   // contexts (sub-batches, streams) per device; unit u = i * S + j
  std::vector<int> dev;
  std::vector<sift_ctx*> ctx;                         // per unit
  std::vector<ncclComm_t> comm;                       // per device
  std::vector<hipStream_t> gstream;                   // per device: the gather stream
  std::vector<hipEvent_t> gdone[2];                   // per slot, per device: slot free again
  std::vector<hipEvent_t> cdone[2];                   // per slot, per unit: compute done
  std::vector<sift_keypoint*> kbuf[2];                // per slot, per unit: cap records
  std::vector<float*> dbuf[2];                        // per slot, per unit: cap x 128
  std::vector<int*> doff[2];                          // per slot, per unit: [max_batch + 1]
  std::vector<int*> hoff[2];                          // pinned copies of doff
  std::vector<int> cnt[2];                            // per slot, per unit: images of the sub-batch
  sift_keypoint* rk = nullptr;                        // device 0: gathered records, U x cap
  float* rd = nullptr;                                // device 0: gathered descriptors (gather_desc)
  std::vector<int> goff;                              // host: global offsets of the last gather
  int max_batch = 0, cap = 0, gather_desc = 0;        // cap: records per unit and slot
  long long steps = 0;       // steps enqueued
  long long gathered = -1;   // step index held by rk / goff (-1: none)
  bool pending = false;      // the last enqueued step is not gathered yet
  long long records = 0, transfers = 0;  // totals gathered (records, RCCL p2p ops)
  long long local_copies = 0;            // device 0's own pieces copied by DMA
  bool self_p2p = false;                 // SIFT_MULTI_SELF_P2P: device 0's pieces over RCCL too
  std::string err;
  std::string broken;        // set when a step or gather failed after enqueueing work: the slots'
                             // state is then undefined and every later step / flush refuses
};

extern "C" int sift_multi_merge_offsets(const int* const* shard_offsets, const int* counts, int n_devices,
                                        int* global_offsets);

namespace {

int mfail(sift_multi* m, int code, const std::string& msg) {
  if (m) m->err = msg;
  return code;
}

#define MHIP(m, call)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) return mfail(m, SIFT_E_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)
#define MNCCL(m, call)                                                                 \
  do {                                                                                 \
    ncclResult_t r_ = (call);                                                          \
    if (r_ != ncclSuccess) return mfail(m, SIFT_E_HIP, std::string(#call ": ") + ncclGetErrorString(r_)); \
  } while (0)

// Gathers slot p (the step whose per-image offsets are in hoff[p]) to device 0.
int gather_slot(sift_multi* m, int p) {
  const int U = m->n * m->S;
  std::vector<long long> nrec(U);
  long long total = 0;
  for (int u = 0; u < U; ++u) {
    MHIP(m, hipSetDevice(m->dev[u / m->S]));
    MHIP(m, hipEventSynchronize(m->cdone[p][u]));  // one step behind: normally already complete
    const int c = m->cnt[p][u];
    const long long k = c > 0 ? m->hoff[p][u][c] : 0;
    if (k > m->cap)
      return mfail(m, SIFT_E_CAPACITY, "device " + std::to_string(m->dev[u / m->S]) + ": " + std::to_string(k) +
                                           " keypoints in a sub-batch exceed its share of kp_cap_per_device (" +
                                           std::to_string(m->cap) + ")");
    nrec[u] = k;
    total += k;
  }
  // global per-image offsets (contiguous shards and sub-batches: unit order = image order)
  int batch_total = 0;
  for (int u = 0; u < U; ++u) batch_total += m->cnt[p][u];
  m->goff.assign(batch_total + 1, 0);
  std::vector<const int*> so(m->hoff[p].begin(), m->hoff[p].end());
  (void)sift_multi_merge_offsets(so.data(), m->cnt[p].data(), U, m->goff.data());
  for (int u = 0; u < U; ++u) {
    MHIP(m, hipSetDevice(m->dev[u / m->S]));
    MHIP(m, hipStreamWaitEvent(m->gstream[u / m->S], m->cdone[p][u], 0));
  }
  // device 0's own sub-batches: a DMA copy on its gather stream (RCCL's self
  // p2p runs a copy kernel on the CUs at a few GB/s: 2.7 ms for 12 MB of
  // records, profiles/r6fin_summary.md); SIFT_MULTI_SELF_P2P keeps them on
  // RCCL too (tests: the p2p path on a one-GPU box)
  long long at = 0;
  if (!m->self_p2p) {
    MHIP(m, hipSetDevice(m->dev[0]));
    for (int u = 0; u < m->S; ++u) {
      if (nrec[u] > 0) {
        MHIP(m, hipMemcpyAsync(m->rk + at, m->kbuf[p][u], (size_t)nrec[u] * sizeof(sift_keypoint),
                               hipMemcpyDeviceToDevice, m->gstream[0]));
        if (m->gather_desc)
          MHIP(m, hipMemcpyAsync(m->rd + at * SIFT_DESC_LEN, m->dbuf[p][u],
                                 (size_t)nrec[u] * SIFT_DESC_LEN * sizeof(float), hipMemcpyDeviceToDevice,
                                 m->gstream[0]));
        m->local_copies += m->gather_desc ? 2 : 1;
      }
      at += nrec[u];
    }
  }
  MNCCL(m, ncclGroupStart());
  for (int u = m->self_p2p ? 0 : m->S; u < U; ++u) {
    const int i = u / m->S;
    if (nrec[u] > 0) {
      // device i sends, device 0 receives at the record offset of unit u;
      // the pairs between two devices match in posting order
      ncclResult_t r = ncclSend(m->kbuf[p][u], (size_t)nrec[u] * sizeof(sift_keypoint), ncclUint8, 0, m->comm[i],
                                m->gstream[i]);
      if (r == ncclSuccess)
        r = ncclRecv(m->rk + at, (size_t)nrec[u] * sizeof(sift_keypoint), ncclUint8, i, m->comm[0], m->gstream[0]);
      if (r == ncclSuccess && m->gather_desc) {
        r = ncclSend(m->dbuf[p][u], (size_t)nrec[u] * SIFT_DESC_LEN, ncclFloat32, 0, m->comm[i], m->gstream[i]);
        if (r == ncclSuccess)
          r = ncclRecv(m->rd + at * SIFT_DESC_LEN, (size_t)nrec[u] * SIFT_DESC_LEN, ncclFloat32, i, m->comm[0],
                       m->gstream[0]);
      }
      if (r != ncclSuccess) {
        (void)ncclGroupEnd();
        return mfail(m, SIFT_E_HIP, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
      }
      m->transfers += m->gather_desc ? 2 : 1;
    }
    at += nrec[u];
  }
  MNCCL(m, ncclGroupEnd());
  for (int i = 0; i < m->n; ++i) {
    MHIP(m, hipSetDevice(m->dev[i]));
    MHIP(m, hipEventRecord(m->gdone[p][i], m->gstream[i]));
  }
  m->records += total;
  return SIFT_OK;
}

}  // namespace

extern "C" {

int sift_multi_shard(int batch, int n_devices, int index, int* first, int* count) {
  if (batch < 0 || n_devices < 1 || index < 0 || index >= n_devices || !first || !count) return SIFT_E_INVALID;
  // contiguous ranges: device i takes [floor(i B / n), floor((i + 1) B / n))
  // (sift_dist.shard, the Python bench's split)
  const long long lo = (long long)index * batch / n_devices;
  const long long hi = (long long)(index + 1) * batch / n_devices;
  *first = (int)lo;
  *count = (int)(hi - lo);
  return SIFT_OK;
}

int sift_multi_merge_offsets(const int* const* shard_offsets, const int* counts, int n_devices, int* global_offsets) {
  if (!shard_offsets || !counts || n_devices < 1 || !global_offsets) return SIFT_E_INVALID;
  long long base = 0;
  int b = 0;
  for (int i = 0; i < n_devices; ++i) {
    if (counts[i] < 0 || (counts[i] > 0 && !shard_offsets[i])) return SIFT_E_INVALID;
    for (int j = 0; j < counts[i]; ++j) global_offsets[b++] = (int)(base + shard_offsets[i][j]);
    base += counts[i] > 0 ? shard_offsets[i][counts[i]] : 0;
  }
  global_offsets[b] = (int)base;
  return SIFT_OK;
}

const char* sift_multi_last_error(const sift_multi* m) { return m ? m->err.c_str() : "null multi context"; }

int sift_multi_destroy(sift_multi* m) {
  if (!m) return SIFT_OK;
  const int U = (int)m->ctx.size();
  for (int u = 0; u < U; ++u)
    if (m->ctx[u]) {
      (void)hipSetDevice(m->dev[u / m->S]);
      (void)hipStreamSynchronize((hipStream_t)sift_get_stream(m->ctx[u]));
    }
  for (int i = 0; i < (int)m->gstream.size(); ++i)
    if (m->gstream[i]) {
      (void)hipSetDevice(m->dev[i]);
      (void)hipStreamSynchronize(m->gstream[i]);
    }
  for (int i = 0; i < (int)m->comm.size(); ++i)
    if (m->comm[i]) (void)ncclCommDestroy(m->comm[i]);
  for (int u = 0; u < U; ++u) {
    (void)hipSetDevice(m->dev[u / m->S]);
    for (int s = 0; s < 2; ++s) {
      if (m->cdone[s][u]) (void)hipEventDestroy(m->cdone[s][u]);
      if (m->kbuf[s][u]) (void)hipFree(m->kbuf[s][u]);
      if (m->dbuf[s][u]) (void)hipFree(m->dbuf[s][u]);
      if (m->doff[s][u]) (void)hipFree(m->doff[s][u]);
      if (m->hoff[s][u]) (void)hipHostFree(m->hoff[s][u]);
    }
    if (m->ctx[u]) (void)sift_ctx_destroy(m->ctx[u]);
  }
  for (int i = 0; i < (int)m->gstream.size(); ++i) {
    (void)hipSetDevice(m->dev[i]);
    for (int s = 0; s < 2; ++s)
      if (m->gdone[s][i]) (void)hipEventDestroy(m->gdone[s][i]);
    if (m->gstream[i]) (void)hipStreamDestroy(m->gstream[i]);
  }
  if (m->n > 0) {
    (void)hipSetDevice(m->dev[0]);
    if (m->rk) (void)hipFree(m->rk);
    if (m->rd) (void)hipFree(m->rd);
  }
  delete m;
  return SIFT_OK;
}

int sift_multi_create(const int* devices, int n_devices, int max_rows, int max_cols, int max_batch_per_device,
                      unsigned flags, int streams_per_device, int kp_cap_per_device, int gather_desc,
                      sift_multi** out) {
  if (!out) return SIFT_E_INVALID;
  *out = nullptr;
  if (!devices || n_devices < 1 || max_batch_per_device < 1 || kp_cap_per_device < 1 || streams_per_device < 0 ||
      streams_per_device > 8)
    return SIFT_E_INVALID;
  for (int i = 0; i < n_devices; ++i)
    for (int j = 0; j < i; ++j)
      if (devices[j] == devices[i]) return SIFT_E_INVALID;  // RCCL: one rank per device
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return SIFT_E_HIP;
  for (int i = 0; i < n_devices; ++i)
    if (devices[i] < 0 || devices[i] >= ndev) return SIFT_E_INVALID;
  if ((long long)kp_cap_per_device * n_devices > (1ll << 31) - 1) return SIFT_E_INVALID;
  sift_multi* m = new sift_multi;
  m->n = n_devices;
  // default 2 sub-batches per device (bench.py's split); never more than images
  m->S = std::max(1, std::min(streams_per_device ? streams_per_device : 2, max_batch_per_device));
  const int U = n_devices * m->S;
  m->dev.assign(devices, devices + n_devices);
  m->max_batch = max_batch_per_device;
  m->cap = (kp_cap_per_device + m->S - 1) / m->S;
  m->gather_desc = gather_desc ? 1 : 0;
  m->self_p2p = (flags & SIFT_MULTI_SELF_P2P) != 0;
  flags &= ~SIFT_MULTI_SELF_P2P;  // not a context flag
  m->ctx.assign(U, nullptr);
  m->gstream.assign(n_devices, nullptr);
  for (int s = 0; s < 2; ++s) {
    m->gdone[s].assign(n_devices, nullptr);
    m->cdone[s].assign(U, nullptr);
    m->kbuf[s].assign(U, nullptr);
    m->dbuf[s].assign(U, nullptr);
    m->doff[s].assign(U, nullptr);
    m->hoff[s].assign(U, nullptr);
    m->cnt[s].assign(U, 0);
  }
  auto bail = [&](int rc, const std::string& msg) {
    // the message outlives m: there is no context to hold it, so it is printed
    fprintf(stderr, "sift_multi_create: %s\n", msg.c_str());
    sift_multi_destroy(m);
    return rc;
  };
  const int sub_batch = (max_batch_per_device + m->S - 1) / m->S;
  for (int i = 0; i < n_devices; ++i) {
    if (hipSetDevice(devices[i]) != hipSuccess ||
        hipStreamCreateWithFlags(&m->gstream[i], hipStreamNonBlocking) != hipSuccess)
      return bail(SIFT_E_HIP, "gather stream");
    for (int s = 0; s < 2; ++s)
      // slot s starts free: gdone[s] complete
      if (hipEventCreateWithFlags(&m->gdone[s][i], hipEventDisableTiming) != hipSuccess ||
          hipEventRecord(m->gdone[s][i], m->gstream[i]) != hipSuccess)
        return bail(SIFT_E_HIP, "event");
    for (int j = 0; j < m->S; ++j) {
      const int u = i * m->S + j;
      int rc = sift_ctx_create(devices[i], max_rows, max_cols, sub_batch, flags, &m->ctx[u]);
      if (rc) return bail(rc, "sift_ctx_create on device " + std::to_string(devices[i]) + " failed");
      if (hipSetDevice(devices[i]) != hipSuccess) return bail(SIFT_E_HIP, "hipSetDevice");
      for (int s = 0; s < 2; ++s)
        if (hipEventCreateWithFlags(&m->cdone[s][u], hipEventDisableTiming) != hipSuccess ||
            hipMalloc(&m->kbuf[s][u], sizeof(sift_keypoint) * (size_t)m->cap) != hipSuccess ||
            hipMalloc(&m->dbuf[s][u], sizeof(float) * SIFT_DESC_LEN * (size_t)m->cap) != hipSuccess ||
            hipMalloc(&m->doff[s][u], sizeof(int) * (size_t)(sub_batch + 1)) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&m->hoff[s][u]), sizeof(int) * (size_t)(sub_batch + 1),
                          hipHostMallocDefault) != hipSuccess)
          return bail(SIFT_E_NOMEM, "per-context result slots");
    }
  }
  if (hipSetDevice(devices[0]) != hipSuccess ||
      hipMalloc(&m->rk, sizeof(sift_keypoint) * (size_t)m->cap * U) != hipSuccess ||
      (m->gather_desc && hipMalloc(&m->rd, sizeof(float) * SIFT_DESC_LEN * (size_t)m->cap * U) != hipSuccess))
    return bail(SIFT_E_NOMEM, "device-0 gather buffers");
  m->comm.assign(n_devices, nullptr);
  const ncclResult_t r = ncclCommInitAll(m->comm.data(), n_devices, devices);
  if (r != ncclSuccess) {
    m->comm.clear();  // ncclCommInitAll leaves nothing to destroy on failure
    return bail(SIFT_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
  }
  *out = m;
  return SIFT_OK;
}

sift_ctx* sift_multi_context(sift_multi* m, int index) {
  if (!m || index < 0 || index >= m->n) return nullptr;
  return m->ctx[index * m->S];
}

int sift_multi_set_octaves(sift_multi* m, int n_octaves) {
  if (!m) return SIFT_E_INVALID;
  for (sift_ctx* c : m->ctx) {
    const int rc = sift_set_octaves(c, n_octaves);
    if (rc) return mfail(m, rc, sift_last_error(c));
  }
  return SIFT_OK;
}

int sift_multi_set_flags(sift_multi* m, unsigned flags) {
  if (!m) return SIFT_E_INVALID;
  for (sift_ctx* c : m->ctx) {
    const int rc = sift_set_flags(c, flags);
    if (rc) return mfail(m, rc, sift_last_error(c));
  }
  return SIFT_OK;
}

static int step_impl(sift_multi* m, const float* const* d_imgs, const int* counts, int rows, int cols, size_t row_stride,
              size_t img_stride);
static int flush_impl(sift_multi* m);

int sift_multi_step(sift_multi* m, const float* const* d_imgs, const int* counts, int rows, int cols,
                    size_t row_stride, size_t img_stride) {
  if (!m) return SIFT_E_INVALID;
  if (!m->broken.empty()) return mfail(m, SIFT_E_INVALID, "a previous step failed (" + m->broken + "): destroy the multi context");
  if (!d_imgs || !counts) return mfail(m, SIFT_E_INVALID, "null argument");
  for (int i = 0; i < m->n; ++i)
    if (counts[i] < 0 || counts[i] > m->max_batch || (counts[i] > 0 && !d_imgs[i]))
      return mfail(m, SIFT_E_INVALID, "shard " + std::to_string(i) + ": bad image count or null buffer");
  const int rc = step_impl(m, d_imgs, counts, rows, cols, row_stride, img_stride);
  if (rc) m->broken = m->err;
  return rc;
}

int sift_multi_flush(sift_multi* m) {
  if (!m) return SIFT_E_INVALID;
  if (!m->broken.empty()) return mfail(m, SIFT_E_INVALID, "a previous step failed (" + m->broken + "): destroy the multi context");
  const int rc = flush_impl(m);
  // the contexts' sticky device errors (sift_sync) leave every stream drained and the slots consistent
  if (rc && m->pending) m->broken = m->err;
  return rc;
}

static int step_impl(sift_multi* m, const float* const* d_imgs, const int* counts, int rows, int cols, size_t row_stride,
              size_t img_stride) {
  const int s = (int)(m->steps & 1), p = s ^ 1;
  for (int i = 0; i < m->n; ++i)
    for (int j = 0; j < m->S; ++j) {
      const int u = i * m->S + j;
      const int first = (int)((long long)j * counts[i] / m->S);
      const int c = (int)((long long)(j + 1) * counts[i] / m->S) - first;
      MHIP(m, hipSetDevice(m->dev[i]));
      hipStream_t cs = (hipStream_t)sift_get_stream(m->ctx[u]);
      MHIP(m, hipStreamWaitEvent(cs, m->gdone[s][i], 0));  // step k - 2's gather has read slot s
      m->cnt[s][u] = c;
      if (c > 0) {
        const int rc = sift_detect_compute_batch(m->ctx[u], d_imgs[i] + (size_t)first * img_stride, c, rows, cols,
                                                 row_stride, img_stride, m->kbuf[s][u], m->dbuf[s][u], m->cap,
                                                 m->doff[s][u]);
        if (rc) return mfail(m, rc, "device " + std::to_string(m->dev[i]) + ": " + sift_last_error(m->ctx[u]));
        MHIP(m, hipMemcpyAsync(m->hoff[s][u], m->doff[s][u], sizeof(int) * (size_t)(c + 1), hipMemcpyDeviceToHost,
                               cs));
      }
      MHIP(m, hipEventRecord(m->cdone[s][u], cs));
    }
  ++m->steps;
  if (m->pending) {
    const int rc = gather_slot(m, p);
    if (rc) return rc;
    m->gathered = m->steps - 2;
  }
  m->pending = true;
  return SIFT_OK;
}

static int flush_impl(sift_multi* m) {
  if (m->pending) {
    const int rc = gather_slot(m, (int)((m->steps - 1) & 1));
    if (rc) return rc;
    m->gathered = m->steps - 1;
    m->pending = false;
  }
  for (int i = 0; i < m->n; ++i) {
    MHIP(m, hipSetDevice(m->dev[i]));
    MHIP(m, hipStreamSynchronize(m->gstream[i]));
  }
  for (int u = 0; u < (int)m->ctx.size(); ++u) {
    const int rc = sift_sync(m->ctx[u]);  // the sticky device status of every step
    if (rc) return mfail(m, rc, "device " + std::to_string(m->dev[u / m->S]) + ": " + sift_last_error(m->ctx[u]));
  }
  return SIFT_OK;
}

int sift_multi_gathered(sift_multi* m, const sift_keypoint** d_kpts, const float** d_desc, int* offsets,
                        int offsets_cap, int* batch_total, long long* step) {
  if (!m) return SIFT_E_INVALID;
  if (m->gathered < 0) return mfail(m, SIFT_E_INVALID, "no step gathered yet (sift_multi_flush)");
  const int slot = (int)(m->gathered & 1);
  // the gather that wrote rk / rd has finished on device 0
  MHIP(m, hipSetDevice(m->dev[0]));
  MHIP(m, hipEventSynchronize(m->gdone[slot][0]));
  const int bt = (int)m->goff.size() - 1;
  if (batch_total) *batch_total = bt;
  if (step) *step = m->gathered;
  if (d_kpts) *d_kpts = m->rk;
  if (d_desc) *d_desc = m->gather_desc ? m->rd : nullptr;
  if (offsets) {
    if (offsets_cap < bt + 1) return mfail(m, SIFT_E_CAPACITY, "offsets_cap < batch_total + 1");
    std::copy(m->goff.begin(), m->goff.end(), offsets);
  }
  return SIFT_OK;
}

int sift_multi_copy_gathered(sift_multi* m, sift_keypoint* kpts, float* desc, int cap, int* n_out) {
  if (!m || !n_out) return SIFT_E_INVALID;
  const sift_keypoint* dk = nullptr;
  const float* dd = nullptr;
  int bt = 0;
  int rc = sift_multi_gathered(m, &dk, &dd, nullptr, 0, &bt, nullptr);
  if (rc) return rc;
  const int n = m->goff.back();
  *n_out = n;
  if (n > cap) return mfail(m, SIFT_E_CAPACITY, "cap " + std::to_string(cap) + " < " + std::to_string(n));
  if (n == 0) return SIFT_OK;
  if (!kpts) return mfail(m, SIFT_E_INVALID, "null keypoint buffer");
  MHIP(m, hipSetDevice(m->dev[0]));
  MHIP(m, hipMemcpy(kpts, dk, sizeof(sift_keypoint) * (size_t)n, hipMemcpyDeviceToHost));
  if (desc) {
    if (!dd) return mfail(m, SIFT_E_INVALID, "descriptors were not gathered (gather_desc = 0)");
    MHIP(m, hipMemcpy(desc, dd, sizeof(float) * SIFT_DESC_LEN * (size_t)n, hipMemcpyDeviceToHost));
  }
  return SIFT_OK;
}

int sift_multi_stats(const sift_multi* m, long long* steps, long long* records, long long* transfers) {
  if (!m) return SIFT_E_INVALID;
  if (steps) *steps = m->steps;
  if (records) *records = m->records;
  if (transfers) *transfers = m->transfers;
  return SIFT_OK;
}

int sift_multi_rccl_version(void) {
  int v = 0;
  return ncclGetVersion(&v) == ncclSuccess ? v : -1;
}

}  // extern "C"
