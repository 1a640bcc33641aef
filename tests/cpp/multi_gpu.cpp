// configs[3] from a C++ host through the C ABI (include/sift_hip.h,
// sift_multi_*): the images of each step are sharded over the visible GPUs
// (64 x 1920x1080 per device by default: 512 on an 8-GPU node), every device
// detects + describes its shard, and the keypoint records are gathered to the
// first device over RCCL one step behind.  Prints one JSON line.
//
//   multi_gpu [--devices N] [--per-device B] [--steps K] [--warmup W] [--rows R --cols C]
//             [--streams S]   (contexts / HIP streams per device, default 2)
//
// Built by tests/test_abi.py (g++, HIP runtime API only) and run at N = 1 by
// tests/test_multi.py on the GPU box; INTEGRATION.md section 4 walks through it.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sift_hip.h"

#define CHECK(call)                                                                   \
  do {                                                                                \
    int rc_ = (call);                                                                 \
    if (rc_ != SIFT_OK) {                                                             \
      fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, m ? sift_multi_last_error(m) : ""); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

int main(int argc, char** argv) {
  int ndev = 0, per = 64, steps = 5, warmup = 2, rows = 1080, cols = 1920, streams = 2;
  for (int i = 1; i + 1 < argc; i += 2) {
    const int v = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--devices")) ndev = v;
    else if (!strcmp(argv[i], "--per-device")) per = v;
    else if (!strcmp(argv[i], "--steps")) steps = v;
    else if (!strcmp(argv[i], "--warmup")) warmup = v;
    else if (!strcmp(argv[i], "--rows")) rows = v;
    else if (!strcmp(argv[i], "--cols")) cols = v;
    else if (!strcmp(argv[i], "--streams")) streams = v;
  }
  int visible = 0;
  if (hipGetDeviceCount(&visible) != hipSuccess || visible < 1) {
    fprintf(stderr, "no HIP device\n");
    return 2;
  }
  if (ndev <= 0 || ndev > visible) ndev = visible;
  std::vector<int> devs(ndev);
  for (int i = 0; i < ndev; ++i) devs[i] = i;
  sift_multi* m = nullptr;
  const int kp_cap = per * 40000;  // ~3x a textured 1080p image's keypoints
  CHECK(sift_multi_create(devs.data(), ndev, rows, cols, per, 0, streams, kp_cap, 0, &m));
  // every device synthesises its own shard of the global batch (image b of
  // the step has seed b): the images are resident in that device's HBM
  std::vector<float*> imgs(ndev, nullptr);
  std::vector<int> counts(ndev, 0);
  const size_t plane = (size_t)rows * cols;
  for (int i = 0; i < ndev; ++i) {
    int first = 0;
    CHECK(sift_multi_shard(per * ndev, ndev, i, &first, &counts[i]));
    if (hipSetDevice(devs[i]) != hipSuccess || hipMalloc(&imgs[i], plane * sizeof(float) * counts[i]) != hipSuccess) {
      fprintf(stderr, "image buffers\n");
      return 1;
    }
    CHECK(sift_synth_images(sift_multi_context(m, i), imgs[i], counts[i], rows, cols, cols, plane, first));
  }
  for (int i = 0; i < ndev; ++i) {  // the images are ready before any context reads them
    (void)hipSetDevice(devs[i]);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
  }
  const float* const* ip = imgs.data();
  for (int s = 0; s < warmup; ++s) CHECK(sift_multi_step(m, ip, counts.data(), rows, cols, cols, plane));
  CHECK(sift_multi_flush(m));
  const auto t0 = std::chrono::steady_clock::now();
  for (int s = 0; s < steps; ++s) CHECK(sift_multi_step(m, ip, counts.data(), rows, cols, cols, plane));
  CHECK(sift_multi_flush(m));  // the last step's gather is part of the timed work
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int batch_total = 0;
  long long step = 0;
  std::vector<int> offs(per * ndev + 1);
  CHECK(sift_multi_gathered(m, nullptr, nullptr, offs.data(), (int)offs.size(), &batch_total, &step));
  long long st = 0, rec = 0, tr = 0;
  CHECK(sift_multi_stats(m, &st, &rec, &tr));
  const double mpix = (double)steps * per * ndev * plane / 1e6;
  printf("{\"devices\": %d, \"images_per_step\": %d, \"steps\": %d, \"ms_per_step\": %.3f, \"Mpix_per_s\": %.1f, "
         "\"keypoints_per_s\": %.1f, \"gathered_keypoints_last_step\": %d, \"image0_keypoints\": %d, "
         "\"rccl_version\": %d, \"p2p_transfers\": %lld, \"streams_per_device\": %d}\n",
         ndev, per * ndev, steps, sec / steps * 1e3, mpix / sec, (double)offs[batch_total] * steps / sec,
         offs[batch_total], offs[1] - offs[0], sift_multi_rccl_version(), tr, streams);
  for (int i = 0; i < ndev; ++i) {
    (void)hipSetDevice(devs[i]);
    (void)hipFree(imgs[i]);
  }
  CHECK(sift_multi_destroy(m));
  return 0;
}
