#!/usr/bin/env python3
"""configs[1] single-image loop for kernel traces: one 1080p image resident in
HBM, 4 octaves, sift_detect_compute_batch(batch 1) (graph replay) + sift_sync,
--reps times; prints the median latency.
  rocprofv3 --kernel-trace --stats -d <dir> -o run -- python3 tools/single_trace.py"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-gpu_amd"))
import siftgpu  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--flags", type=int, default=0)
    p.add_argument("--rows", type=int, default=1080)
    p.add_argument("--cols", type=int, default=1920)
    p.add_argument("--octaves", type=int, default=4)
    p.add_argument("--cap", type=int, default=40000)
    a = p.parse_args()
    R, C = a.rows, a.cols
    with siftgpu.Context(R, C, 1, device=0) as ctx:
        ctx.set_octaves(a.octaves)
        ctx.set_flags(a.flags)
        img = torch.empty((1, R, C), dtype=torch.float32, device="cuda")
        ctx.synth_images(img.data_ptr(), 1, R, C, C, R * C, seed_base=0)
        cap = a.cap
        kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((2,), dtype=torch.int32, device="cuda")
        ts = []
        for i in range(a.reps + 3):
            t0 = time.perf_counter()
            ctx.detect_compute_batch(img.data_ptr(), 1, R, C, C, R * C, kpts.data_ptr(), desc.data_ptr(), cap,
                                     offs.data_ptr())
            ctx.sync()
            if i >= 3:
                ts.append(time.perf_counter() - t0)
        n = int(offs[1].item())
        h = int(desc[:n].contiguous().view(torch.int32).to(torch.int64).mul_(
            torch.arange(1, n * 128 + 1, device="cuda", dtype=torch.int64).view(n, 128)).sum().item())
        print(f'{{"latency_ms": {np.median(ts) * 1e3:.4f}, "keypoints": {n}, "desc_hash": {h}}}', flush=True)


if __name__ == "__main__":
    main()
