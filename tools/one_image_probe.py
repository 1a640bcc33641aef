#!/usr/bin/env python3
"""Device latency of one synthetic image of a given size (exact mode, graph
replay, image resident in HBM): the A/B probe for the one-image kernel
variants' size limit (SIFT_HIP_ONE_IMAGE_PX, common.hpp kOneImagePx).
  python tools/one_image_probe.py ROWS COLS [--octaves 5] [--reps 20] [--tag T]"""
import argparse
import json
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
    p.add_argument("rows", type=int)
    p.add_argument("cols", type=int)
    p.add_argument("--octaves", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--tag", default="")
    a = p.parse_args()
    R, C = a.rows, a.cols
    with siftgpu.Context(R, C, 1, device=0) as ctx:
        ctx.set_octaves(a.octaves)
        img = torch.empty((1, R, C), dtype=torch.float32, device="cuda")
        ctx.synth_images(img.data_ptr(), 1, R, C, C, R * C, seed_base=0)
        cap = 1 << 20
        kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((2,), dtype=torch.int32, device="cuda")

        def call():
            ctx.detect_compute_batch(img.data_ptr(), 1, R, C, C, R * C, kpts.data_ptr(), desc.data_ptr(), cap,
                                     offs.data_ptr())
            ctx.sync()
        for _ in range(3):
            call()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
        n = int(offs[1].item())
    print(json.dumps({"tag": a.tag, "rows": R, "cols": C, "keypoints": n,
                      "latency_ms": round(float(np.median(ts)) * 1e3, 4)}), flush=True)


if __name__ == "__main__":
    main()
