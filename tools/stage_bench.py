#!/usr/bin/env python3
"""Per-stage device times of the batch pipeline (HIP events), for A/B work.

  python tools/stage_bench.py [--batch 64] [--rows 1080 --cols 1920] [--reps 3]

Runs the whole SIFT_NCL batch path on device-resident synthetic images with
SIFT_FLAG_PROFILE and prints ms per stage per step.  Environment switches read
by the library (e.g. SIFT_HIP_DESC_V1=1) select kernel variants, so several
invocations in one gpurun call compare variants on the same device.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-gpu_amd"))
import siftgpu  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--rows", type=int, default=1080)
    p.add_argument("--cols", type=int, default=1920)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--tag", default="")
    p.add_argument("--fast", action="store_true", help="SIFT_FLAG_FAST pyramid")
    p.add_argument("--ignore-status", action="store_true",
                   help="ablation runs: ignore capacity overflows of garbage planes")
    a = p.parse_args()
    B, R, C = a.batch, a.rows, a.cols
    ctx = siftgpu.Context(R, C, B, flags=siftgpu.SIFT_FLAG_PROFILE | (siftgpu.SIFT_FLAG_FAST if a.fast else 0))
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, 0)
    cap = B * 40000
    kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
    offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")

    def run():
        ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kpts.data_ptr(), desc.data_ptr(), cap,
                                 offs.data_ptr())

    def sync():
        try:
            ctx.sync()
        except siftgpu.SiftError:
            if not a.ignore_status:
                raise

    run()
    sync()
    ctx.stage_stats(reset=True)
    for _ in range(a.reps):
        run()
    sync()
    st = ctx.stage_stats(reset=True)
    total = sum(v["ms"] for v in st.values()) / a.reps
    out = {"tag": a.tag, "batch": B, "shape": [R, C], "keypoints": int(offs[-1].item()),
           "total_ms": round(total, 3),
           "stages_ms": {k: round(v["ms"] / a.reps, 3) for k, v in st.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
