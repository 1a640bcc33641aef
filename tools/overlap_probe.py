#!/usr/bin/env python3
"""Probe: does splitting the batch over S contexts on S HIP streams overlap
their stages (blur VALU vs extrema HBM vs orientation LDS)?  Times K steps of
64 x 1080p as 1 x 64 and as S x (64/S) on S streams.

  python tools/overlap_probe.py [--splits 2 4] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-gpu_amd"))
import siftgpu  # noqa: E402


def run(split, B, R, C, steps, warmup, fast, same):
    n = B // split
    streams = [torch.cuda.Stream() for _ in range(1 if same else split)]
    flags = siftgpu.SIFT_FLAG_FAST if fast else 0
    ctxs, bufs = [], []
    for s in range(split):
        ctx = siftgpu.Context(R, C, n, flags=flags)
        ctx.set_stream(streams[0 if same else s].cuda_stream)
        imgs = torch.empty((n, R, C), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), n, R, C, C, R * C, s * n)
        cap = n * 40000
        kp = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        de = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        of = torch.empty((n + 1,), dtype=torch.int32, device="cuda")
        ctxs.append(ctx)
        bufs.append((imgs, kp, de, of, cap))

    def step():
        for ctx, (imgs, kp, de, of, cap) in zip(ctxs, bufs):
            ctx.detect_compute_batch(imgs.data_ptr(), n, R, C, C, R * C, kp.data_ptr(), de.data_ptr(), cap,
                                     of.data_ptr())

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    nkp = sum(int(b[3][-1].item()) for b in bufs)
    for c in ctxs:
        c.close()
    return dt, nkp


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--fast", action="store_true")
    p.add_argument("--same-stream", action="store_true", help="all contexts on one stream (batch-size effect only)")
    a = p.parse_args()
    B, R, C = 64, 1080, 1920
    for s in a.splits:
        dt, nkp = run(s, B, R, C, a.steps, 2, a.fast, a.same_stream)
        print(json.dumps({"split": s, "fast": a.fast, "same_stream": a.same_stream, "ms_per_step": round(dt * 1e3, 3),
                          "mpix_s": round(B * R * C / dt / 1e6, 1), "keypoints": nkp}), flush=True)


if __name__ == "__main__":
    main()
