#!/usr/bin/env python3
"""Per-wave wait split of pyr_pc_kernel from the stamps build
(tools/patches/pc_stamps.patch, built by tools/build_patch.sh pcstamps ...).

  python tools/pc_stamps.py [--lib sift-gpu_amd/lib/libsift_hip_pcstamps.so] [--reps 5]

Runs the SIFT_FLAG_FAST pyramid of configs[2] (64 x 1920x1080, device-resident
synthetic images; --shape 1x4320x7680 for configs[4]) and prints, per octave and wave (producer, w18, w12,
w8+w4), the average cycles per wave and per step and the share of the wave's
lifetime spent in its LDS-counter waits (producer: for the slowest consumer
to free a ring slot; consumers: for the producer to publish a step), with the
fraction of waits that had to poll at least once.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-gpu_amd"))
import siftgpu  # noqa: E402

WAVES = ["producer", "w18", "w12", "w8+w4"]
NBLK = 16384


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=os.path.join(ROOT, "sift-gpu_amd", "lib", "libsift_hip_pcstamps.so"))
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--json", default="")
    p.add_argument("--shape", default="64x1080x1920", help="BxROWSxCOLS (configs[4]: 1x4320x7680)")
    a = p.parse_args()
    siftgpu.LIB_PATH = a.lib
    siftgpu._lib = None
    B, R, C = (int(v) for v in a.shape.split("x"))
    ctx = siftgpu.Context(R, C, B, flags=siftgpu.SIFT_FLAG_PROFILE | siftgpu.SIFT_FLAG_FAST)
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, 0)
    cap = max(B * 40000, 1 << 20)
    kp = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
    de = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
    off = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
    L = siftgpu.lib()
    dbg = L.sift_dbg_pc_stamps
    dbg.restype = ctypes.c_int
    dbg.argtypes = [ctypes.c_void_p, ctypes.c_int]

    def run():
        ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kp.data_ptr(), de.data_ptr(), cap,
                                 off.data_ptr())
    for _ in range(3):
        run()
    ctx.sync()
    ctx.stage_stats(reset=True)
    torch.cuda.synchronize()
    dbg(None, 1)
    for _ in range(a.reps):
        run()
    ctx.sync()
    st = ctx.stage_stats(reset=True)
    ms = st["pyramid_fast"]["ms"] / a.reps
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (5 * NBLK * 4 * 4))()
    assert dbg(buf, 0) > 0
    arr = np.frombuffer(buf, dtype=np.uint64).reshape(5, NBLK, 4, 4).astype(np.float64)
    print(f"stamps build: pyramid {ms:.3f} ms per step ({a.reps} reps)")
    out = {"pyramid_ms_stamps": ms, "rows": []}
    print(f"{'octave':>6s} {'wave':>9s} {'waves':>7s} {'cyc/wave':>9s} {'cyc/step':>9s} {'wait share':>10s} "
          f"{'waits that polled':>17s}")
    for o in range(5):
        for w in range(4):
            v = arr[o, :, w, :]
            nw = int((v[:, 3] > 0).sum())
            tot, wait, nwait, steps = v[:, 0].sum(), v[:, 1].sum(), v[:, 2].sum(), v[:, 3].sum()
            if not nw:
                continue
            row = {"octave": o, "wave": WAVES[w], "waves": nw, "cycles_per_wave": tot / nw,
                   "cycles_per_step": tot / max(steps, 1), "wait_share": wait / max(tot, 1),
                   "polled_share": nwait / max(steps, 1)}
            out["rows"].append(row)
            print(f"{o:6d} {WAVES[w]:>9s} {nw:7d} {row['cycles_per_wave']:9.0f} {row['cycles_per_step']:9.0f} "
                  f"{row['wait_share']:10.3f} {row['polled_share']:17.3f}")
    ctx.close()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
