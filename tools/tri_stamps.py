#!/usr/bin/env python3
"""Per-wave-role time split of pyr_tri_kernel from the stamps build
(tools/patches/tri_stamps.patch, built by tools/build_patch.sh stamps ...).

  python tools/tri_stamps.py [--lib sift-gpu_amd/lib/libsift_hip_stamps.so] [--reps 5]

Runs the SIFT_FLAG_FAST pyramid of configs[2] (64 x 1920x1080, device-resident
synthetic images), reads the per-(octave, role, segment) s_memtime sums and
prints, per octave and role, the average cycles per step in each segment and
its share of the wave's lifetime.  Segments (stamp order within a step; round-5 form of the shipped kernel):
  vmwait  s_waitcnt vmcnt(N) for the step's own LDS-DMA source rows (io roles;
          on gfx9 it also waits for every older store)
  bar     the step's one s_barrier (LDS drained by the stamp before it)
  dma     issuing the next step's LDS-DMA source rows (io roles)
  base    octave 0: base blur one step ahead -- row pass, wave sync, column
          pass, LDS base rows, plane-0 transpose + stores (io roles)
  row     row pass of the role's scales (LDS window reads, FMAs, h writes), 2 rounds
  xpose   wave syncs + column reads of the h rows, 2 rounds
  col     column-pass FMAs (register scatter)
  stx     store transposes through the h rows (writes, sync, b128 reads), 2 rounds
  store   plane store issue (dwordx4 / dwordx2), 2 rounds
  loop    loop overhead between steps
Each stamp is s_memtime behind s_waitcnt lgkmcnt(0), so a segment's own LDS
latency is charged to it and the instrumented kernel runs slower than the
product one (both times are printed).
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-gpu_amd"))
import siftgpu  # noqa: E402

SEGS = ["vmwait", "bar", "dma", "base", "row", "xpose", "col", "stx", "store", "loop"]
K_TOTAL, K_STEPS, K_LIVE, K_WAVES, NSEG = 12, 13, 14, 15, 16
ROLES = ["role0 w18", "role1 w12+io", "role2 w8,w4+io+dec"]


def pyramid_ms(lib_path, B, R, C, reps, want_stamps):
    siftgpu.LIB_PATH = lib_path
    siftgpu._lib = None
    ctx = siftgpu.Context(R, C, B, flags=siftgpu.SIFT_FLAG_PROFILE | siftgpu.SIFT_FLAG_FAST)
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, 0)
    cap = B * 40000
    kp = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
    de = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
    off = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
    L = siftgpu.lib()
    buf = (ctypes.c_ulonglong * (5 * 16384 * 3 * NSEG))()
    dbg = getattr(L, "sift_dbg_tri_stamps", None) if want_stamps else None
    if dbg:
        dbg.restype = ctypes.c_int
        dbg.argtypes = [ctypes.c_void_p, ctypes.c_int]

    def run():
        ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kp.data_ptr(), de.data_ptr(), cap,
                                 off.data_ptr())

    for _ in range(3):
        run()
    ctx.sync()
    ctx.stage_stats(reset=True)
    if dbg:
        torch.cuda.synchronize()
        dbg(None, 1)
    for _ in range(reps):
        run()
    ctx.sync()
    st = ctx.stage_stats(reset=True)
    ms = st["pyramid_fast"]["ms"] / reps
    stamps = None
    if dbg:
        torch.cuda.synchronize()
        assert dbg(buf, 0) > 0
        import numpy as np
        arr = np.frombuffer(buf, dtype=np.uint64).reshape(5, 16384, 3, NSEG).sum(axis=1)
        stamps = [[[int(arr[o, r, k]) for k in range(NSEG)] for r in range(3)] for o in range(5)]
    ctx.close()
    return ms, stamps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=os.path.join(ROOT, "sift-gpu_amd", "lib", "libsift_hip_stamps.so"))
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--json", default="")
    a = p.parse_args()
    B, R, C = 64, 1080, 1920
    ms, stamps = pyramid_ms(a.lib, B, R, C, a.reps, True)
    print(f"stamps build: pyramid {ms:.3f} ms per step (SIFT_FLAG_PROFILE events, {a.reps} reps)")
    out = {"pyramid_ms_stamps": ms, "octaves": []}
    for o in range(5):
        print(f"\noctave {o}")
        print(f"{'role':20s} {'waves':>7s} {'steps':>6s} {'live':>5s} {'cyc/wave':>9s} " +
              " ".join(f"{s:>6s}" for s in SEGS))
        for r in range(3):
            v = stamps[o][r]
            w = max(v[K_WAVES], 1)
            steps = v[K_STEPS] / w
            tot = v[K_TOTAL] / w
            per_step = [v[k] / max(v[K_STEPS], 1) for k in range(len(SEGS))]
            share = [v[k] / max(v[K_TOTAL], 1) for k in range(len(SEGS))]
            print(f"{ROLES[r]:20s} {v[K_WAVES]:7d} {steps:6.1f} {v[K_LIVE] / w:5.1f} {tot:9.0f} " +
                  " ".join(f"{x:6.0f}" for x in per_step) + "   cyc/step")
            print(f"{'':20s} {'':7s} {'':6s} {'':5s} {'':9s} " + " ".join(f"{x:6.3f}" for x in share) +
                  "   share of wave time")
            out["octaves"].append({"octave": o, "role": r, "waves": v[K_WAVES], "steps_per_wave": steps,
                                   "cycles_per_wave": tot,
                                   "cycles_per_step": dict(zip(SEGS, per_step)),
                                   "share": dict(zip(SEGS, share))})
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
