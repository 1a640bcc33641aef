#!/usr/bin/env python3
"""Minimal sift_ctx_pair run: two contexts, two streams, a few alternating
batch calls; prints each step so a native fault names its call."""
import faulthandler
import sys

import torch

sys.path.insert(0, "sift-gpu_amd")
import siftgpu  # noqa: E402

faulthandler.enable()
R, C, NB = 1080, 1920, int(sys.argv[1]) if len(sys.argv) > 1 else 4
imgs = torch.empty((2 * NB, R, C), dtype=torch.float32, device="cuda")
ctxs, outs, streams = [], [], []
for p in range(2):
    s = torch.cuda.Stream()
    c = siftgpu.Context(R, C, NB, device=0)
    c.set_stream(s.cuda_stream)
    streams.append(s)
    ctxs.append(c)
    cap = NB * 40000
    outs.append((torch.empty((cap, 7), dtype=torch.int32, device="cuda"),
                 torch.empty((cap, 128), dtype=torch.float32, device="cuda"),
                 torch.empty((NB + 1,), dtype=torch.int32, device="cuda"), cap))
ctxs[0].synth_images(imgs.data_ptr(), 2 * NB, R, C, C, R * C, seed_base=0)
torch.cuda.synchronize()
print("created", flush=True)
mode = sys.argv[2] if len(sys.argv) > 2 else "pair"
if mode == "pair":
    ctxs[0].pair(ctxs[1])
    print("paired", flush=True)
if len(sys.argv) > 3:
    for c in ctxs:
        c.set_flags(int(sys.argv[3]))
for step in range(3):
    for p in range(2):
        k, d, o, cap = outs[p]
        with torch.cuda.stream(streams[p]):
            ctxs[p].detect_compute_batch(imgs[p * NB].data_ptr(), NB, R, C, C, R * C, k.data_ptr(), d.data_ptr(),
                                         cap, o.data_ptr())
        print("step", step, "part", p, "enqueued", flush=True)
torch.cuda.synchronize()
for c in ctxs:
    c.sync()
print("synced", [int(o[2][-1].item()) for o in outs], flush=True)
for c in ctxs:
    c.close()
print("closed", flush=True)
