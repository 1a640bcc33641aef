"""The bench's N > 1 gather (sift-gpu_amd/sift_dist.py) on the GPU with the
"nccl" backend (RCCL): a one-rank process group on the test box's device, so
the code path bench.py runs at N > 1 -- pinned offset copies, the gloo
metadata group beside the nccl group, the side stream and its events, the
transfer timing -- executes on hardware with RCCL initialised, and one RCCL
collective runs.  (Two ranks cannot share one device under RCCL, so the p2p
transfers themselves run only on a multi-GPU node; test_distributed.py covers
them at world 2 over gloo.)"""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sift-gpu_amd")

_CHILD = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
import siftgpu, sift_dist
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
x = torch.ones(4, device="cuda")
dist.all_reduce(x)                                   # one RCCL collective
assert x.tolist() == [1.0] * 4
R, C, B, cap = 240, 320, 3, 20000
ctx = siftgpu.Context(R, C, B, device=0)
strm = torch.cuda.Stream()
ctx.set_stream(strm.cuda_stream)
imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, seed_base=5)
bufs = [(torch.empty((cap, 7), dtype=torch.int32, device="cuda"), torch.empty((cap, 128), device="cuda"),
         torch.empty((B + 1,), dtype=torch.int32, device="cuda")) for _ in range(2)]
got = []
def on_result(step, out):
    ks, offs, ds = out
    got.append((step, ks[0].cpu().numpy().copy(), offs[0].numpy().copy(), ds[0].cpu().numpy().copy()))
pipe = sift_dist.GatherPipeline([B], cap, dst=0, timing=True)
run = sift_dist.PipelinedSteps(pipe, bufs, with_desc=True, on_result=on_result)
def compute(k, d, o):
    ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, k.data_ptr(), d.data_ptr(), cap, o.data_ptr())
with torch.cuda.stream(strm):
    for _ in range(3):
        run.step(compute)
    run.flush()
torch.cuda.synchronize()
ctx.sync()
st = pipe.stats()
assert [g[0] for g in got] == [0, 1, 2] and st["gathers"] == 3 and st["backend"] == "nccl", st
assert st["transfer_ms"] is not None
ref = siftgpu.Context(R, C, B, device=0)
k, d, o = (torch.empty_like(t) for t in bufs[0])
ref.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, k.data_ptr(), d.data_ptr(), cap, o.data_ptr())
ref.sync()
n = int(o[B].item())
for step, ks, offs, ds in got:
    assert offs.tolist() == o.cpu().tolist(), step
    assert ks.tobytes() == k[:n].cpu().numpy().tobytes() and ds.tobytes() == d[:n].cpu().numpy().tobytes(), step
ctx.close(); ref.close()
dist.destroy_process_group()
print("nccl gather ok", n, "records per step", st)
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_bench_gather_path_on_rccl_world1():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    r = subprocess.run([sys.executable, "-c", _CHILD, PKG], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "nccl gather ok" in r.stdout
