"""world_size-2 gloo tests (CPU) of the batch-mode sharding and the keypoint
gather (sift-gpu_amd/sift_dist.py) that bench.py runs over RCCL at N > 1."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sift_dist as sdist


def test_shard_covers_every_image_once():
    for total in (1, 7, 64, 512):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                a, b = sdist.shard(total, world, r)
                assert 0 <= a <= b <= total
                seen.extend(range(a, b))
            assert seen == list(range(total))
    assert sdist.shard(512, 8, 3) == (192, 256)   # C4: 64 images per GPU


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap, batch = 50, 3
        # rank r has 10*(r+1) keypoints (rank 1 overflows nothing), image split 2/3/rest
        n = 10 * (rank + 1)
        kp = torch.full((cap, 7), -1, dtype=torch.int32)
        kp[:n] = torch.arange(n * 7, dtype=torch.int32).reshape(n, 7) + 1000 * rank
        desc = torch.zeros((cap, 128), dtype=torch.float32)
        desc[:n] = rank + 1
        offs = torch.tensor([0, 2, 5, n], dtype=torch.int32)
        out = sdist.gather_keypoints(kp, offs, dst=0, desc=desc)
        if rank == 0:
            ks, os_, ds = out
            q.put(([k.numpy().copy() for k in ks], [o.numpy().copy() for o in os_],
                   [d.numpy().copy() for d in ds]))
        else:
            assert out is None
        # zero-keypoint rank must not deadlock
        offs0 = torch.tensor([0, 0, 0, 0 if rank == 1 else 4], dtype=torch.int32)
        out = sdist.gather_keypoints(kp, offs0, dst=0)
        if rank == 0:
            q.put([k.shape[0] for k in out[0]])
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gather_keypoints_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        ks, offs, ds = q.get(timeout=120)
        shapes = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert [p.exitcode for p in procs] == [0, 0]
    assert [k.shape for k in ks] == [(10, 7), (20, 7)]
    for r, k in enumerate(ks):
        n = 10 * (r + 1)
        np.testing.assert_array_equal(k, np.arange(n * 7).reshape(n, 7) + 1000 * r)
        np.testing.assert_array_equal(offs[r], [0, 2, 5, n])
        assert np.all(ds[r] == r + 1)
    assert shapes == [4, 0]
