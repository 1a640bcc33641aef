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


def test_shard_sizes():
    assert sdist.shard_sizes(10, 4) == [2, 3, 2, 3]
    assert sdist.shard_sizes(512, 8) == [64] * 8


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
        # uneven shards: 2 images on rank 0, 3 on rank 1
        batches = [2, 3]
        b = batches[rank]
        nk = 4 + rank
        offs_u = torch.tensor([0] + [min(nk, j + 1) for j in range(b - 1)] + [nk], dtype=torch.int32)
        out = sdist.gather_keypoints(kp, offs_u, dst=0, batches=batches)
        if rank == 0:
            q.put(([k.shape[0] for k in out[0]], [o.tolist() for o in out[1]]))
        # the same without `batches`: the shard sizes are exchanged
        out = sdist.gather_keypoints(kp, offs_u, dst=0)
        if rank == 0:
            q.put(([k.shape[0] for k in out[0]], [o.tolist() for o in out[1]]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _fake_step(rank, step, cap):
    """Deterministic stand-in for one detect_compute_batch call of this rank."""
    batch = [2, 3][rank]
    per = [(step * 3 + rank * 5 + j) % 7 for j in range(batch)]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(per)]), dtype=torch.int32)
    n = int(offs[-1])
    kp = torch.arange(n * 7, dtype=torch.int32).reshape(n, 7) + 100000 * rank + 1000 * step
    desc = torch.full((n, 128), float(step * 10 + rank))
    return offs, kp, desc


def _pipeline_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap = 64
        pipe = sdist.GatherPipeline(sdist.shard_sizes(5, world), cap, dst=0)
        bufs = [(torch.zeros((cap, 7), dtype=torch.int32), torch.zeros((cap, 128)),
                 torch.zeros(4, dtype=torch.int32)) for _ in range(2)]
        got = {}

        def on_result(step, out):
            ks, offs, ds = out
            got[step] = ([k.clone() for k in ks], [o.clone() for o in offs], [d.clone() for d in ds])

        runner = sdist.PipelinedSteps(pipe, bufs, with_desc=True, on_result=on_result)
        for step in range(5):
            def compute(k, d, o, step=step):
                offs, kp, desc = _fake_step(rank, step, cap)
                o[:len(offs)] = offs
                k[:len(kp)] = kp
                d[:len(desc)] = desc
            runner.step(compute)
        runner.flush()
        st = pipe.stats()   # the bench line's N > 1 evidence
        n1 = sum(int(_fake_step(1, step, cap)[0][-1]) for step in range(5))
        ok_stats = st["gathers"] == 5 and st["world_size"] == world and st["backend"] == "gloo"
        if rank == 0:
            ok_stats = ok_stats and st["received_records_per_rank"] == [0, n1] and st["sent_records"] == 0
        else:
            ok_stats = ok_stats and st["sent_records"] == n1
        assert ok_stats, st
        if rank == 0:
            ok = sorted(got) == list(range(5))
            for step in range(5):
                for r in range(world):
                    offs, kp, desc = _fake_step(r, step, cap)
                    ks, os_, ds = got[step]
                    ok = ok and torch.equal(ks[r], kp) and torch.equal(os_[r], offs) and torch.equal(ds[r], desc)
            q.put(ok)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _parts_fake(part, rank, step, nb):
    n = 3 + part + 2 * rank + step
    offs = torch.tensor([n * i // nb for i in range(nb + 1)], dtype=torch.int32)
    kp = torch.arange(n * 7, dtype=torch.int32).reshape(n, 7) + 10000 * part + 1000 * rank + 100 * step
    return offs, kp


def _parts_worker(rank, world, port, q):
    """bench.py's streams layout at N > 1: several sub-batches per rank, each
    with its own GatherPipeline, stepped in the same order on every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap, sizes = 64, [2, 3]
        got = {}
        runners = []
        for part, nb in enumerate(sizes):
            pipe = sdist.GatherPipeline([nb] * world, cap, dst=0)
            bufs = [(torch.zeros((cap, 7), dtype=torch.int32), torch.zeros((cap, 128)),
                     torch.zeros(nb + 1, dtype=torch.int32)) for _ in range(2)]

            def on_result(step, out, part=part):
                ks, offs, _ = out
                got[(part, step)] = ([k.clone() for k in ks], [o.clone() for o in offs])
            runners.append(sdist.PipelinedSteps(pipe, bufs, with_desc=False, on_result=on_result))
        for step in range(4):
            for part, nb in enumerate(sizes):
                def compute(k, d, o, part=part, nb=nb, step=step):
                    offs, kp = _parts_fake(part, rank, step, nb)
                    o[:] = offs
                    k[:len(kp)] = kp
                runners[part].step(compute)
        for r in runners:
            r.flush()
        if rank == 0:
            ok = sorted(got) == [(p, s) for p in range(len(sizes)) for s in range(4)]
            for (part, step), (ks, os_) in got.items():
                for r in range(world):
                    offs, kp = _parts_fake(part, r, step, sizes[part])
                    ok = ok and torch.equal(ks[r], kp) and torch.equal(os_[r], offs)
            q.put(ok)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(target, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    return procs, q


def test_pipelined_steps_world2_uneven():
    """The bench's N > 1 step loop (compute of step i beside the gather of
    step i-1, double-buffered) with uneven shards: every step's keypoints,
    offsets and descriptors arrive on rank 0 intact."""
    procs, q = _spawn(_pipeline_worker)
    try:
        ok = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert [p.exitcode for p in procs] == [0, 0]
    assert ok


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
        uneven = q.get(timeout=120)
        uneven_default = q.get(timeout=120)
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
    assert uneven == ([4, 5], [[0, 1, 4], [0, 1, 2, 5]])
    assert uneven_default == uneven


@pytest.mark.parametrize("world", [2, 8])
def test_pipelined_parts(world):
    """Two sub-batches per rank, each gathered one step behind by its own
    pipeline (bench.py --streams at N > 1): every part's every step arrives
    -- at world 2 and at the 8 ranks of configs[3] (a gloo rehearsal of the
    node the driver's scaling bench runs on)."""
    procs, q = _spawn(_parts_worker, world)
    try:
        ok = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert [p.exitcode for p in procs] == [0] * world
    assert ok
