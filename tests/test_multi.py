"""Multi-GPU batch mode behind the C ABI (sift_multi_*, csrc/multi.hip;
SURVEY.md 8(e), BASELINE configs[3]).

CPU: the shard and offset arithmetic (no GPU needed) against the Python
bench's split (sift_dist.shard).  GPU: one process driving the visible
devices through sift_multi_create / _step / _flush -- at n = 1 on the test
box, where the gather is RCCL's self send/recv on device 0 -- with the
gathered records, descriptors and offsets equal byte for byte to
sift_detect_compute_batch on the same images, and the configs[3] shard shape
(1080p) checked against the CPU path's digests."""
import ctypes
import json
import subprocess

import numpy as np
import pytest

from conftest import kp_bytes, load_golden, sha
from test_abi import build_multi_gpu_host


def test_shard_arithmetic_matches_the_python_split(siftgpu):
    import sift_dist
    for batch in (0, 1, 3, 7, 64, 100, 512, 513):
        for n in (1, 2, 3, 4, 7, 8):
            got = [siftgpu.multi_shard(batch, n, i) for i in range(n)]
            assert [(f, f + c) for f, c in got] == [sift_dist.shard(batch, n, i) for i in range(n)]
            assert sum(c for _, c in got) == batch and got[0][0] == 0
            assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(n - 1))
    # configs[3]: 512 images over 8 devices, 64 each
    assert [siftgpu.multi_shard(512, 8, i) for i in range(8)] == [(64 * i, 64) for i in range(8)]
    f, c = ctypes.c_int(), ctypes.c_int()
    L = siftgpu.lib()
    assert L.sift_multi_shard(10, 0, 0, ctypes.byref(f), ctypes.byref(c)) == siftgpu.SIFT_E_INVALID
    assert L.sift_multi_shard(10, 2, 2, ctypes.byref(f), ctypes.byref(c)) == siftgpu.SIFT_E_INVALID


def test_merge_offsets(siftgpu):
    shards = [np.array([0, 5, 9, 9], np.int32), np.array([0], np.int32), np.array([0, 0, 4], np.int32)]
    out = siftgpu.multi_merge_offsets(shards)
    assert out.tolist() == [0, 5, 9, 9, 9, 13]
    rng = np.random.default_rng(3)
    shards = [np.concatenate([[0], np.cumsum(rng.integers(0, 20000, size=k))]).astype(np.int32) for k in (64,) * 8]
    out = siftgpu.multi_merge_offsets(shards)
    ref = [0]
    for s in shards:
        ref = ref[:-1] + [ref[-1] + int(x) for x in s]
    assert out.tolist() == ref


def test_create_rejects_bad_device_lists(siftgpu):
    """Argument checks before any device work (no GPU here: every list fails,
    duplicates and empty lists with SIFT_E_INVALID on a GPU box too)."""
    L = siftgpu.lib()
    h = ctypes.c_void_p()
    for devs in ([], [0, 0]):
        dv = (ctypes.c_int * max(1, len(devs)))(*devs)
        rc = L.sift_multi_create(dv, len(devs), 64, 64, 1, 0, 0, 100, 0, ctypes.byref(h))
        assert rc != siftgpu.SIFT_OK and not h.value


# ---- GPU ----------------------------------------------------------------------
def _reference(siftgpu, torch, imgs, B, R, C, cap):
    with siftgpu.Context(R, C, B, device=0) as ref:
        k = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        d = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        o = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
        ref.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, k.data_ptr(), d.data_ptr(), cap, o.data_ptr())
        ref.sync()
        n = int(o[B].item())
        return (k[:n].cpu().numpy().view(np.uint8).reshape(n, 28), d[:n].cpu().numpy(), o.cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("streams", [1, 2, 3])
def test_multi_n1_equals_batch_call(siftgpu, streams):
    """Three steps over two alternating image sets through the multi context
    on device 0, the shard split over 1-3 contexts/streams: after every step
    the previous step is gathered (RCCL self p2p forced, one transfer per context),
    after flush the last one; each equals one sift_detect_compute_batch call
    on the same images, records, descriptors and offsets byte for byte."""
    import torch
    R, C, B, cap = 240, 320, 4, 20000
    sets = [torch.empty((B, R, C), dtype=torch.float32, device="cuda") for _ in range(2)]
    assert siftgpu.rccl_version() >= 20000
    # SIFT_MULTI_SELF_P2P: device 0's own records over RCCL (self send/recv) instead of a DMA copy,
    # so the p2p path runs on a one-GPU box
    with siftgpu.MultiContext([0], R, C, B, cap, gather_desc=True, streams_per_device=streams,
                              flags=siftgpu.SIFT_MULTI_SELF_P2P) as m:
        for j, t in enumerate(sets):
            m.synth_images(0, t.data_ptr(), B, R, C, C, R * C, seed_base=10 * j)
        torch.cuda.synchronize()
        refs = [_reference(siftgpu, torch, t, B, R, C, cap) for t in sets]
        order = [0, 1, 0]
        for step, j in enumerate(order):
            m.step([sets[j].data_ptr()], [B], R, C, C, R * C)
            if step == 0:
                continue
            kps, desc = m.copy_gathered()
            _, _, offs, st = m.gathered(B + 1)
            assert st == step - 1
            rk, rd, ro = refs[order[step - 1]]
            assert offs.tolist() == ro.tolist()
            assert kp_bytes(kps).tobytes() == rk.tobytes() and desc.tobytes() == rd.tobytes()
        m.flush()
        kps, desc = m.copy_gathered()
        _, _, offs, st = m.gathered(B + 1)
        rk, rd, ro = refs[order[-1]]
        assert st == len(order) - 1 and offs.tolist() == ro.tolist()
        assert kp_bytes(kps).tobytes() == rk.tobytes() and desc.tobytes() == rd.tobytes()
        s = m.stats()
        assert s["steps"] == 3 and s["transfers"] == 6 * streams and s["records"] == sum(
            int(refs[j][2][B]) for j in order)


@pytest.mark.gpu
def test_multi_configs3_shard_shape_1080p(siftgpu):
    """A configs[3] shard shape on one device (1080p, 5 octaves, records only,
    graph replay across steps): image 0 of the gathered step equals the CPU
    path's digests (tests/golden/synth0_1080x1920.npz)."""
    import torch
    R, C, B = 1080, 1920, 2
    g = load_golden("synth0_1080x1920")
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    with siftgpu.MultiContext([0], R, C, B, B * 40000, gather_desc=True) as m:
        m.synth_images(0, imgs.data_ptr(), B, R, C, C, R * C, seed_base=0)
        torch.cuda.synchronize()   # the images are ready before the step's contexts read them
        for _ in range(2):
            m.step([imgs.data_ptr()], [B], R, C, C, R * C)
        m.flush()
        kps, desc = m.copy_gathered()
        _, _, offs, _ = m.gathered(B + 1)
    a, e = int(offs[0]), int(offs[1])
    assert e - a == int(g["n"])
    assert sha(kps[a:e]) == str(g["kp_sha"]) and sha(desc[a:e]) == str(g["desc_sha"])


@pytest.mark.gpu
def test_cpp_multi_gpu_host_runs(siftgpu, tmp_path):
    """The C++ configs[3] host (tests/cpp/multi_gpu.cpp) on the visible
    devices, a short run: one JSON line with every image gathered."""
    exe = build_multi_gpu_host(tmp_path / "multi_gpu")
    r = subprocess.run([str(exe), "--devices", "1", "--per-device", "4", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["devices"] == 1 and d["images_per_step"] == 4 and d["p2p_transfers"] == 0   # device 0: DMA copies
    assert d["image0_keypoints"] == int(load_golden("synth0_1080x1920")["n"])
    assert d["gathered_keypoints_last_step"] > 4 * 10000 and d["rccl_version"] >= 20000


@pytest.mark.gpu
def test_multi_capacity_overflow_is_reported_and_final(siftgpu):
    """A context's share of kp_cap_per_device too small for its sub-batch:
    the gather reports SIFT_E_CAPACITY naming the device, and the multi
    context refuses every later step (its slots are undefined) until it is
    destroyed; a new one works."""
    import torch
    R, C, B = 240, 320, 2
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    with siftgpu.MultiContext([0], R, C, B, 20, streams_per_device=2) as m:
        m.synth_images(0, imgs.data_ptr(), B, R, C, C, R * C, seed_base=3)
        torch.cuda.synchronize()
        m.step([imgs.data_ptr()], [B], R, C, C, R * C)
        with pytest.raises(siftgpu.SiftError) as ex:
            m.flush()
        assert ex.value.code == siftgpu.SIFT_E_CAPACITY and "kp_cap_per_device" in str(ex.value)
        with pytest.raises(siftgpu.SiftError) as ex:
            m.step([imgs.data_ptr()], [B], R, C, C, R * C)
        assert ex.value.code == siftgpu.SIFT_E_INVALID and "destroy" in str(ex.value)
    with siftgpu.MultiContext([0], R, C, B, 20000) as m:
        m.step([imgs.data_ptr()], [B], R, C, C, R * C)
        m.flush()
        _, _, offs, _ = m.gathered(B + 1)
    assert offs[-1] > 20
