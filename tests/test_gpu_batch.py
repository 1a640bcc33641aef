"""GPU tests of the device batch path at the bench's own sizes, the graphed
single-image path, and the capacity / error contract, all through the C ABI.

* configs[2] (the credited bench workload): 64 x 1920x1080 synthetic images in
  one sift_detect_compute_batch call; images 0, 31 and 63 against the CPU
  path's SHA-256 digests (tests/golden/make_golden.py --batch), every image
  against size-independent properties, graph replay == first launch ==
  direct launches.
* configs[1]: one 1080p image, 4 octaves, host entry point (hipGraph replay).
* batch > 128 images (the per-image offset gather strides over the batch).
* overflow: candidate workspace -> SIFT_E_WORKSPACE (never the sizing case),
  batch keypoint capacity -> SIFT_E_CAPACITY with the true total reported.
"""
import numpy as np
import pytest

from conftest import assert_bits_equal, kp_bytes, load_golden, sha

pytestmark = pytest.mark.gpu

R, C = 1080, 1920


def _run_batch(ctx, imgs, B, cap, torch):
    kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
    offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
    ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kpts.data_ptr(), desc.data_ptr(), cap,
                             offs.data_ptr())
    ctx.sync()
    return kpts, desc, offs


def test_headline_batch_64x1080p(siftgpu):
    """configs[2]: the exact workload bench.py times, checked."""
    import torch
    B = 64
    g0 = load_golden("synth0_1080x1920")
    gb = load_golden("batch_1080x1920")
    with siftgpu.Context(R, C, B, device=0) as ctx:
        imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, seed_base=0)
        cap = B * 40000
        kpts, desc, offs = _run_batch(ctx, imgs, B, cap, torch)
        o = offs.cpu().numpy().astype(np.int64)
        assert o[0] == 0 and np.all(np.diff(o) > 0) and o[-1] <= cap
        k = kpts[:o[-1]].cpu().numpy().view(np.uint8).reshape(-1, 28)
        d = desc[:o[-1]].cpu().numpy()
        # image 0 = the 1080p golden; images 31 and 63 = the batch digests
        assert o[1] - o[0] == int(g0["n"]) == 12932
        assert sha(k[o[0]:o[1]]) == str(g0["kp_sha"])
        assert sha(d[o[0]:o[1]]) == str(g0["desc_sha"])
        for s, n, ks, ds in zip(gb["seeds"], gb["n"], gb["kp_sha"], gb["desc_sha"]):
            s = int(s)
            assert o[s + 1] - o[s] == int(n), f"seed {s}"
            assert sha(k[o[s]:o[s + 1]]) == str(ks), f"seed {s} keypoints"
            assert sha(d[o[s]:o[s + 1]]) == str(ds), f"seed {s} descriptors"
        # every image: unit-L2 RootSIFT rows, non-decreasing octaves, in-image coordinates
        np.testing.assert_allclose(np.linalg.norm(d.astype(np.float64), axis=1), 1.0, atol=2e-6)
        kv = k.view(np.float32).reshape(-1, 7)
        ki = k.view(np.int32).reshape(-1, 7)
        for b in range(B):
            oc = ki[o[b]:o[b + 1], 5] & 255
            assert np.all(np.diff(oc) >= 0), f"image {b} octave order"
        assert np.all((kv[:, 0] >= 0) & (kv[:, 0] < C) & (kv[:, 1] >= 0) & (kv[:, 1] < R))
        # replay of the captured graph, and direct launches, give the same bytes
        kpts2, desc2, offs2 = _run_batch(ctx, imgs, B, cap, torch)
        assert torch.equal(offs, offs2) and torch.equal(kpts[:o[-1]], kpts2[:o[-1]])
        assert torch.equal(desc[:o[-1]], desc2[:o[-1]])
        ctx.set_flags(siftgpu.SIFT_FLAG_NO_GRAPH)
        kpts3, desc3, offs3 = _run_batch(ctx, imgs, B, cap, torch)
        assert torch.equal(offs, offs3) and torch.equal(kpts[:o[-1]], kpts3[:o[-1]])
        assert torch.equal(desc[:o[-1]], desc3[:o[-1]])
        del imgs, kpts, desc, kpts2, desc2, kpts3, desc3
    torch.cuda.empty_cache()


def test_single_image_1080p_4_octaves(siftgpu, oracle):
    """configs[1]: one 1080p image, 4 octaves x 5 scales, the host entry
    point (graphed device sequence, one wait) -- twice, the second a replay."""
    gb = load_golden("batch_1080x1920")
    img = oracle.synth_image(0, R, C)
    with siftgpu.Context(R, C, 1, device=0) as ctx:
        ctx.set_octaves(4)
        for _ in range(2):
            kps, desc = ctx.SIFT_NCL(img)
            assert len(kps) == int(gb["oct4_n"])
            assert sha(kps) == str(gb["oct4_kp_sha"])
            assert sha(desc) == str(gb["oct4_desc_sha"])


def test_batch_over_128_images(siftgpu, oracle):
    """More than 128 images in one call: every image's offsets and output."""
    import torch
    B, r, c = 160, 48, 64
    with siftgpu.Context(r, c, B, device=0) as ctx:
        imgs = torch.empty((B, r, c), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), B, r, c, c, r * c, seed_base=300)
        cap = B * 200
        kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        offs = torch.full((B + 1,), -7, dtype=torch.int32, device="cuda")
        ctx.detect_compute_batch(imgs.data_ptr(), B, r, c, c, r * c, kpts.data_ptr(), desc.data_ptr(), cap,
                                 offs.data_ptr())
        ctx.sync()
        o = offs.cpu().numpy()
        k = kpts.cpu().numpy().view(np.uint8).reshape(cap, 28)
        d = desc.cpu().numpy()
    assert o[0] == 0 and np.all(np.diff(o) >= 0)
    total = 0
    for b in range(B):
        kr, dr = oracle.sift(oracle.synth_image(300 + b, r, c))
        assert o[b + 1] - o[b] == len(kr), f"image {b}"
        assert_bits_equal(k[o[b]:o[b + 1]], kp_bytes(kr), f"image {b} keypoints")
        assert_bits_equal(d[o[b]:o[b + 1]], dr, f"image {b} descriptors")
        total += len(kr)
    assert total > 0 and o[B] == total


def test_candidate_workspace_overflow_is_an_error(siftgpu, oracle):
    """A candidate overflow raises SIFT_E_WORKSPACE (not the two-call sizing
    case), leaves no stale result behind, and the context recovers."""
    import ctypes
    import torch
    img = oracle.synth_image(1, 240, 320)
    g = load_golden("synth1_240x320")
    with siftgpu.Context(240, 320, 2, device=0) as ctx:
        kps, _ = ctx.SIFT_NCL(img)  # a result is held ...
        assert len(kps) == int(g["n"])
        ctx.set_candidate_capacity(8)
        n = ctypes.c_int(5)
        rc = siftgpu.lib().sift_detect_compute(ctx.h, img.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 240, 320,
                                               320 * 4, None, None, 0, ctypes.byref(n))
        assert rc == siftgpu.SIFT_E_WORKSPACE and n.value == -1
        # ... and none after the overflow: the copy step refuses
        kp = np.zeros(4, siftgpu.KEYPOINT_DTYPE)
        rc = siftgpu.lib().sift_copy_results(ctx.h, kp.ctypes.data, None, 4, ctypes.byref(n))
        assert rc == siftgpu.SIFT_E_INVALID
        with pytest.raises(siftgpu.SiftError) as e:
            ctx.SIFT_NCL(img)
        assert e.value.code == siftgpu.SIFT_E_WORKSPACE
        # batch path: reported by sift_sync
        imgs = torch.empty((2, 240, 320), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), 2, 240, 320, 320, 240 * 320, seed_base=1)
        kpts = torch.empty((4000, 7), dtype=torch.int32, device="cuda")
        desc = torch.empty((4000, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((3,), dtype=torch.int32, device="cuda")
        ctx.detect_compute_batch(imgs.data_ptr(), 2, 240, 320, 320, 240 * 320, kpts.data_ptr(), desc.data_ptr(),
                                 4000, offs.data_ptr())
        with pytest.raises(siftgpu.SiftError) as e:
            ctx.sync()
        assert e.value.code == siftgpu.SIFT_E_WORKSPACE
        ctx.sync()  # reported once, then clear
        # calDescriptor never looks at candidates (stale overflow)
        ctx.detect_compute_batch(imgs.data_ptr(), 2, 240, 320, 320, 240 * 320, kpts.data_ptr(), desc.data_ptr(),
                                 4000, offs.data_ptr())
        gp = oracle.build_gaussian_pyramid(img)
        gpl = oracle.split_planes(gp, 240, 320, 5, 5)
        kr = oracle.sift(img)[0]
        assert_bits_equal(ctx.calDescriptor(gpl, kr, 0), oracle.calc_descriptors(gp, 240, 320, kr), "descriptors")
        with pytest.raises(siftgpu.SiftError):
            ctx.sync()  # the batch overflow above is still reported to the batch caller
        ctx.set_candidate_capacity(16384)
        kps, desc1 = ctx.SIFT_NCL(img)
        assert_bits_equal(kp_bytes(kps), g["kps"], "keypoints after recovery")
        assert_bits_equal(desc1, g["desc"], "descriptors after recovery")


def test_batch_keypoint_capacity(siftgpu, oracle):
    """A batch call whose kp_cap is too small: sift_sync reports
    SIFT_E_CAPACITY, d_img_offsets[batch] holds the true total, and the
    first kp_cap keypoints are the right ones."""
    import torch
    B, r, c = 3, 240, 320
    with siftgpu.Context(r, c, B, device=0) as ctx:
        imgs = torch.empty((B, r, c), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), B, r, c, c, r * c, seed_base=40)
        cap = 50
        kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
        ctx.detect_compute_batch(imgs.data_ptr(), B, r, c, c, r * c, kpts.data_ptr(), desc.data_ptr(), cap,
                                 offs.data_ptr())
        with pytest.raises(siftgpu.SiftError) as e:
            ctx.sync()
        assert e.value.code == siftgpu.SIFT_E_CAPACITY
        o = offs.cpu().numpy()
        ref = [oracle.sift(oracle.synth_image(40 + b, r, c)) for b in range(B)]
        assert o[B] == sum(len(k) for k, _ in ref)
        k0, d0 = ref[0]
        assert len(k0) > cap
        assert_bits_equal(kpts.cpu().numpy().view(np.uint8).reshape(cap, 28), kp_bytes(k0[:cap]), "first kp_cap")
        assert_bits_equal(desc.cpu().numpy(), d0[:cap], "first kp_cap descriptors")
        ctx.sync()  # reported once


def test_batch_kp_cap_larger_than_the_buffers_need(siftgpu, oracle):
    """kp_cap is the caller's promise, not an allocation hint: a 2^30 capacity
    over buffers sized for the real keypoints works (the descriptor's ranking
    scratch is bounded by the candidate capacity, not by kp_cap)."""
    import torch
    B, r, c = 2, 240, 320
    with siftgpu.Context(r, c, B, device=0) as ctx:
        imgs = torch.empty((B, r, c), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), B, r, c, c, r * c, seed_base=60)
        ref = [oracle.sift(oracle.synth_image(60 + b, r, c)) for b in range(B)]
        n = sum(len(k) for k, _ in ref)
        kpts = torch.empty((n, 7), dtype=torch.int32, device="cuda")
        desc = torch.empty((n, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
        ctx.detect_compute_batch(imgs.data_ptr(), B, r, c, c, r * c, kpts.data_ptr(), desc.data_ptr(), 1 << 30,
                                 offs.data_ptr())
        ctx.sync()
        o = offs.cpu().numpy()
        assert o[B] == n
        kb = np.concatenate([kp_bytes(k) for k, _ in ref])
        assert_bits_equal(kpts.cpu().numpy().view(np.uint8).reshape(n, 28), kb, "keypoints")
        assert_bits_equal(desc.cpu().numpy(), np.concatenate([d for _, d in ref]), "descriptors")


def test_graph_cache_rotating_buffers(siftgpu, oracle):
    """a caller rotating among more output buffers than the graph
    cache holds (6 slots, 4 entries) with one shape.  Each new buffer set
    patches the cached executable in place (hipGraphExecUpdate) instead of
    instantiating; every call's output is the CPU path's, in its own slot,
    and replays of earlier slots still land in those slots."""
    import torch
    B, r, c = 3, 96, 128
    ref = [oracle.sift(oracle.synth_image(70 + b, r, c)) for b in range(B)]
    n = [len(k) for k, _ in ref]
    with siftgpu.Context(r, c, B, device=0) as ctx:
        imgs = torch.empty((B, r, c), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), B, r, c, c, r * c, seed_base=70)
        cap = 4 * sum(n)
        slots = [(torch.full((cap, 7), -1, dtype=torch.int32, device="cuda"),
                  torch.full((cap, 128), -1.0, dtype=torch.float32, device="cuda"),
                  torch.full((B + 1,), -1, dtype=torch.int32, device="cuda")) for _ in range(6)]
        order = [0, 1, 2, 3, 4, 5, 0, 3, 5, 1]
        for i in order:
            k, d, o = slots[i]
            k.fill_(-1)
            d.fill_(-1.0)
            o.fill_(-1)
            ctx.detect_compute_batch(imgs.data_ptr(), B, r, c, c, r * c, k.data_ptr(), d.data_ptr(), cap,
                                     o.data_ptr())
            ctx.sync()
            oo = o.cpu().numpy()
            kk = k.cpu().numpy().view(np.uint8).reshape(cap, 28)
            dd = d.cpu().numpy()
            for b in range(B):
                assert oo[b + 1] - oo[b] == n[b], f"slot {i} image {b}"
                assert_bits_equal(kk[oo[b]:oo[b + 1]], kp_bytes(ref[b][0]), f"slot {i} image {b} keypoints")
                assert_bits_equal(dd[oo[b]:oo[b + 1]], ref[b][1], f"slot {i} image {b} descriptors")
            assert np.all(kk[oo[B]:].view(np.int32) == -1), f"slot {i}: writes past the total"
        caps, upd, inst = ctx.graph_stats()
    assert inst == 1, (caps, upd, inst)          # one shape: one executable
    assert upd == caps - 1 == len(order) - 1, (caps, upd, inst)  # every other call patched it
