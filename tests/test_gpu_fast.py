"""GPU tests of SIFT_FLAG_FAST: the separable row/column Gaussian pyramid
(sift-gpu_amd/csrc/pyramid_pc.hip) in front of the exact downstream kernels.

Fast mode is NOT bit-exact with the reference's 2-D float chain
(src/sift.cpp:137-146): it applies K[a][b] = 8192 g(a) g(b) as a row pass and
a column pass with fused multiply-adds, so the pyramid differs from the CPU
path by float rounding only.  These tests
  * pin the kernel to its own specification: every plane equals
    oracle.fast_pyramid (oracle/sift_oracle.c so_fast_pyramid, the separable
    form in its exact operation order) bit for bit;
  * bound the difference to the reference's arithmetic: every Gaussian plane
    within an absolute tolerance of the exact CPU path (values are 0..255);
  * match the full SIFT_NCL output keypoint by keypoint against the
    north_star tolerance -- (x, y, size, angle) within 1e-3 and descriptor L2
    within 1e-4 -- with the match rates asserted (a rounding difference can
    flip a discrete decision: a DoG threshold, a cvRound step, an orientation
    peak or a uchar quantisation step, so some keypoints legitimately differ).
"""
import numpy as np
import pytest

from conftest import book_image

pytestmark = pytest.mark.gpu

FAST = 0x1
PLANE_ATOL = 2e-3      # |fast - exact| on 0..255 planes
KP_TOL = 1e-3          # north_star: keypoint (x, y, sigma, theta) within 1e-3
DESC_TOL = 1e-4        # north_star: descriptor L2 within 1e-4
SHAPES = [((1080, 1920), 0), ((203, 157), 2), ((33, 1200), 12), ((300, 210), 3), ((130, 90), 6),
          ((540, 960), 5), ((257, 4100), 7)]


@pytest.fixture(scope="module")
def fctx(siftgpu):
    c = siftgpu.Context(1080, 1920, 4, device=0, flags=FAST)
    yield c
    c.close()


@pytest.mark.parametrize("shape,b", SHAPES + [((4320, 7680), 1)])
def test_fast_pyramid_equals_its_oracle(siftgpu, oracle, shape, b):
    """Every plane of pyr_pc_kernel == so_fast_pyramid, bit for bit (the
    producer wave's base blur, the consumers' register transposes, chunk
    seams, strip edges, odd shapes, a 4100-column strip count, the 8K image)."""
    img = oracle.synth_image(b, *shape)
    ctx = siftgpu.Context(*shape, 1, device=0, flags=FAST)
    try:
        gp = ctx.buildGaussianPyramid(img, 5)
    finally:
        ctx.close()
    ref = oracle.split_planes(oracle.fast_pyramid(img, 5), *shape, 5, 5)
    assert len(gp) == len(ref)
    for i, (a, c) in enumerate(zip(gp, ref)):
        if a.tobytes() != c.tobytes():
            bad = np.argwhere(a != c)
            pytest.fail(f"plane {i} (octave {i // 5}, scale {i % 5}) {a.shape}: {len(bad)} values differ, "
                        f"first at {bad[0].tolist()}: {a[tuple(bad[0])]!r} vs {c[tuple(bad[0])]!r}")


@pytest.mark.parametrize("shape,b", SHAPES)
def test_fast_pyramid_close_to_exact(fctx, siftgpu, oracle, shape, b):
    img = oracle.synth_image(b, *shape)
    if shape[0] <= 1080 and shape[1] <= 1920:
        gp = fctx.buildGaussianPyramid(img, 5)
    else:
        ctx = siftgpu.Context(*shape, 1, device=0, flags=FAST)
        try:
            gp = ctx.buildGaussianPyramid(img, 5)
        finally:
            ctx.close()
    ref = oracle.split_planes(oracle.build_gaussian_pyramid(img), *shape, 5, 5)
    errs = [float(np.abs(p.astype(np.float64) - q).max()) for p, q in zip(gp, ref)]
    assert max(errs) < PLANE_ATOL, errs
    # octave-0 base: a 9-tap row pass then column pass of integer pixels
    assert errs[0] < 5e-4, errs[0]


def test_fast_pyramid_border_rule(fctx):
    """The last source row and column never contribute (getSubMatrix, src/sift.cpp:116)."""
    img = np.zeros((64, 80), np.float32)
    img[-1, :] = 255
    img[:, -1] = 255
    gp = fctx.buildGaussianPyramid(img, 3)
    for i, p in enumerate(gp):
        assert not p.any(), f"plane {i}"


def test_fast_rejects_planes_past_the_offset_range(siftgpu):
    """the separable kernel drops out-of-range loads and stores by
    a 0x7f000000-byte offset, so an input whose rows span that range must be
    refused (SIFT_E_SIZE) before any kernel runs, never silently mis-padded."""
    import torch
    ctx = siftgpu.Context(1080, 1920, 2, device=0, flags=FAST)
    try:
        imgs = torch.zeros((16,), dtype=torch.float32, device="cuda")
        kp = torch.empty((16, 7), dtype=torch.int32, device="cuda")
        de = torch.empty((16, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((3,), dtype=torch.int32, device="cuda")
        stride = (0x7f000000 // 4) // 1080 + 64  # 1080 rows of this stride pass the range
        with pytest.raises(siftgpu.SiftError) as e:
            ctx.detect_compute_batch(imgs.data_ptr(), 2, 1080, 1920, stride, 1080 * stride, kp.data_ptr(),
                                     de.data_ptr(), 16, offs.data_ptr())
        assert e.value.code == siftgpu.SIFT_E_SIZE, e.value
    finally:
        ctx.close()


def _match(ka, da, kb, db):
    """For each keypoint of a, a keypoint of b with the same octave word and
    (x, y, size, angle) within KP_TOL (angle modulo 360).  Returns the fraction
    of a matched and, of those, the fraction whose descriptors are within
    DESC_TOL in L2."""
    if len(ka) == 0:
        return 1.0, 1.0
    buckets = {}
    for j, (x, y) in enumerate(zip(kb["x"], kb["y"])):
        buckets.setdefault((int(x), int(y)), []).append(j)
    matched = dok = 0
    for i in range(len(ka)):
        x, y = float(ka["x"][i]), float(ka["y"][i])
        best = None
        for gx in (int(x) - 1, int(x), int(x) + 1):
            for gy in (int(y) - 1, int(y), int(y) + 1):
                for j in buckets.get((gx, gy), ()):
                    if kb["octave"][j] != ka["octave"][i]:
                        continue
                    da_ = abs(float(kb["angle"][j]) - float(ka["angle"][i]))
                    da_ = min(da_, 360 - da_)
                    if (abs(float(kb["x"][j]) - x) <= KP_TOL and abs(float(kb["y"][j]) - y) <= KP_TOL
                            and abs(float(kb["size"][j]) - float(ka["size"][i])) <= KP_TOL and da_ <= KP_TOL):
                        d = float(np.linalg.norm(da[i].astype(np.float64) - db[j]))
                        if best is None or d < best:
                            best = d
        if best is not None:
            matched += 1
            dok += best <= DESC_TOL
    return matched / len(ka), dok / max(matched, 1)


@pytest.mark.parametrize("name", ["synth480x640", "book"])
def test_fast_sift_matches_cpu_path(fctx, oracle, name):
    img = book_image() if name == "book" else oracle.synth_image(9, 480, 640)
    kr, dr = oracle.sift(img)
    kf, df = fctx.SIFT_NCL(img)
    assert abs(len(kf) - len(kr)) <= 0.03 * len(kr) + 2, (len(kf), len(kr))
    rate, drate = _match(kr, dr, kf, df)
    back, _ = _match(kf, df, kr, dr)
    print(f"{name}: {len(kr)} cpu / {len(kf)} fast keypoints; matched {rate:.4f} (reverse {back:.4f}); "
          f"descriptor L2 <= 1e-4 for {drate:.4f} of matches")
    assert rate >= 0.95 and back >= 0.95
    assert drate >= 0.9
    np.testing.assert_allclose(np.linalg.norm(df, axis=1), 1.0, atol=2e-6)


def test_fast_1080p_match_rate(fctx, oracle):
    img = oracle.synth_image(0, 1080, 1920)
    kr, dr = oracle.sift(img)
    kf, df = fctx.SIFT_NCL(img)
    rate, drate = _match(kr, dr, kf, df)
    print(f"1080p: {len(kr)} cpu / {len(kf)} fast; matched {rate:.4f}; descriptor ok {drate:.4f}")
    assert rate >= 0.95 and drate >= 0.9


@pytest.mark.parametrize("B,R,C", [(3, 240, 320)])
def test_fast_batch_equals_single(fctx, oracle, B, R, C):
    """Batch mode and the single-image path run the same kernels: bit-identical."""
    import torch
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    fctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, seed_base=30)
    fctx.sync()
    host = imgs.cpu().numpy()
    cap = 20000
    kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
    offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
    fctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kpts.data_ptr(), desc.data_ptr(), cap,
                              offs.data_ptr())
    fctx.sync()
    o = offs.cpu().numpy()
    k = kpts.cpu().numpy().view(np.uint8).reshape(cap, 28)
    dd = desc.cpu().numpy()
    for b in range(B):
        ks, ds = fctx.SIFT_NCL(host[b])
        assert o[b + 1] - o[b] == len(ks)
        assert k[o[b]:o[b + 1]].tobytes() == np.ascontiguousarray(ks).view(np.uint8).tobytes()
        assert dd[o[b]:o[b + 1]].tobytes() == ds.tobytes()


@pytest.mark.parametrize("flags", [0, FAST])
@pytest.mark.parametrize("shape,b", [((203, 157), 2), ((540, 960), 5), ((257, 4100), 7)])
def test_pitch_padding_is_never_read(siftgpu, oracle, monkeypatch, flags, shape, b):
    """the fast pyramid's wide stores leave unspecified values in
    the pitch padding (common.hpp, kPitchAlign).  With the test hook
    SIFT_HIP_TEST_HOOKS=poison_pad the library writes a NaN into every padding
    column of every plane after the pyramid; the detect + describe output must
    not change, in fast and exact mode (shapes with padding at every octave)."""
    img = oracle.synth_image(b, *shape)
    out = []
    for poison in ("", "poison_pad"):
        monkeypatch.setenv("SIFT_HIP_TEST_HOOKS", poison)   # read at context creation
        ctx = siftgpu.Context(*shape, 1, device=0, flags=flags)
        try:
            out.append(ctx.SIFT_NCL(img))
        finally:
            ctx.close()
    (k0, d0), (k1, d1) = out
    assert len(k0) > 10
    assert np.ascontiguousarray(k0).tobytes() == np.ascontiguousarray(k1).tobytes()
    assert d0.tobytes() == d1.tobytes()


def test_fast_headline_batch_equals_single(siftgpu):
    """configs[2] in fast mode: one 64 x 1080p batch call (other chunk seams
    than a single image's launch) gives images 0, 31 and 63 bit-identical to
    the single-image fast path, which test_fast_pyramid_equals_its_oracle pins."""
    import torch
    B, R, C = 64, 1080, 1920
    ctx = siftgpu.Context(R, C, B, device=0, flags=FAST)
    one = siftgpu.Context(R, C, 1, device=0, flags=FAST)
    try:
        imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
        ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, seed_base=0)
        cap = B * 40000
        kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
        ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kpts.data_ptr(), desc.data_ptr(), cap,
                                 offs.data_ptr())
        ctx.sync()
        o = offs.cpu().numpy()
        for b in (0, 31, 63):
            ks, ds = one.SIFT_NCL(imgs[b].cpu().numpy())
            assert o[b + 1] - o[b] == len(ks) > 5000
            kb = kpts[o[b]:o[b + 1]].cpu().numpy().view(np.uint8).reshape(-1, 28)
            assert kb.tobytes() == np.ascontiguousarray(ks).view(np.uint8).tobytes(), b
            assert desc[o[b]:o[b + 1]].cpu().numpy().tobytes() == ds.tobytes(), b
    finally:
        ctx.close()
        one.close()


def test_expired_pipeline_wait_is_reported_once(siftgpu, oracle, monkeypatch):
    """pyr_pc_kernel's bounded LDS-counter waits.  The test hook
    pc_stall_once gives the context's next launch a wait bound of zero, so its
    waves give up at their first unpublished counter (garbage planes, no
    hang); buildGaussianPyramid must report SIFT_E_HIP for that call, consume
    the sticky bit, and the next call must be clean and equal the oracle."""
    shape, b = (300, 210), 3
    img = oracle.synth_image(b, *shape)
    monkeypatch.setenv("SIFT_HIP_TEST_HOOKS", "pc_stall_once")   # read at context creation
    ctx = siftgpu.Context(*shape, 1, device=0, flags=FAST)
    try:
        with pytest.raises(siftgpu.SiftError) as ex:
            ctx.buildGaussianPyramid(img, 5)
        assert ex.value.code == siftgpu.SIFT_E_HIP and "wait expired" in str(ex.value)
        gp = ctx.buildGaussianPyramid(img, 5)           # the bit was consumed: clean
        ctx.sync()                                      # and nothing left for the sticky report
        kps, _ = ctx.SIFT_NCL(img)
    finally:
        ctx.close()
    ref = oracle.split_planes(oracle.fast_pyramid(img, 5), *shape, 5, 5)
    for i, (a, c) in enumerate(zip(gp, ref)):
        assert a.tobytes() == c.tobytes(), f"plane {i} after the stalled call"
    assert len(kps) > 0
