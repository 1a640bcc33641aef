"""GPU tests of SIFT_FLAG_FAST: the separable row/column Gaussian pyramid
(sift-gpu_amd/csrc/pyramid_tri.hip; pyramid_pair.hip and pyramid_fast.hip
behind switches) in front of the exact downstream kernels.

Fast mode is NOT bit-exact with the reference's 2-D float chain
(src/sift.cpp:137-146): it applies K[a][b] = 8192 g(a) g(b) as a row pass and
a column pass with fused multiply-adds, so the pyramid differs from the CPU
path by float rounding only.  These tests bound that difference against the
CPU oracle:
  * every Gaussian plane within an absolute tolerance (values are 0..255);
  * the full SIFT_NCL output matched keypoint by keypoint against the
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


@pytest.fixture(scope="module")
def fctx(siftgpu):
    c = siftgpu.Context(1080, 1920, 4, device=0, flags=FAST)
    yield c
    c.close()


def _fast_ctx(siftgpu, kind, rows=1080, cols=1920, batch=4):
    """A SIFT_FLAG_FAST context on one of the three separable pyramids:
    pyramid_tri.hip (default, round 3), pyramid_pair.hip (SIFT_HIP_FAST_PAIR=1)
    and round 2's pyramid_fast.hip (SIFT_HIP_FAST_V1=1); the switches are read
    at context creation."""
    import os
    env = {"tri": {}, "pair": {"SIFT_HIP_FAST_PAIR": "1"}, "v1": {"SIFT_HIP_FAST_V1": "1"}}[kind]
    keys = ("SIFT_HIP_FAST_PAIR", "SIFT_HIP_FAST_V1")
    old = {k: os.environ.pop(k, None) for k in keys}
    os.environ.update(env)
    try:
        return siftgpu.Context(rows, cols, batch, device=0, flags=FAST)
    finally:
        for k in keys:
            os.environ.pop(k, None)
            if old[k] is not None:
                os.environ[k] = old[k]


@pytest.fixture(scope="module", params=["tri", "pair", "v1"])
def fctx_both(request, siftgpu):
    c = _fast_ctx(siftgpu, request.param)
    yield c
    c.close()


@pytest.mark.parametrize("shape,b", [((1080, 1920), 0), ((203, 157), 2), ((33, 1200), 12), ((540, 960), 5)])
def test_fast_tri_equals_pair(siftgpu, oracle, shape, b):
    """pyramid_tri.hip and pyramid_pair.hip apply the same row-pass chains and the
    same in-order column scatter, so their planes are bit-identical."""
    img = oracle.synth_image(b, *shape)
    t = _fast_ctx(siftgpu, "tri", *shape, 1)
    p = _fast_ctx(siftgpu, "pair", *shape, 1)
    try:
        gt = t.buildGaussianPyramid(img, 5)
        gp = p.buildGaussianPyramid(img, 5)
    finally:
        t.close()
        p.close()
    assert len(gt) == len(gp)
    for i, (a, c) in enumerate(zip(gt, gp)):
        assert a.tobytes() == c.tobytes(), f"plane {i} differs"


@pytest.mark.parametrize("shape,b", [((1080, 1920), 0), ((203, 157), 2), ((33, 1200), 12),
                                     ((300, 210), 3), ((130, 90), 6)])
def test_fast_pyramid_close_to_exact(fctx_both, oracle, shape, b):
    img = oracle.synth_image(b, *shape)
    gp = fctx_both.buildGaussianPyramid(img, 5)
    ref = oracle.split_planes(oracle.build_gaussian_pyramid(img), *shape, 5, 5)
    errs = [float(np.abs(p.astype(np.float64) - q).max()) for p, q in zip(gp, ref)]
    assert max(errs) < PLANE_ATOL, errs
    # octave-0 base: a 9-tap row pass then column pass of integer pixels
    assert errs[0] < 5e-4, errs[0]


def test_fast_pyramid_border_rule(fctx_both):
    """The last source row and column never contribute (getSubMatrix, src/sift.cpp:116)."""
    img = np.zeros((64, 80), np.float32)
    img[-1, :] = 255
    img[:, -1] = 255
    gp = fctx_both.buildGaussianPyramid(img, 3)
    for i, p in enumerate(gp):
        assert not p.any(), f"plane {i}"


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


def test_fast_batch_equals_single(fctx, oracle):
    """Batch mode and the single-image path run the same kernels: bit-identical."""
    import torch
    B, R, C = 3, 240, 320
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
