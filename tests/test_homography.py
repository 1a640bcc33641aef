"""Homography: findHomography(obj, scene, RANSAC) and
perspectiveTransform (src/main.cpp:44-62), host code in libsift_hip.so
(homography.hip) behind sift_find_homography / sift_perspective_transform.

OpenCV is not in this image, so parity with its RANSAC (RNG stream, Jacobi,
LMSolver) is unpinned.  The library is pinned value for value against an
independent numpy restatement of the same algorithm (oracle/homography.py:
cv::RNG stream, subset checks, normalised DLT, float reprojection test,
refit + LM), on noisy data with outliers.  The CPU tests also check what the
application relies on:
the model is recovered from correspondences with outliers (exactly without
noise), the inlier mask is the true one, degenerate input gives OpenCV's empty
result, the run is deterministic, and perspectiveTransform equals its double
formula bit for bit.  No GPU is touched.  The GPU test runs the whole
reference application flow on the book image and a shifted crop of it."""
import numpy as np
import pytest


def _H_true():
    return np.array([[0.9, -0.12, 31.0], [0.08, 1.05, -12.5], [2e-4, -1e-4, 1.0]])


def _project(H, p):
    q = np.c_[p, np.ones(len(p))] @ H.T
    return (q[:, :2] / q[:, 2:]).astype(np.float32)


def _data(rng, n, out_frac, noise=0.0):
    src = rng.uniform(0, 640, (n, 2)).astype(np.float32)
    dst = _project(_H_true(), src.astype(np.float64))
    if noise:
        dst = (dst + rng.normal(0, noise, dst.shape)).astype(np.float32)
    bad = rng.random(n) < out_frac
    dst[bad] = rng.uniform(0, 640, (bad.sum(), 2)).astype(np.float32)
    return src, dst, ~bad


def test_recovers_model_and_inliers(siftgpu):
    rng = np.random.default_rng(0)
    src, dst, good = _data(rng, 300, 0.3)
    H, mask = siftgpu.findHomography(src, dst, siftgpu.RANSAC)
    assert H is not None and H[2, 2] == 1.0
    np.testing.assert_allclose(H, _H_true(), rtol=1e-5, atol=1e-7)
    # outliers thrown anywhere can land within 3 px of the model by chance
    far = np.linalg.norm(_project(_H_true(), src.astype(np.float64)) - dst, axis=1) > 3.0
    assert mask[good].all() and not mask[far].any()


def test_noisy_model_maps_corners(siftgpu):
    rng = np.random.default_rng(1)
    src, dst, good = _data(rng, 400, 0.4, noise=0.5)
    H, mask = siftgpu.findHomography(src, dst)
    corners = np.array([[0, 0], [640, 0], [640, 480], [0, 480]], np.float32)
    err = np.linalg.norm(siftgpu.perspectiveTransform(corners, H) - _project(_H_true(), corners), axis=1)
    assert err.max() < 1.0
    assert mask[good].mean() > 0.95


def test_deterministic(siftgpu):
    rng = np.random.default_rng(2)
    src, dst, _ = _data(rng, 120, 0.5, noise=0.3)
    H1, m1 = siftgpu.findHomography(src, dst)
    H2, m2 = siftgpu.findHomography(src, dst)
    assert H1.tobytes() == H2.tobytes() and m1.tobytes() == m2.tobytes()


def test_degenerate_inputs(siftgpu):
    src = np.array([[0, 0], [1, 0], [2, 0]], np.float32)
    assert siftgpu.findHomography(src, src)[0] is None                     # n < 4
    line = np.c_[np.arange(10), 2 * np.arange(10)].astype(np.float32)      # all collinear
    assert siftgpu.findHomography(line, line)[0] is None
    sq = np.array([[0, 0], [10, 0], [10, 10], [0, 10]], np.float32)        # exactly 4: direct fit
    H, m = siftgpu.findHomography(sq, sq * 2 + 5)
    np.testing.assert_allclose(H, [[2, 0, 5], [0, 2, 5], [0, 0, 1]], atol=1e-9)
    assert m.all()


@pytest.mark.parametrize("seed,n,out_frac,noise", [(10, 60, 0.3, 0.5), (11, 150, 0.5, 1.0), (12, 40, 0.1, 0.0),
                                                    (13, 200, 0.6, 2.0), (14, 5, 0.0, 0.3)])
def test_matches_oracle_bitexact(siftgpu, seed, n, out_frac, noise):
    """sift_find_homography == oracle/homography.py: every H entry (float64
    bits) and the inlier mask."""
    import homography as HO  # oracle/ (the checker)
    rng = np.random.default_rng(seed)
    src, dst, _ = _data(rng, n, out_frac, noise=noise)
    H, mask = siftgpu.findHomography(src, dst, siftgpu.RANSAC)
    Hr, mr = HO.find_homography(src, dst)
    assert H is not None and Hr is not None
    assert H.reshape(9).tobytes() == np.array(Hr, np.float64).tobytes(), (H.reshape(9), Hr)
    assert mask.tobytes() == mr.tobytes()
    corners = np.array([[0, 0], [640, 0], [640, 480], [0, 480]], np.float32)
    assert siftgpu.perspectiveTransform(corners, H).tobytes() == HO.perspective_transform(Hr, corners).tobytes()


def test_oracle_degenerate_like_library(siftgpu):
    import homography as HO
    line = np.c_[np.arange(10), 2 * np.arange(10)].astype(np.float32)
    assert HO.find_homography(line, line)[0] is None and siftgpu.findHomography(line, line)[0] is None
    sq = np.array([[0, 0], [10, 0], [10, 10], [0, 10]], np.float32)
    H, _ = siftgpu.findHomography(sq, sq * 2 + 5)
    assert H.reshape(9).tobytes() == np.array(HO.find_homography(sq, sq * 2 + 5)[0], np.float64).tobytes()


def test_rng_stream():
    """cv::RNG((uint64)-1): the multiply-with-carry recurrence, restated."""
    import homography as HO
    r = HO.RNG()
    first = [r.next() for _ in range(4)]
    st = (1 << 64) - 1
    ref = []
    for _ in range(4):
        st = ((st & 0xffffffff) * 4164903690 + (st >> 32)) & ((1 << 64) - 1)
        ref.append(st & 0xffffffff)
    assert first == ref


def test_perspective_transform_formula(siftgpu):
    rng = np.random.default_rng(4)
    p = rng.uniform(-100, 700, (1000, 2)).astype(np.float32)
    H = _H_true()
    out = siftgpu.perspectiveTransform(p, H)
    x, y = p[:, 0].astype(np.float64), p[:, 1].astype(np.float64)
    w = H[2, 0] * x + H[2, 1] * y + H[2, 2]
    iw = 1.0 / w
    ref = np.c_[((H[0, 0] * x + H[0, 1] * y + H[0, 2]) * iw).astype(np.float32),
                ((H[1, 0] * x + H[1, 1] * y + H[1, 2]) * iw).astype(np.float32)]
    assert out.tobytes() == ref.tobytes()
    Hz = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 0]], np.float64)            # |w| <= FLT_EPSILON -> (0, 0)
    assert (siftgpu.perspectiveTransform(p[:5], Hz) == 0).all()


@pytest.mark.gpu
def test_gpu_reference_app_flow(siftgpu):
    """src/main.cpp:19-62 end to end: readImage (scene resized to 960x960 is
    not needed here), SIFT_NCL x2, knnMatch + ratio, findHomography,
    perspectiveTransform of the object corners.  Object = a crop of the book
    image shifted by (dx, dy): H must be that translation."""
    from conftest import book_image
    img0 = book_image()
    dy, dx = 13, 9
    img1 = np.ascontiguousarray(img0[dy:dy + 250, dx:dx + 180])
    kp0, d0 = siftgpu.SIFT_NCL(img0)
    kp1, d1 = siftgpu.SIFT_NCL(img1)
    good = siftgpu.ratio_test(siftgpu.BFMatcher(siftgpu.NORM_L1).knnMatch(d1, d0, 2))
    obj = np.array([[kp1[m.queryIdx]["x"], kp1[m.queryIdx]["y"]] for m in good], np.float32)
    scene = np.array([[kp0[m.trainIdx]["x"], kp0[m.trainIdx]["y"]] for m in good], np.float32)
    H, mask = siftgpu.findHomography(obj, scene, siftgpu.RANSAC)
    assert H is not None and mask.sum() >= 8
    corners = np.array([[0, 0], [180, 0], [180, 250], [0, 250]], np.float32)
    mapped = siftgpu.perspectiveTransform(corners, H)
    np.testing.assert_allclose(mapped, corners + np.array([dx, dy], np.float32), atol=1.0)
