"""Matcher: BFMatcher(NORM_L1).knnMatch(k=2) + the 0.86
ratio test of src/main.cpp:25-40.

CPU: the restatement oracle/match.py against an independent scalar
restatement of normL1_'s summation order, the tie rule, edge cases and the
committed fixture tests/golden/match.npz (made by make_match_golden.py from
the oracle on the real descriptors of book.npz / synth1_240x320.npz).
GPU (-m gpu): match.hip through the C ABI, bit-exact (indices and float
distances) against the fixture and the oracle, including ties, n_train < k,
empty inputs and a 5000 x 7000 case checked on a sample of queries.
Parity against OpenCV itself is unpinned (OpenCV is not in this image)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_bits_equal, load_golden

import match as M


def _scalar_l1(a, b):
    """normL1_ with two 4-lane accumulators (x86 SSE3 baseline), one pair."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    p = [np.float32(0)] * 8
    for j in range(128):
        p[j % 8] = np.float32(p[j % 8] + np.float32(abs(np.float32(a[j] - b[j]))))
    q = [np.float32(p[k] + p[k + 4]) for k in range(4)]
    return np.float32(np.float32(q[0] + q[1]) + np.float32(q[2] + q[3]))


def _rootsift_like(rng, n):
    x = rng.random((n, 128)).astype(np.float32) ** 3
    x /= x.sum(1, keepdims=True)
    return np.sqrt(x).astype(np.float32)


# ---- CPU: oracle ---------------------------------------------------------------
def test_oracle_matches_scalar_order():
    rng = np.random.default_rng(1)
    q, t = _rootsift_like(rng, 7), _rootsift_like(rng, 9)
    d = M.l1_distances(q, t)
    for i in range(len(q)):
        for j in range(len(t)):
            assert d[i, j].tobytes() == _scalar_l1(q[i], t[j]).tobytes()
    ref = np.abs(q[:, None, :].astype(np.float64) - t[None, :, :]).sum(-1)
    np.testing.assert_allclose(d, ref, rtol=1e-5)


def test_oracle_tie_keeps_earlier_index_and_short_train():
    rng = np.random.default_rng(2)
    t = _rootsift_like(rng, 5)
    t = np.concatenate([t, t[1:2], t[1:2]])         # rows 5 and 6 duplicate row 1
    idx, dist = M.knn_match(t[1:2], t, 2)
    assert idx.tolist() == [[1, 5]] and dist[0, 0] == 0 and dist[0, 1] == 0
    idx, dist = M.knn_match(t[:3], t[:1], 2)         # n_train < k
    assert (idx[:, 0] == 0).all() and (idx[:, 1] == -1).all() and np.isinf(dist[:, 1]).all()
    idx, dist = M.knn_match(t[:3], t[:0], 2)
    assert (idx == -1).all()


def test_ratio_test_semantics():
    idx = np.array([[3, 4], [5, -1], [1, 2]], np.int32)
    dist = np.array([[0.86, 1.0], [0.1, np.inf], [0.9, 1.0]], np.float32)
    kept = M.ratio_test(idx, dist)
    # 0.86f <= 0.86 * 1.0 in double: float(0.86f) = 0.8600000143 > 0.86 -> rejected
    assert kept == []
    dist[0, 0] = np.float32(0.859)
    assert [k[:2] for k in M.ratio_test(idx, dist)] == [(0, 3)]


def test_oracle_matches_fixture():
    g = load_golden("match")
    book = load_golden("book")["desc"]
    synth = load_golden("synth1_240x320")["desc"]
    for name, q, t in [("book_synth", book, synth), ("synth_book", synth, book),
                       ("book_dup", book, g["dup"]), ("book_noisy", book, g["noisy"])]:
        idx, dist = M.knn_match(q, t, 2)
        assert_bits_equal(idx, g[f"{name}_idx"], name)
        assert_bits_equal(dist, g[f"{name}_dist"], name)
    # the duplicated rows produce real ties: earlier index first, equal distances
    ti = g["book_dup_idx"]
    td = g["book_dup_dist"]
    ties = (ti[:, 0] < 40) & (ti[:, 1] == ti[:, 0] + 104)
    assert ties.any() and (td[ties, 0] == td[ties, 1]).all()


def test_python_mirror_api_shape(siftgpu):
    """BFMatcher / ratio_test mirror the reference's types without a GPU call."""
    m = [[siftgpu.DMatch(0, 3, 0, 0.5), siftgpu.DMatch(0, 4, 0, 1.0)],
         [siftgpu.DMatch(1, 2, 0, 0.9), siftgpu.DMatch(1, 7, 0, 1.0)], [siftgpu.DMatch(2, 1, 0, 0.1)]]
    good = siftgpu.ratio_test(m)
    assert [(x.queryIdx, x.trainIdx) for x in good] == [(0, 3)]
    with pytest.raises(ValueError):
        siftgpu.BFMatcher(normType=4)


# ---- GPU: match.hip through the C ABI -------------------------------------------
@pytest.mark.gpu
def test_gpu_knn_matches_fixture(ctx):
    g = load_golden("match")
    book = load_golden("book")["desc"]
    synth = load_golden("synth1_240x320")["desc"]
    for name, q, t in [("book_synth", book, synth), ("synth_book", synth, book),
                       ("book_dup", book, g["dup"]), ("book_noisy", book, g["noisy"])]:
        idx, dist = ctx.knnMatch(q, t, 2)
        assert_bits_equal(idx, g[f"{name}_idx"], name + " idx")
        assert_bits_equal(dist, g[f"{name}_dist"], name + " dist")


@pytest.mark.gpu
@pytest.mark.parametrize("nq,nt,k", [(1, 1, 2), (3, 0, 2), (5, 2, 2), (64, 65, 1), (200, 333, 2),
                                     (129, 4097, 2)])
def test_gpu_knn_edges_vs_oracle(ctx, nq, nt, k):
    rng = np.random.default_rng(nq * 1000 + nt)
    q, t = _rootsift_like(rng, nq), _rootsift_like(rng, nt)
    if nt > 3:
        t[nt // 2] = t[1]                       # a duplicated train row
        q[0] = t[1]                             # exact hit, tied with the duplicate
    idx, dist = ctx.knnMatch(q, t, k)
    ridx, rdist = M.knn_match(q, t, k)
    assert_bits_equal(idx, ridx, "idx")
    assert_bits_equal(dist, rdist, "dist")


@pytest.mark.gpu
def test_gpu_knn_empty_query(ctx):
    idx, dist = ctx.knnMatch(np.zeros((0, 128), np.float32), np.ones((4, 128), np.float32), 2)
    assert idx.shape == (0, 2)


@pytest.mark.gpu
def test_gpu_knn_large_sampled(ctx):
    """5000 x 7000 (many splits): a sample of queries against the oracle."""
    rng = np.random.default_rng(11)
    q, t = _rootsift_like(rng, 5000), _rootsift_like(rng, 7000)
    idx, dist = ctx.knnMatch(q, t, 2)
    s = rng.choice(5000, 150, replace=False)
    ridx, rdist = M.knn_match(q[s], t, 2)
    assert_bits_equal(idx[s], ridx, "idx")
    assert_bits_equal(dist[s], rdist, "dist")
    assert (dist[:, 0] <= dist[:, 1]).all()


@pytest.mark.gpu
def test_gpu_reference_app_flow(siftgpu):
    """src/main.cpp:23-40 on the book image and a shifted crop of it: SIFT_NCL
    twice, knnMatch(d1, d0, 2), ratio 0.86; the kept matches are the oracle's
    and mostly agree with the known shift."""
    from conftest import book_image
    img0 = book_image()
    dy, dx = 7, 11
    img1 = np.ascontiguousarray(img0[dy:, dx:])
    kp0, d0 = siftgpu.SIFT_NCL(img0)
    kp1, d1 = siftgpu.SIFT_NCL(img1)
    matches = siftgpu.BFMatcher(siftgpu.NORM_L1).knnMatch(d1, d0, 2)
    good = siftgpu.ratio_test(matches)
    ridx, rdist = M.knn_match(d1, d0, 2)
    ref = M.ratio_test(ridx, rdist)
    assert [(m.queryIdx, m.trainIdx, np.float32(m.distance)) for m in good] == \
        [(a, b, np.float32(c)) for a, b, c in ref]
    assert len(good) >= 10
    ok = sum(abs(kp1[m.queryIdx]["x"] + dx - kp0[m.trainIdx]["x"]) < 1.5 and
             abs(kp1[m.queryIdx]["y"] + dy - kp0[m.trainIdx]["y"]) < 1.5 for m in good)
    assert ok >= 0.8 * len(good)
