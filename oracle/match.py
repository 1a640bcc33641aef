"""CPU restatement of the reference application's matcher.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline
legs as the checker -- never by the product library.

Reference: src/main.cpp:25-40 --
    BFMatcher matcher(NORM_L1);
    matcher.knnMatch(descriptors1, descriptors0, matches, 2);
    keep matches[i][0] if matches[i].size() == 2 and m1.distance <= 0.86 * m2.distance
The algorithm lives in OpenCV (not in /root/reference, not installed here):
  * distance: hal normL1_(const float*, const float*, int) -- with the x86
    SSE3 baseline, two 4-lane accumulators over 8-element steps (partial sum k
    collects elements j = k mod 8 in j order), v_reduce_sum of their sum by two
    horizontal adds, i.e. ((q0 + q1) + (q2 + q3)) with q = p[0:4] + p[4:8];
    128 elements leave no scalar tail;
  * order: batchDistance keeps the K best per query by insertion with a strict
    '<', so at equal distance the earlier train index stays first.
PARITY UNPINNED against OpenCV itself: its SIMD dispatch (e.g. AVX2, 16
partial sums) can round differently, and no OpenCV output is available here.
match.hip follows this restatement bit for bit.
"""
from __future__ import annotations

import numpy as np

RATIO = 0.86  # src/main.cpp:37


def l1_distances(query: np.ndarray, train: np.ndarray, block: int = 256) -> np.ndarray:
    """[n_query, n_train] float32 L1 distances in normL1_'s summation order."""
    q = np.ascontiguousarray(query, dtype=np.float32)
    t = np.ascontiguousarray(train, dtype=np.float32)
    assert q.ndim == 2 and t.ndim == 2 and q.shape[1] == 128 and t.shape[1] == 128
    out = np.empty((q.shape[0], t.shape[0]), np.float32)
    tg = t.reshape(t.shape[0], 16, 8)
    for s in range(0, q.shape[0], block):
        qg = q[s:s + block].reshape(-1, 1, 16, 8)
        p = np.abs(qg[:, :, 0, :] - tg[None, :, 0, :])          # p[k] = |a_k - b_k|  (0 + x == x)
        for g in range(1, 16):
            p = p + np.abs(qg[:, :, g, :] - tg[None, :, g, :])   # element 8g + k, in g order
        q4 = p[..., 0:4] + p[..., 4:8]
        out[s:s + block] = (q4[..., 0] + q4[..., 1]) + (q4[..., 2] + q4[..., 3])
    return out


def knn_match(query: np.ndarray, train: np.ndarray, k: int = 2):
    """(idx, dist) [n_query, k]: the k nearest train rows per query, ascending,
    earlier index first at equal distance; idx -1 / dist +inf where n_train < k."""
    assert k in (1, 2)
    nq, nt = len(query), len(train)
    idx = np.full((nq, k), -1, np.int32)
    dist = np.full((nq, k), np.inf, np.float32)
    if nq == 0 or nt == 0:
        return idx, dist
    d = l1_distances(query, train)
    order = np.argsort(d, axis=1, kind="stable")[:, :k]   # stable: ties keep index order
    m = order.shape[1]
    idx[:, :m] = order
    dist[:, :m] = np.take_along_axis(d, order, axis=1)
    return idx, dist


def ratio_test(idx: np.ndarray, dist: np.ndarray, ratio: float = RATIO):
    """src/main.cpp:28-40: (query index, train index, distance) of the kept
    best matches -- m1.distance <= 0.86 * m2.distance, evaluated in double."""
    keep = []
    for i in range(len(idx)):
        if idx.shape[1] < 2 or idx[i, 1] < 0:
            continue
        if float(dist[i, 0]) <= ratio * float(dist[i, 1]):
            keep.append((i, int(idx[i, 0]), float(dist[i, 0])))
    return keep
