"""CPU restatement of findHomography(obj, scene, RANSAC) + perspectiveTransform
as the reference application calls them (src/main.cpp:54-62), for checking
sift_find_homography / sift_perspective_transform value for value.

TEST INFRASTRUCTURE ONLY (tests/ import it; the product never does).

The algorithm restated is OpenCV 4.x calib3d's (not in this image, so parity
with OpenCV itself is unpinned):
  * RANSACPointSetRegistrator::run -- modelPoints 4, cv::RNG((uint64)-1)
    (multiply-with-carry: state = (uint32)state * 4164903690 + (state >> 32);
    uniform(a, b) = a + next() % (b - a)), getSubset without partial checks
    (up to 10000 attempts per hypothesis), RANSACUpdateNumIters after each
    better model, "better" = more than max(best, 3) inliers;
  * HomographyEstimatorCallback::checkSubset -- collinearity of the last point
    with every earlier pair, then the 4 triangle orientations must all agree
    between the two point sets;
  * runKernel -- normalised DLT: centroid / mean-absolute-deviation scaling,
    L^T L accumulated point by point, the eigenvector of its smallest
    eigenvalue (cyclic Jacobi, rows / columns rotated in index order), then
    de-normalisation and division by H[2][2];
  * computeError -- float reprojection error, inlier if <= (float)thr^2;
  * the final refit on the inliers and 10 Levenberg-Marquardt steps on the 8
    free entries (plain LM with Gaussian elimination; OpenCV uses LMSolver);
  * perspectiveTransform -- double arithmetic, (0, 0) when |w| <= FLT_EPSILON.
Every float sum runs in the same order as the C++ (Python floats and numpy
element-wise ops are IEEE double / float32 without contraction), so results
compare bit for bit.
"""
from __future__ import annotations

import math

import numpy as np

FLT_EPSILON = float(np.finfo(np.float32).eps)
DBL_EPSILON = float(np.finfo(np.float64).eps)
DBL_MIN = float(np.finfo(np.float64).tiny)
M32 = (1 << 32) - 1
M64 = (1 << 64) - 1


class RNG:
    """cv::RNG (multiply-with-carry)."""

    def __init__(self, state=M64):
        self.state = state & M64

    def next(self) -> int:
        self.state = ((self.state & M32) * 4164903690 + (self.state >> 32)) & M64
        return self.state & M32

    def uniform(self, a: int, b: int) -> int:
        return a if a == b else self.next() % (b - a) + a


def _collinear_last(p) -> bool:
    i = len(p) - 1
    for j in range(i):
        dx1, dy1 = p[j][0] - p[i][0], p[j][1] - p[i][1]
        for k in range(j):
            dx2, dy2 = p[k][0] - p[i][0], p[k][1] - p[i][1]
            if abs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (abs(dx1) + abs(dy1) + abs(dx2) + abs(dy2)):
                return True
    return False


def _det3(a0, a1, b0, b1, c0, c1):
    return a0 * (b1 - c1) - a1 * (b0 - c0) + (b0 * c1 - b1 * c0)


def check_subset(s, d) -> bool:
    if _collinear_last(s) or _collinear_last(d):
        return False
    neg = 0
    for t in ((0, 1, 2), (1, 2, 3), (0, 2, 3), (0, 1, 3)):
        A = _det3(s[t[0]][0], s[t[0]][1], s[t[1]][0], s[t[1]][1], s[t[2]][0], s[t[2]][1])
        B = _det3(d[t[0]][0], d[t[0]][1], d[t[1]][0], d[t[1]][1], d[t[2]][0], d[t[2]][1])
        neg += A * B < 0
    return neg == 0 or neg == 4


def smallest_eigvec(A: np.ndarray) -> np.ndarray:
    """Cyclic Jacobi on a symmetric 9x9 (float64, modified in place)."""
    with np.errstate(over="ignore"):  # th * th may overflow to inf, as in the C++: t -> 0
        return _jacobi(A)


def _jacobi(A: np.ndarray) -> np.ndarray:
    V = np.eye(9)
    for _ in range(60):
        off = 0.0
        for i in range(9):
            for j in range(i + 1, 9):
                off += A[i, j] * A[i, j]
        if off < 1e-300:
            break
        for p in range(9):
            for q in range(p + 1, 9):
                apq = A[p, q]
                if abs(apq) < 1e-300:
                    continue
                th = (A[q, q] - A[p, p]) / (2 * apq)
                t = (1.0 if th >= 0 else -1.0) / (abs(th) + math.sqrt(th * th + 1))
                c = 1 / math.sqrt(t * t + 1)
                s = t * c
                cp, cq = A[:, p].copy(), A[:, q].copy()
                A[:, p] = c * cp - s * cq
                A[:, q] = s * cp + c * cq
                rp, rq = A[p, :].copy(), A[q, :].copy()
                A[p, :] = c * rp - s * rq
                A[q, :] = s * rp + c * rq
                vp, vq = V[:, p].copy(), V[:, q].copy()
                V[:, p] = c * vp - s * vq
                V[:, q] = s * vp + c * vq
    m = 0
    for i in range(1, 9):
        if A[i, i] < A[m, m]:
            m = i
    return V[:, m].copy()


def _mat3mul(a, b):
    return [a[i * 3] * b[j] + a[i * 3 + 1] * b[3 + j] + a[i * 3 + 2] * b[6 + j] for i in range(3) for j in range(3)]


def run_kernel(M, m):
    """Normalised DLT: H mapping M (src points) to m (dst points), or None."""
    n = len(M)
    cMx = cMy = cmx = cmy = 0.0
    for i in range(n):
        cmx += m[i][0]
        cmy += m[i][1]
        cMx += M[i][0]
        cMy += M[i][1]
    cmx /= n
    cmy /= n
    cMx /= n
    cMy /= n
    smx = smy = sMx = sMy = 0.0
    for i in range(n):
        smx += abs(m[i][0] - cmx)
        smy += abs(m[i][1] - cmy)
        sMx += abs(M[i][0] - cMx)
        sMy += abs(M[i][1] - cMy)
    if abs(smx) < DBL_EPSILON or abs(smy) < DBL_EPSILON or abs(sMx) < DBL_EPSILON or abs(sMy) < DBL_EPSILON:
        return None
    smx, smy, sMx, sMy = n / smx, n / smy, n / sMx, n / sMy
    invHnorm = [1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1]
    Hnorm2 = [sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1]
    LtL = np.zeros((9, 9))
    for i in range(n):
        x, y = (m[i][0] - cmx) * smx, (m[i][1] - cmy) * smy
        X, Y = (M[i][0] - cMx) * sMx, (M[i][1] - cMy) * sMy
        Lx = np.array([X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x])
        Ly = np.array([0, 0, 0, X, Y, 1, -y * X, -y * Y, -y])
        LtL += np.outer(Lx, Lx) + np.outer(Ly, Ly)
    iu = np.triu_indices(9)
    LtL.T[iu] = LtL[iu]
    H0 = smallest_eigvec(LtL)
    R = _mat3mul(_mat3mul(invHnorm, list(H0)), Hnorm2)
    if abs(R[8]) < DBL_MIN:
        return None
    return [r / R[8] for r in R]


def find_inliers(src, dst, H, thr):
    """computeError + inlier test, float32 arithmetic where the C++ uses float."""
    sx, sy = src[:, 0].astype(np.float64), src[:, 1].astype(np.float64)
    ww = (1.0 / (H[6] * sx + H[7] * sy + 1.0)).astype(np.float32).astype(np.float64)
    dx = ((H[0] * sx + H[1] * sy + H[2]) * ww - dst[:, 0].astype(np.float64)).astype(np.float32)
    dy = ((H[3] * sx + H[4] * sy + H[5]) * ww - dst[:, 1].astype(np.float64)).astype(np.float32)
    e = dx * dx + dy * dy
    mask = (e <= np.float32(thr * thr)).astype(np.uint8)
    return mask, int(mask.sum())


def update_num_iters(p, ep, model_points, max_iters):
    p = min(max(p, 0.), 1.)
    ep = min(max(ep, 0.), 1.)
    num = max(1. - p, DBL_MIN)
    denom = 1. - math.pow(1. - ep, model_points)
    if denom < DBL_MIN:
        return 0
    num, denom = math.log(num), math.log(denom)
    if denom >= 0 or -num >= max_iters * (-denom):
        return max_iters
    return int(round(num / denom))


def refine_lm(s, d, H):
    """10 Levenberg-Marquardt steps on H[0..7] (H[8] = 1)."""
    n = len(s)
    lam = 1e-3

    def cost(h):
        c = 0.0
        for i in range(n):
            w = h[6] * s[i][0] + h[7] * s[i][1] + 1
            ex = (h[0] * s[i][0] + h[1] * s[i][1] + h[2]) / w - d[i][0]
            ey = (h[3] * s[i][0] + h[4] * s[i][1] + h[5]) / w - d[i][1]
            c += ex * ex + ey * ey
        return c

    c0 = cost(H)
    for _ in range(10):
        JtJ = np.zeros((8, 8))
        Jtr = np.zeros(8)
        for i in range(n):
            X, Y = s[i][0], s[i][1]
            w = H[6] * X + H[7] * Y + 1
            iw = 1 / w
            u = (H[0] * X + H[1] * Y + H[2]) * iw
            v = (H[3] * X + H[4] * Y + H[5]) * iw
            Jx = np.array([X * iw, Y * iw, iw, 0, 0, 0, -X * u * iw, -Y * u * iw])
            Jy = np.array([0, 0, 0, X * iw, Y * iw, iw, -X * v * iw, -Y * v * iw])
            rx, ry = u - d[i][0], v - d[i][1]
            Jtr += Jx * rx + Jy * ry
            JtJ += np.outer(Jx, Jx) + np.outer(Jy, Jy)
        A = np.zeros((8, 9))
        A[:, :8] = JtJ
        for a in range(8):
            A[a, a] = JtJ[a, a] + lam * JtJ[a, a]
        A[:, 8] = -Jtr
        ok = True
        for c in range(8):
            piv = c
            for r in range(c + 1, 8):
                if abs(A[r, c]) > abs(A[piv, c]):
                    piv = r
            if abs(A[piv, c]) < 1e-300:
                ok = False
                break
            if piv != c:
                A[[c, piv]] = A[[piv, c]]
            for r in range(c + 1, 8):
                f = A[r, c] / A[c, c]
                A[r, c:] -= f * A[c, c:]
        if not ok:
            break
        dx = [0.0] * 8
        for c in range(7, -1, -1):
            v = A[c, 8]
            for k in range(c + 1, 8):
                v -= A[c, k] * dx[k]
            dx[c] = v / A[c, c]
        Hn = [H[k] + dx[k] for k in range(8)] + [1.0]
        c1 = cost(Hn)
        if c1 < c0:
            H[:] = Hn
            c0 = c1
            lam = max(lam * 0.1, 1e-12)
        else:
            lam *= 10
    return H


def find_homography(src, dst, thr=3.0, max_iters=2000, confidence=0.995):
    """-> (H as 9 floats or None, inlier mask uint8[n])."""
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 2)
    dst = np.ascontiguousarray(dst, np.float32).reshape(-1, 2)
    n = len(src)
    none = (None, np.zeros(n, np.uint8))
    if n < 4 or not (0 < confidence < 1) or max_iters < 1:
        return none
    s = [(float(a), float(b)) for a, b in src]
    d = [(float(a), float(b)) for a, b in dst]
    if n == 4:
        best = run_kernel(s, d)
        if best is None:
            return none
        best_mask = np.ones(n, np.uint8)
    else:
        rng = RNG()
        niters, max_good, best, best_mask = max_iters, 0, None, np.zeros(n, np.uint8)
        it = 0
        while it < niters:
            idx = [0] * 4
            ok_subset = False
            for _attempt in range(10000):
                ms, md = [], []
                for i in range(4):
                    while True:
                        idx[i] = rng.uniform(0, n)
                        if idx[i] not in idx[:i]:
                            break
                    ms.append(s[idx[i]])
                    md.append(d[idx[i]])
                if check_subset(ms, md):
                    ok_subset = True
                    break
            if not ok_subset:
                if it == 0:
                    return none
                break
            model = run_kernel(ms, md)
            it += 1
            if model is None:
                continue
            mask, good = find_inliers(src, dst, model, thr)
            if good > max(max_good, 3):
                best_mask, best, max_good = mask, model, good
                niters = update_num_iters(confidence, (n - good) / n, 4, niters)
        if max_good <= 0:
            return none
        si = [s[i] for i in range(n) if best_mask[i]]
        di = [d[i] for i in range(n) if best_mask[i]]
        refit = run_kernel(si, di)
        if refit is not None:
            best = refit
        best = refine_lm(si, di, list(best))
    return [b / best[8] for b in best], best_mask


def perspective_transform(H, pts):
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
    out = np.zeros_like(pts)
    for i, (x, y) in enumerate(pts.astype(np.float64)):
        w = H[6] * x + H[7] * y + H[8]
        if abs(w) > FLT_EPSILON:
            iw = 1. / w
            out[i] = ((H[0] * x + H[1] * y + H[2]) * iw, (H[3] * x + H[4] * y + H[5]) * iw)
    return out
