"""CPU tests of the oracle (oracle/sift_oracle.c): each OpenCV helper it
restates is checked against an independent numpy/double re-derivation, the
whole path against the committed golden fixtures, plus size-independent
properties.  PARITY UNPINNED vs the real reference (see sift_oracle.h)."""
import math
import os

import numpy as np
import pytest

from conftest import ROOT, book_image, kp_bytes, load_golden, sha

PI_REF = 3.14159265359          # src/sift.cpp:7
PYR_SIGMAS = [math.sqrt(1.6 * 1.6 + 0.2 * 0.2)] + [
    float(np.float32(math.sqrt((2 ** (i / 2) * 1.6) ** 2 - 1.6 ** 2))) for i in range(1, 5)]


def np_gaussian_kernel(sigma):
    """src/sift.cpp:95-108 in Python doubles (float chain for 2*sigma*sigma)."""
    s = np.float32(sigma)
    w = int(math.floor(np.float32(3) * s))
    norm = 1.0 / (2 * PI_REF * float(s) * float(s))
    den = float(np.float32(np.float32(2) * s) * s)
    k = np.empty((2 * w + 1, 2 * w + 1), np.float32)
    for a in range(-w, w + 1):
        for b in range(-w, w + 1):
            k[a + w, b + w] = np.float32(norm * math.exp(-(a * a + b * b) * 1.0 / den) * 8192)
    return k


@pytest.mark.parametrize("sigma", PYR_SIGMAS + [0.7, 2.0, 3.3])
def test_gaussian_kernel_bitexact(oracle, sigma):
    k = oracle.gaussian_kernel(sigma)
    ref = np_gaussian_kernel(sigma)
    assert k.shape == ref.shape
    assert k.tobytes() == ref.tobytes()


def test_pyramid_kernel_widths(oracle):
    # ksize 9, 9, 17, 25, 37
    assert [oracle.gaussian_kernel(s).shape[0] for s in PYR_SIGMAS] == [9, 9, 17, 25, 37]


def np_exp32f(x):
    """hal::exp32f restated in numpy float32 (independent of the C code)."""
    A0 = .9670371139572337719125840413672004409288e-2
    pre = 1.4426950408889634073599246810019 * 64
    tab = np.array([np.float32(float(np.longdouble(2) ** (np.longdouble(j) / 64)) * A0)
                    for j in range(64)], np.float32)
    A1 = np.float32(.5550339366753125211915322047004666939128e-1 / A0)
    A2 = np.float32(.2402265109513301490103372422686535526573 / A0)
    A3 = np.float32(.6931471805521448196800669615864773144641 / A0)
    A4 = np.float32(1.000000000000002438532970795181890933776 / A0)
    lo, hi = np.float32(-3000. * 64 / pre), np.float32(3000. * 64 / pre)
    v = np.minimum(np.maximum(x.astype(np.float32), lo), hi) * np.float32(pre)
    vi = np.rint(v).astype(np.int32)
    v = (v - vi.astype(np.float32)) * np.float32(1. / 64)
    t = (vi >> 6) + 127
    t = np.where((t & ~255) == 0, t, np.where(t < 0, 0, 255)).astype(np.int32)
    sc = (t << 23).view(np.float32)
    poly = (((v + A1) * v + A2) * v + A3) * v + A4
    return (sc * tab[vi & 63]) * poly


def test_scatter_blur_tables_match_oracle(oracle, tmp_path):
    """The compile-time tables of the scatter-form blur (blur.hip,
    build/sym_coefs.inc, printed by csrc/gen_sym_coefs.cpp) against the
    oracle's getGaussianKernel for the same sigmas: every quadrant entry
    K[|a|][|b|], bit for bit, and the five SIFT_NCL widths."""
    import re
    import subprocess
    src = os.path.join(ROOT, "sift-gpu_amd", "csrc", "gen_sym_coefs.cpp")
    exe = str(tmp_path / "gen")
    subprocess.run(["g++", "-O0", "-fno-builtin", "-std=c++17", "-o", exe, src, "-lm"], check=True)
    text = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    tables = re.findall(r"constexpr int kSymW(\d) = (\d+);  // sigma (\S+)\nconstexpr float kSymK\d\[\d+\]\[\d+\] = "
                        r"\{\n(.*?)\n\};", text, re.S)
    assert [int(t[1]) for t in tables] == [4, 4, 8, 12, 18]
    for _, w, sig, body in tables:
        w = int(w)
        got = np.array([float.fromhex(v.rstrip("f")) for v in re.findall(r"-?0x[0-9a-fp.+-]+f", body)],
                       np.float32).reshape(w + 1, w + 1)
        ref = oracle.gaussian_kernel(float.fromhex(sig))
        assert ref.shape == (2 * w + 1, 2 * w + 1)
        np.testing.assert_array_equal(got.view(np.uint32), ref[w:, w:].view(np.uint32))


def test_exp32f(oracle):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-30, 5, 200000), np.linspace(-12.5, 0, 5001)]).astype(np.float32)
    y = oracle.exp32f(x)
    assert y.tobytes() == np_exp32f(x).tobytes()
    rel = np.abs(y.astype(np.float64) / np.exp(x.astype(np.float64)) - 1)
    assert rel.max() < 3e-6   # exp32f: a few float ulps


def np_fast_atan2(y, x):
    deg = np.float32(180 / math.pi)
    p1, p3 = np.float32(0.9997878412794807) * deg, np.float32(-0.3258083974640975) * deg
    p5, p7 = np.float32(0.1555786518463281) * deg, np.float32(-0.04432655554792128) * deg
    ax, ay = np.abs(x), np.abs(y)
    c = np.minimum(ax, ay) / (np.maximum(ax, ay) + np.float32(np.finfo(np.float64).eps))
    c2 = c * c
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    a = np.where(ax >= ay, a, np.float32(90) - a)
    a = np.where(x < 0, np.float32(180) - a, a)
    return np.where(y < 0, np.float32(360) - a, a).astype(np.float32)


def test_fast_atan2(oracle):
    rng = np.random.default_rng(1)
    y = rng.integers(-255, 256, 300000).astype(np.float32)
    x = rng.integers(-255, 256, 300000).astype(np.float32)
    a = oracle.fast_atan2(y, x)
    assert a.tobytes() == np_fast_atan2(y, x).tobytes()
    ref = np.degrees(np.arctan2(y.astype(np.float64), x.astype(np.float64))) % 360
    err = np.abs(a - ref)
    err = np.minimum(err, 360 - err)
    assert err.max() < 0.01   # OpenCV documents ~0.3 degree; this polynomial is ~0.005
    assert a.min() >= 0 and a.max() <= 360


def test_magnitude(oracle):
    rng = np.random.default_rng(2)
    x = rng.normal(0, 50, 100000).astype(np.float32)
    y = rng.normal(0, 50, 100000).astype(np.float32)
    assert oracle.magnitude(x, y).tobytes() == np.sqrt(x * x + y * y).astype(np.float32).tobytes()


def test_solve3(oracle):
    rng = np.random.default_rng(3)
    for _ in range(200):
        a = rng.normal(size=(3, 3)).astype(np.float32)
        a = a + a.T + np.eye(3, dtype=np.float32) * 3
        b = rng.normal(size=3).astype(np.float32)
        x, ok = oracle.solve3(a, b)
        assert ok
        np.testing.assert_allclose(x, np.linalg.solve(a.astype(np.float64), b), rtol=1e-4, atol=1e-5)
    x, ok = oracle.solve3(np.ones((3, 3), np.float32), np.ones(3, np.float32))
    assert not ok and not x.any()        # singular -> Matx::zeros()


def test_cv_round_half_even(oracle):
    assert [oracle.cv_round(v) for v in (0.5, 1.5, 2.5, -0.5, -1.5, 2.4999, 2.5001)] == [0, 2, 2, 0, -2, 2, 3]


@pytest.mark.parametrize("shape", [(300, 210), (150, 105), (135, 240), (75, 52)])
def test_resize_nn(oracle, shape):
    r, c = shape
    src = np.arange(r * c, dtype=np.float32).reshape(r, c)
    dst = oracle.resize_nn(src, r // 2, c // 2)
    ify, ifx = 1.0 / ((r // 2) / r), 1.0 / ((c // 2) / c)
    ys = np.minimum(np.floor(np.arange(r // 2) * ify).astype(int), r - 1)
    xs = np.minimum(np.floor(np.arange(c // 2) * ifx).astype(int), c - 1)
    assert dst.tobytes() == src[np.ix_(ys, xs)].tobytes()
    if r % 2 == 0 and c % 2 == 0:
        assert dst.tobytes() == src[::2, ::2].tobytes()


def test_blur_ignores_last_row_and_col(oracle):
    # getSubMatrix treats rows >= rows-1 and cols >= cols-1 as zero (src/sift.cpp:116)
    img = np.zeros((40, 50), np.float32)
    img[-1, :] = 255
    img[:, -1] = 255
    assert not oracle.gaussian_blur(img, 1.6).any()


def test_blur_delta_is_kernel(oracle):
    img = np.zeros((41, 41), np.float32)
    img[20, 20] = 1
    out = oracle.gaussian_blur(img, 1.6)
    k = np_gaussian_kernel(1.6)
    np.testing.assert_array_equal(out[16:25, 16:25], k[::-1, ::-1] / np.float32(8192))


def np_synth(b, rows, cols):
    S = [3, 6, 12, 24, 48, 96]
    A = [48, 56, 56, 48, 40, 32]
    s = np.uint32(0x5EED0000 + b)
    y, x = np.mgrid[0:rows, 0:cols].astype(np.int64)

    def lowbias(v):
        v = v.astype(np.uint64) & 0xFFFFFFFF
        v ^= v >> 16
        v = (v * 0x7feb352d) & 0xFFFFFFFF
        v ^= v >> 15
        v = (v * 0x846ca68b) & 0xFFFFFFFF
        v ^= v >> 16
        return v

    acc = np.zeros((rows, cols), np.int64)
    for k in range(6):
        salt = (int(s) * 0x9E3779B1 + k * 0x85EBCA6B) & 0xFFFFFFFF
        gx, gy = x // S[k], y // S[k]
        fx, fy = (x % S[k]) * 256 // S[k], (y % S[k]) * 256 // S[k]

        def L(a, bb):
            h = ((a * 73856093) & 0xFFFFFFFF) ^ ((bb * 19349663) & 0xFFFFFFFF) ^ salt
            return (lowbias(h) & 255).astype(np.int64) - 128
        v = ((L(gx, gy) * (256 - fx) + L(gx + 1, gy) * fx) * (256 - fy)
             + (L(gx, gy + 1) * (256 - fx) + L(gx + 1, gy + 1) * fx) * fy) >> 16
        acc += A[k] * v
    return np.clip(128 + (acc >> 7), 0, 255).astype(np.float32)


@pytest.mark.parametrize("b,shape", [(0, (64, 96)), (7, (33, 57))])
def test_synth_generator(oracle, b, shape):
    assert oracle.synth_image(b, *shape).tobytes() == np_synth(b, *shape).tobytes()


GOLDEN_CASES = ["book", "synth0_160x128", "synth1_240x320", "synth2_203x157"]


def golden_input(name, oracle):
    if name == "book":
        return book_image()
    g = load_golden(name)
    b = int(name[5])
    return oracle.synth_image(b, int(g["rows"]), int(g["cols"]))


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_golden(oracle, name):
    g = load_golden(name)
    img = golden_input(name, oracle)
    r, c = img.shape
    gp = oracle.build_gaussian_pyramid(img)
    dp = oracle.build_dog_pyramid(gp, r, c)
    assert [sha(p) for p in oracle.split_planes(gp, r, c, 5, 5)] == list(g["gpyr_sha"])
    assert [sha(p) for p in oracle.split_planes(dp, r, c, 5, 4)] == list(g["dog_sha"])
    kps, desc = oracle.sift(img)
    assert kp_bytes(kps).tobytes() == g["kps"].tobytes()
    assert desc.tobytes() == g["desc"].tobytes()


def test_oracle_1080p_golden(oracle):
    """Full-size pin of the oracle (about 10 s on one core)."""
    g = load_golden("synth0_1080x1920")
    img = oracle.synth_image(0, 1080, 1920)
    kps, desc = oracle.sift(img)
    assert len(kps) == int(g["n"])
    assert sha(kps) == str(g["kp_sha"]) and sha(desc) == str(g["desc_sha"])


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_descriptor_properties(name):
    g = load_golden(name)
    desc = g["desc"]
    kps = g["kps"].view(np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                   ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])).reshape(-1)
    assert len(kps) == len(desc) > 0
    # RootSIFT of uchar-quantised values: unit L2 norm, non-negative (src/sift.cpp:711-721)
    np.testing.assert_allclose(np.linalg.norm(desc, axis=1), 1.0, atol=2e-6)
    assert desc.min() >= 0
    # squares are q_k / sum(q): multiples of a common 1/sum -> ratios of small integers
    q = desc.astype(np.float64) ** 2
    qn = q / q[q > 0].min(axis=None)
    assert np.all(qn < 300)
    o = kps["octave"] & 255
    layer = (kps["octave"] >> 8) & 255
    assert np.all(o <= 4) and np.all((layer >= 1) & (layer <= 2))
    assert np.all(kps["class_id"] == -1)
    assert np.all((kps["angle"] >= 0) & (kps["angle"] < 360))
    # reference emission order is octave-major (the stored layer is the refined
    # one, which may move between 1 and 2, so only the octave is monotone)
    assert np.all(np.diff(o) >= 0)


def test_flat_image_has_no_keypoints(oracle):
    kps, desc = oracle.sift(np.full((64, 64), 100, np.float32))
    assert len(kps) == 0 and desc.shape == (0, 128)
