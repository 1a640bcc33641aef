"""GPU parity tests: the HIP path, called through the C ABI, against the CPU
oracle and the committed golden fixtures.  Bar: bit-exact for every stage and
for the full SIFT_NCL output (keypoints and descriptors), at small sizes live
against the oracle and at 1920x1080 against golden SHA-256 digests."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import (GOLDEN, PKG, ROOT, assert_bits_equal, book_image, kp_bytes, load_golden,
                      sha)

pytestmark = pytest.mark.gpu

PYR_SIGMAS = [1.6124515496597098, 1.6, 2.7712812921102037, 4.233202097703346, 6.196773353931867]


# ---- device arithmetic helpers vs the oracle ---------------------------------
def _helper_inputs(op, rng, n):
    if op == 0:   # exp32f arguments: Gaussian weights are <= 0
        return rng.uniform(-40, 2, n).astype(np.float32), None
    if op in (1, 2):  # gradients: differences of 0..255 image values, and general floats
        a = np.concatenate([rng.integers(-255, 256, n // 2), rng.normal(0, 40, n - n // 2)]).astype(np.float32)
        b = np.concatenate([rng.integers(-255, 256, n // 2), rng.normal(0, 40, n - n // 2)]).astype(np.float32)
        return a, b
    if op in (3, 4):  # angles in radians, [0, 2pi)
        return (rng.random(n) * 2 * np.pi).astype(np.float32), None
    if op == 5:   # (layer + xi) / 2 in (0.25, 1.25)
        return rng.uniform(0.2, 1.3, n).astype(np.float32), None
    x = rng.normal(0, 100, n).astype(np.float32)
    x[: n // 8] = np.round(x[: n // 8]) + 0.5       # exact halves for cvRound
    return x, None


@pytest.mark.parametrize("op", range(8))
def test_device_math_helpers_bitexact(ctx, oracle, op):
    rng = np.random.default_rng(100 + op)
    a, b = _helper_inputs(op, rng, 1 << 21)
    gpu = ctx.selftest_math(op, a, b)
    cpu = oracle.helper(op, a, b)
    bad = np.count_nonzero(gpu.view(np.uint32) != cpu.view(np.uint32))
    # cos/sin/exp2 go through double precision on both sides; a mismatch could
    # only come from a double result within 2^-29 ulp of a float midpoint.
    assert bad == 0, f"op {op}: {bad} of {a.size} differ"


# ---- single stages ---------------------------------------------------------------
@pytest.mark.parametrize("sigma", PYR_SIGMAS + [0.7, 1.0, 3.3])
def test_gaussian_blur_bitexact(ctx, oracle, sigma):
    img = oracle.synth_image(3, 97, 131)
    assert_bits_equal(ctx.Gaussian_Blur(img, sigma), oracle.gaussian_blur(img, sigma), f"blur {sigma}")


def test_gaussian_blur_book_and_1080p(ctx, oracle):
    book = book_image()
    assert_bits_equal(ctx.Gaussian_Blur(book, PYR_SIGMAS[4]), oracle.gaussian_blur(book, PYR_SIGMAS[4]), "book")
    img = oracle.synth_image(4, 1080, 1920)
    assert_bits_equal(ctx.Gaussian_Blur(img, PYR_SIGMAS[4]), oracle.gaussian_blur(img, PYR_SIGMAS[4]), "1080p")


@pytest.mark.parametrize("sigma", [1.6, 2.5, 4.0])
def test_gaussian_blur_1d_bitexact(ctx, oracle, sigma):
    img = oracle.synth_image(5, 97, 131)
    assert_bits_equal(ctx.Gaussian_Blur_1D(img, sigma), oracle.gaussian_blur_1d(img, sigma), f"blur1d {sigma}")


@pytest.mark.parametrize("shape,b", [((130, 90), 3), ((203, 157), 2), ((256, 256), 6)])
def test_gaussian_pyramid_bitexact(ctx, oracle, shape, b):
    img = oracle.synth_image(b, *shape)
    gp = ctx.buildGaussianPyramid(img, 5)
    ref = oracle.split_planes(oracle.build_gaussian_pyramid(img), *shape, 5, 5)
    for i, (p, q) in enumerate(zip(gp, ref)):
        assert_bits_equal(p, q, f"gpyr plane {i}")


def test_dog_extrema_descriptors_bitexact(ctx, oracle):
    img = oracle.synth_image(7, 240, 320)
    r, c = img.shape
    g = oracle.build_gaussian_pyramid(img)
    d = oracle.build_dog_pyramid(g, r, c)
    gpl = oracle.split_planes(g, r, c, 5, 5)
    dpl = oracle.split_planes(d, r, c, 5, 4)
    for i, (p, q) in enumerate(zip(ctx.buildDoGPyramid(gpl, 5), dpl)):
        assert_bits_equal(p, q, f"dog plane {i}")
    kps_ref = oracle.find_scale_space_extrema(g, d, r, c)
    kps = ctx.findScaleSpaceExtrema(gpl, dpl, 5)
    assert len(kps) == len(kps_ref) > 50
    assert_bits_equal(kp_bytes(kps), kp_bytes(kps_ref), "keypoints")
    desc_ref = oracle.calc_descriptors(g, r, c, kps_ref)
    assert_bits_equal(ctx.calDescriptor(gpl, kps_ref, 0), desc_ref, "descriptors")


def test_descriptors_caller_keypoints_bitexact(ctx, oracle):
    """calDescriptor (src/sift.cpp:733-753) on caller-supplied keypoints: every
    octave, layers 1-2, sub-pixel positions including the image border and
    beyond it, angles 0 / near 360 / random, and sizes whose window radius
    exceeds 40 (the whole-window enumeration path) -- windows that reach the
    border cells and the trash row of the interior-only histogram."""
    img = oracle.synth_image(11, 240, 320)
    r, c = img.shape
    g = oracle.build_gaussian_pyramid(img)
    gpl = oracle.split_planes(g, r, c, 5, 5)
    rng = np.random.default_rng(5)
    n = 600
    kps = np.zeros(n, oracle.KEYPOINT_DTYPE)
    o = rng.integers(0, 5, n)
    layer = rng.integers(1, 3, n)
    size_oct = np.where(rng.random(n) < 0.25, rng.uniform(7.6, 12.0, n), rng.uniform(1.5, 7.0, n))
    kps["x"] = rng.uniform(-3.0, c + 3.0, n).astype(np.float32)
    kps["y"] = rng.uniform(-3.0, r + 3.0, n).astype(np.float32)
    kps["size"] = (size_oct * (1 << o)).astype(np.float32)
    ang = rng.uniform(0, 360, n).astype(np.float32)
    ang[:40] = 0.0
    ang[40:80] = np.nextafter(np.float32(360), np.float32(0))
    kps["angle"] = ang
    kps["octave"] = (o + (layer << 8)).astype(np.int32)
    desc_ref = oracle.calc_descriptors(g, r, c, kps)
    assert_bits_equal(ctx.calDescriptor(gpl, kps, 0), desc_ref, "descriptors")


# ---- full SIFT_NCL ---------------------------------------------------------------
GOLDEN_CASES = ["book", "synth0_160x128", "synth1_240x320", "synth2_203x157"]


def _golden_img(name, oracle):
    if name == "book":
        return book_image()
    g = load_golden(name)
    return oracle.synth_image(int(name[5]), int(g["rows"]), int(g["cols"]))


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_sift_ncl_matches_golden(ctx, oracle, name):
    g = load_golden(name)
    kps, desc = ctx.SIFT_NCL(_golden_img(name, oracle))
    assert len(kps) == int(g["n"])
    assert_bits_equal(kp_bytes(kps), g["kps"], f"{name} keypoints")
    assert_bits_equal(desc, g["desc"], f"{name} descriptors")


@pytest.mark.parametrize("shape,b", [((256, 384), 5), ((480, 640), 9), ((16, 16), 11), ((33, 1200), 12)])
def test_sift_ncl_matches_oracle(ctx, oracle, shape, b):
    img = oracle.synth_image(b, *shape)
    kps_ref, desc_ref = oracle.sift(img)
    kps, desc = ctx.SIFT_NCL(img)
    assert_bits_equal(kp_bytes(kps), kp_bytes(kps_ref), "keypoints")
    assert_bits_equal(desc, desc_ref, "descriptors")


def test_sift_ncl_1080p_golden(ctx, oracle):
    g = load_golden("synth0_1080x1920")
    img = oracle.synth_image(0, 1080, 1920)
    gp = ctx.buildGaussianPyramid(img, 5)
    assert [sha(p) for p in gp] == list(g["gpyr_sha"])
    dp = ctx.buildDoGPyramid(gp, 5)
    assert [sha(p) for p in dp] == list(g["dog_sha"])
    kps, desc = ctx.SIFT_NCL(img)
    assert len(kps) == int(g["n"]) == 12932
    assert sha(kps) == str(g["kp_sha"])
    assert sha(desc) == str(g["desc_sha"])
    # size-independent properties at full size
    np.testing.assert_allclose(np.linalg.norm(desc, axis=1), 1.0, atol=2e-6)
    assert np.all(np.diff(kps["octave"] & 255) >= 0)


def test_sift_ncl_8k_golden(siftgpu, oracle):
    """Maximum size: a 7680x4320 image (16x the 1080p workload) against the
    oracle's digests (tests/golden/make_golden.py --8k): every Gaussian and DoG
    plane, the 214,633 keypoints and their descriptors, bit for bit."""
    g = load_golden("synth0_4320x7680")
    img = oracle.synth_image(0, 4320, 7680)
    with siftgpu.Context(4320, 7680, 1, device=0) as c8k:
        gp = c8k.buildGaussianPyramid(img, 5)
        assert [sha(p) for p in gp] == list(g["gpyr_sha"])
        dp = c8k.buildDoGPyramid(gp, 5)
        assert [sha(p) for p in dp] == list(g["dog_sha"])
        del gp, dp
        kps, desc = c8k.SIFT_NCL(img)
    assert len(kps) == int(g["n"]) == 214633
    assert sha(kps) == str(g["kp_sha"])
    assert sha(desc) == str(g["desc_sha"])


def test_plateaus_and_ties(ctx, oracle):
    """Blocky input: many exactly-equal DoG neighbours exercise the >= ties."""
    rng = np.random.default_rng(4)
    img = np.kron(rng.integers(0, 4, (24, 32)) * 60.0, np.ones((8, 8))).astype(np.float32)
    kps_ref, desc_ref = oracle.sift(img)
    kps, desc = ctx.SIFT_NCL(img)
    assert_bits_equal(kp_bytes(kps), kp_bytes(kps_ref), "keypoints")
    assert_bits_equal(desc, desc_ref, "descriptors")


def test_flat_and_dark_images(ctx):
    for v in (0.0, 100.0, 255.0):
        kps, desc = ctx.SIFT_NCL(np.full((64, 80), v, np.float32))
        assert len(kps) == 0 and desc.shape == (0, 128)


def test_four_octaves_is_prefix_of_five(ctx, oracle):
    img = oracle.synth_image(8, 300, 420)
    kps5, desc5 = oracle.sift(img, 5)
    keep = (kps5["octave"] & 255) <= 3
    ctx.set_octaves(4)
    try:
        kps4, desc4 = ctx.SIFT_NCL(img)
    finally:
        ctx.set_octaves(5)
    assert_bits_equal(kp_bytes(kps4), kp_bytes(kps5[keep]), "keypoints")
    assert_bits_equal(desc4, desc5[keep], "descriptors")


# ---- scatter-form blur (blur.hip blur_sym_kernel) --------------------------------
# The library picks the scatter walk for launches of >= SIFT_HIP_SYM_MIN
# (256) 64-column strips x images (octaves 0-3 of a 64 x 1080p batch) and the
# 2-D tiles otherwise; these tests force each path (the variables are read
# when a context is created).
@pytest.mark.parametrize("shape,b", [((130, 90), 3), ((203, 157), 2), ((300, 421), 9), ((40, 1500), 4),
                                     ((700, 70), 6)])
def test_scatter_blur_pyramid_bitexact(siftgpu, oracle, monkeypatch, shape, b):
    monkeypatch.setenv("SIFT_HIP_SYM_MIN", "0")
    monkeypatch.setenv("SIFT_HIP_SYM_ROWS_MIN", "0")
    img = oracle.synth_image(b, *shape)
    ref = oracle.split_planes(oracle.build_gaussian_pyramid(img), *shape, 5, 5)
    with siftgpu.Context(*shape, 1, device=0) as c:
        gp = c.buildGaussianPyramid(img, 5)
    for i, (p, q) in enumerate(zip(gp, ref)):
        assert_bits_equal(p, q, f"gpyr plane {i}")


@pytest.mark.parametrize("mode", ["sym", "gather", "small"])
def test_blur_paths_1080p_and_8k_planes(siftgpu, oracle, monkeypatch, mode):
    """Every blur path at full size against the CPU path's plane digests: the
    scatter walk's multi-chunk plans (a 1080p or 8K image is split into
    chunks per scale) in XCD-contiguous wave order (padding blocks included),
    the 2-D 8-pixel tiles, and the 2-output tiles of small launches
    (blur_small_kernel) forced onto every octave."""
    monkeypatch.setenv("SIFT_HIP_SYM_MIN", "0" if mode == "sym" else "1000000000")
    monkeypatch.setenv("SIFT_HIP_SYM_ROWS_MIN", "0")
    monkeypatch.setenv("SIFT_HIP_SMALL_MAX", "1000000000" if mode == "small" else "0")
    for name, (R, C) in (("synth0_1080x1920", (1080, 1920)), ("synth0_4320x7680", (4320, 7680))):
        g = load_golden(name)
        img = oracle.synth_image(0, R, C)
        with siftgpu.Context(R, C, 1, device=0) as c:
            gp = c.buildGaussianPyramid(img, 5)
        assert [sha(p) for p in gp] == list(g["gpyr_sha"]), f"{name} {mode}"
        del gp


def test_scatter_blur_sift_ncl_and_batch(siftgpu, oracle, monkeypatch):
    import torch
    monkeypatch.setenv("SIFT_HIP_SYM_MIN", "0")
    monkeypatch.setenv("SIFT_HIP_SYM_ROWS_MIN", "0")
    img = oracle.synth_image(9, 480, 640)
    kps_ref, desc_ref = oracle.sift(img)
    B, R, C = 3, 240, 320
    with siftgpu.Context(480, 640, B, device=0) as c:
        kps, desc = c.SIFT_NCL(img)
        assert_bits_equal(kp_bytes(kps), kp_bytes(kps_ref), "keypoints")
        assert_bits_equal(desc, desc_ref, "descriptors")
        imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
        c.synth_images(imgs.data_ptr(), B, R, C, C, R * C, seed_base=40)
        cap = 20000
        kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
        dsc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
        offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
        c.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kpts.data_ptr(), dsc.data_ptr(), cap,
                               offs.data_ptr())
        c.sync()
        o = offs.cpu().numpy()
        k = kpts.cpu().numpy().view(np.uint8).reshape(cap, 28)
        dd = dsc.cpu().numpy()
    for b in range(B):
        kr, dr = oracle.sift(oracle.synth_image(40 + b, R, C))
        assert o[b + 1] - o[b] == len(kr)
        assert_bits_equal(k[o[b]:o[b + 1]], kp_bytes(kr), f"batch image {b} keypoints")
        assert_bits_equal(dd[o[b]:o[b + 1]], dr, f"batch image {b} descriptors")


# ---- batch mode on device memory -----------------------------------------------
def test_batch_mode_matches_single(ctx, oracle):
    import torch
    B, R, C = 4, 240, 320
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, seed_base=20)
    ctx.sync()
    host = imgs.cpu().numpy()
    for b in range(B):
        assert_bits_equal(host[b], oracle.synth_image(20 + b, R, C), f"synth image {b}")
    cap = 20000
    kpts = torch.empty((cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
    offs = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
    ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, kpts.data_ptr(), desc.data_ptr(), cap,
                             offs.data_ptr())
    ctx.sync()
    o = offs.cpu().numpy()
    k = kpts.cpu().numpy().view(np.uint8).reshape(cap, 28)
    dd = desc.cpu().numpy()
    assert o[0] == 0 and np.all(np.diff(o) >= 0)
    for b in range(B):
        kr, dr = oracle.sift(host[b])
        assert o[b + 1] - o[b] == len(kr)
        assert_bits_equal(k[o[b]:o[b + 1]], kp_bytes(kr), f"batch image {b} keypoints")
        assert_bits_equal(dd[o[b]:o[b + 1]], dr, f"batch image {b} descriptors")


# ---- error behaviour -------------------------------------------------------------
def test_errors(ctx, siftgpu, oracle):
    with pytest.raises(siftgpu.SiftError) as e:
        ctx.SIFT_NCL(np.zeros((15, 40), np.float32))      # octave 4 would be empty
    assert e.value.code == siftgpu.SIFT_E_INVALID
    with siftgpu.Context(64, 64, 1) as small:
        with pytest.raises(siftgpu.SiftError) as e:
            small.SIFT_NCL(np.zeros((65, 64), np.float32))
        assert e.value.code == siftgpu.SIFT_E_SIZE
    # capacity: the raw ABI reports the required count
    import ctypes
    img = oracle.synth_image(1, 240, 320)
    n = ctypes.c_int(0)
    kp = np.zeros(1, siftgpu.KEYPOINT_DTYPE)
    d = np.zeros((1, 128), np.float32)
    rc = siftgpu.lib().sift_detect_compute(ctx.h, img.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 240,
                                           320, 320 * 4, kp.ctypes.data,
                                           d.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 1, ctypes.byref(n))
    assert rc == siftgpu.SIFT_E_CAPACITY and n.value == int(load_golden("synth1_240x320")["n"])
    # CV_Assert analogue: keypoint octave outside the pyramid
    gp = ctx.buildGaussianPyramid(img, 5)
    bad = np.zeros(1, siftgpu.KEYPOINT_DTYPE)
    bad["octave"] = 7 | (1 << 8)
    bad["size"] = 3
    with pytest.raises(siftgpu.SiftError) as e:
        ctx.calDescriptor(gp, bad, 0)
    assert e.value.code == siftgpu.SIFT_E_INVALID
    # the context stays usable after errors
    kps, _ = ctx.SIFT_NCL(img)
    assert len(kps) == int(load_golden("synth1_240x320")["n"])


def test_profile_stats(ctx, oracle):
    ctx.set_flags(0x2)
    try:
        ctx.SIFT_NCL(oracle.synth_image(0, 160, 128))
        st = ctx.stage_stats(reset=True)
    finally:
        ctx.set_flags(0)
    for k in ("blur_base", "blur_octave", "extrema", "refine_orient", "emit", "descriptor"):  # DoG is fused into extrema
        assert st[k]["launches"] >= 1 and st[k]["ms"] > 0
    assert st["blur_octave"]["launches"] == 5


# ---- the C++ drop-in (include/sift.hpp) --------------------------------------------
@pytest.mark.parametrize("mode", ["ncl", "modules"])
def test_cpp_shim_book(tmp_path, siftgpu, mode):
    exe = tmp_path / "sift_cli"
    lib = os.path.join(PKG, "lib")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "sift_cli.cpp"), "-o", str(exe), "-L", lib,
                    "-lsift_shim", "-lsift_hip", f"-Wl,-rpath,{lib}"], check=True)
    out = tmp_path / "out.bin"
    args = [str(exe), os.path.join(GOLDEN, "book_gray.pgm"), str(out)] + (["modules"] if mode == "modules" else [])
    subprocess.run(args, check=True, timeout=300)
    raw = out.read_bytes()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    g = load_golden("book")
    assert n == int(g["n"])
    kb = np.frombuffer(raw[4:4 + 28 * n], np.uint8).reshape(n, 28)
    db = np.frombuffer(raw[4 + 28 * n:], np.float32).reshape(n, 128)
    assert_bits_equal(kb, g["kps"], "shim keypoints")
    assert_bits_equal(db, g["desc"], "shim descriptors")


def test_cpp_main_shaped_caller_runs(tmp_path, siftgpu, oracle):
    """tests/cpp/main_shape.cpp (includes only sift.hpp, like src/main.cpp)
    runs SIFT_NCL on the GPU through the shim; its keypoint count equals the
    CPU path's on the same synthetic pattern."""
    exe = tmp_path / "main_shape"
    lib = os.path.join(PKG, "lib")
    subprocess.run(["g++", "-O1", "-std=c++17", "-fopenmp", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "main_shape.cpp"), "-o", str(exe), "-L", lib,
                    "-lsift_shim", "-lsift_hip", f"-Wl,-rpath,{lib}"], check=True)
    out = subprocess.run([str(exe), "200", "240"], check=True, timeout=300, capture_output=True, text=True).stdout
    i, j = np.meshgrid(np.arange(200), np.arange(240), indexing="ij")
    img = ((i * 7 + j * 13) % 251).astype(np.float32)
    n_ref = len(oracle.sift(img)[0])
    assert f"{n_ref} keypoints, {n_ref} x 128 descriptors" in out, (out, n_ref)


_VARIANT_RUN = r"""
import hashlib, sys
import numpy as np
import torch  # noqa: F401  (one process-wide HIP runtime)
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import oracle, siftgpu
img = oracle.synth_image(0, 1080, 1920)
with siftgpu.Context(1080, 1920, 1, device=0) as ctx:
    kps, desc = ctx.SIFT_NCL(img)
sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
print(len(kps), sha(kps), sha(desc))
"""


@pytest.mark.parametrize("env", [{"SIFT_HIP_ONE_IMAGE_PX": "0"}])
def test_kernel_variants_match_golden(env):
    """The shape-dependent variants forced onto a shape that does not pick
    them (read once per process, so each runs in a child process): one 1080p
    image through the batch orientation and descriptor kernels gives the same
    keypoints and descriptors as the one-image kernels and the CPU path.  (The
    A/B losers left the library in round 6: tools/patches/r5_variants.patch.)"""
    g = load_golden("synth0_1080x1920")
    r = subprocess.run([sys.executable, "-c", _VARIANT_RUN, PKG, os.path.join(ROOT, "oracle")],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    n, ksha, dsha = r.stdout.split()[-3:]
    assert int(n) == int(g["n"]) and ksha == str(g["kp_sha"]) and dsha == str(g["desc_sha"]), env
