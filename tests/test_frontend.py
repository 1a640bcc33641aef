"""Image front end: readImage's conversion,
src/main.cpp:79-87 -- INTER_LINEAR resize of the 8-bit BGR image (scene:
960 x 960), COLOR_RGB2GRAY on BGR bytes, CV_32F.

CPU: the restatement oracle/frontend.py against the committed fixture
(book_bgr.npz -> book_gray.pgm, the gray conversion) and resize properties.
GPU (-m gpu): frontend.hip through the C ABI, bit-exact against the fixture
and the oracle (up- and down-scaling, odd sizes with a scalar row tail,
batched device API).  Resize parity against OpenCV itself is unpinned."""
import numpy as np
import pytest

from conftest import GOLDEN, assert_bits_equal, load_golden, read_pgm

import frontend as F


def _book_bgr():
    return load_golden("book_bgr")["bgr"]


def _book_gray():
    import os
    return read_pgm(os.path.join(GOLDEN, "book_gray.pgm"))


# ---- CPU ---------------------------------------------------------------------
def test_oracle_gray_matches_fixture():
    assert_bits_equal(F.rgb2gray_on_bgr(_book_bgr()), _book_gray(), "gray")
    assert F.read_image_gray(_book_bgr(), False).dtype == np.float32


def test_oracle_resize_properties():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (41, 67, 3), dtype=np.uint8)
    assert_bits_equal(F.resize_linear_u8(img, 41, 67), img, "identity")
    const = np.full((23, 31, 3), 201, np.uint8)
    assert (F.resize_linear_u8(const, 60, 17) == 201).all()
    # within one LSB of a float bilinear with the same pixel-centre mapping
    out = F.resize_linear_u8(img, 97, 29).astype(np.float64)
    ys = np.clip((np.arange(97) + 0.5) * 41 / 97 - 0.5, 0, 40)
    xs = np.clip((np.arange(29) + 0.5) * 67 / 29 - 0.5, 0, 66)
    y0, x0 = np.floor(ys).astype(int), np.floor(xs).astype(int)
    y1, x1 = np.minimum(y0 + 1, 40), np.minimum(x0 + 1, 66)
    fy, fx = (ys - y0)[:, None, None], (xs - x0)[None, :, None]
    f = img.astype(np.float64)
    ref = (f[y0][:, x0] * (1 - fy) * (1 - fx) + f[y0][:, x1] * (1 - fy) * fx +
           f[y1][:, x0] * fy * (1 - fx) + f[y1][:, x1] * fy * fx)
    assert np.abs(out - ref).max() <= 1.01


# ---- GPU ---------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_gray_matches_fixture(ctx):
    g = ctx.bgr8_to_gray(_book_bgr())
    assert_bits_equal(g, _book_gray().astype(np.float32), "gray")


@pytest.mark.gpu
@pytest.mark.parametrize("shape,out", [((300, 210), (960, 960)), ((97, 131), (960, 960)),
                                       ((123, 77), (50, 31)), ((64, 64), (17, 200)), ((5, 3), (2, 9))])
def test_gpu_resize_gray_vs_oracle(ctx, shape, out):
    rng = np.random.default_rng(shape[0] * 7 + out[1])
    bgr = _book_bgr() if shape == (300, 210) else rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    g = ctx.bgr8_to_gray(bgr, *out)
    ref = F.rgb2gray_on_bgr(F.resize_linear_u8(bgr, *out)).astype(np.float32)
    assert_bits_equal(g, ref, f"{shape}->{out}")


@pytest.mark.gpu
def test_gpu_read_image_then_sift(siftgpu):
    """readImage(scene, resized=1) then SIFT_NCL: the GPU gray equals the oracle's
    and feeds the detector (src/main.cpp:19-23)."""
    _, gray = siftgpu.readImage(_book_bgr(), True)
    assert gray.shape == (960, 960)
    assert_bits_equal(gray, F.read_image_gray(_book_bgr(), True), "gray")
    kps, desc = siftgpu.SIFT_NCL(gray)
    assert len(kps) > 100 and desc.shape == (len(kps), 128)


@pytest.mark.gpu
def test_gpu_device_batch(siftgpu, ctx):
    import torch
    rng = np.random.default_rng(5)
    B, H, W, OH, OW = 3, 45, 70, 32, 100
    bgr = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    d_src = torch.from_numpy(bgr).cuda()
    d_out = torch.empty((B, OH, OW + 12), dtype=torch.float32, device="cuda")  # padded rows
    ctx.bgr8_to_gray_device(d_src.data_ptr(), B, H, W, W * 3, H * W * 3, OH, OW, d_out.data_ptr(),
                            (OW + 12) * 4, OH * (OW + 12) * 4)
    ctx.sync()
    out = d_out.cpu().numpy()[:, :, :OW]
    for b in range(B):
        ref = F.rgb2gray_on_bgr(F.resize_linear_u8(bgr[b], OH, OW)).astype(np.float32)
        assert_bits_equal(out[b], ref, f"image {b}")
