"""CPU restatement of the reference application's image front end (SURVEY.md
§8(f) f1): readImage, src/main.cpp:79-87.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker -- never by the
product library (sift-gpu_amd/csrc/frontend.hip).

    img = imread(filename);                       // 8-bit BGR
    if (resized) resize(img, img, Size(960,960)); // INTER_LINEAR, 8UC3
    cvtColor(img, gray, cv::COLOR_RGB2GRAY);      // on BGR bytes
    gray.convertTo(gray, DATATYPE);               // CV_32F

OpenCV is not in this image.  The gray conversion is OpenCV's fixed-point
RGB2Gray<uchar> (R2Y 4899, G2Y 9617, B2Y 1868, 14-bit shift, round half up)
with the R weight on channel 0 -- the B byte of imread's BGR -- and is pinned by
the committed fixture tests/golden/book_gray.pgm.  The resize restates
resizeGeneric_ for INTER_LINEAR 8-bit as built on x86 (SSE2 universal
intrinsics, no IPP): coefficient setup in float/double as in OpenCV,
HResizeLinear in exact ints, VResizeLinearVec_32s8u's 16-bit mul_hi form for
the elements its 16-/8-lane loops cover and FixedPtCast for the row tail.
Resize parity against OpenCV itself is UNPINNED (IPP or another SIMD width
would round differently).
"""
from __future__ import annotations

import numpy as np

COEF_SCALE = 2048  # INTER_RESIZE_COEF_SCALE


def _round_half_even(x: np.ndarray) -> np.ndarray:
    return np.rint(x).astype(np.int64)  # cvRound(float): round to nearest even


def _taps(n_out: int, n_in: int, clamp: bool):
    scale = float(n_in) / n_out
    d = np.arange(n_out, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)                     # cvFloor
    f = (f - s.astype(np.float32)).astype(np.float32)
    if clamp:
        lo = s < 0
        f[lo], s[lo] = 0, 0
        hi = s >= n_in - 1
        f[hi], s[hi] = 0, n_in - 1
    a0 = _round_half_even((np.float32(1) - f).astype(np.float32) * np.float32(COEF_SCALE))
    a1 = _round_half_even(f * np.float32(COEF_SCALE))
    return s, a0, a1


def resize_linear_u8(img: np.ndarray, out_rows: int, out_cols: int) -> np.ndarray:
    """cv::resize(img, dst, Size(out_cols, out_rows)), INTER_LINEAR, 8UC3."""
    src = np.asarray(img, np.uint8)
    h, w, cn = src.shape
    if (h, w) == (out_rows, out_cols):
        return src.copy()
    sx, ax0, ax1 = _taps(out_cols, w, clamp=True)
    sy, by0, by1 = _taps(out_rows, h, clamp=False)
    sx1 = np.minimum(sx + 1, w - 1)
    s = src.astype(np.int64)
    # horizontal pass, exact ints: [h, out_cols, cn]
    hr = s[:, sx, :] * ax0[None, :, None] + s[:, sx1, :] * ax1[None, :, None]
    r0 = np.clip(sy, 0, h - 1)
    r1 = np.clip(sy + 1, 0, h - 1)
    h0 = hr[r0]
    h1 = hr[r1]
    b0 = by0[:, None, None]
    b1 = by1[:, None, None]
    simd = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16)
    simd = (simd + 2) >> 2
    scal = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22
    n = out_cols * cn
    vtail = n // 16 * 16
    while vtail < n - 8:
        vtail += 8
    elem = (np.arange(out_cols)[:, None] * cn + np.arange(cn)[None, :])[None]
    v = np.where(elem < vtail, simd, scal)
    return np.clip(v, 0, 255).astype(np.uint8)


def rgb2gray_on_bgr(img: np.ndarray) -> np.ndarray:
    """cvtColor(COLOR_RGB2GRAY) applied to imread's BGR bytes (uint8 result)."""
    s = np.asarray(img, np.int64)
    return ((4899 * s[..., 0] + 9617 * s[..., 1] + 1868 * s[..., 2] + 8192) >> 14).astype(np.uint8)


def read_image_gray(bgr: np.ndarray, resized: bool) -> np.ndarray:
    """readImage's gray output (CV_32F) from decoded BGR bytes."""
    img = resize_linear_u8(bgr, 960, 960) if resized else np.asarray(bgr, np.uint8)
    return rgb2gray_on_bgr(img).astype(np.float32)
