"""ctypes binding for the CPU oracle (oracle/sift_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker -- never by the product
library.  PARITY UNPINNED (see sift_oracle.h): the reference cannot be built in
this image and has no golden vectors of its own.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libsift_oracle.so")

KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        L.so_gaussian_kernel.restype = ctypes.c_int
        L.so_gaussian_kernel.argtypes = [ctypes.c_float, fp]
        L.so_gaussian_blur.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_double, fp]
        L.so_gaussian_blur_1d.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_double, fp]
        L.so_resize_nn.argtypes = [fp, ctypes.c_int, ctypes.c_int, fp, ctypes.c_int, ctypes.c_int]
        L.so_build_gaussian_pyramid.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp]
        L.so_fast_pyramid.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp]
        L.so_build_dog_pyramid.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp]
        L.so_pyramid_offsets.restype = ctypes.c_size_t
        L.so_pyramid_offsets.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_size_t)]
        L.so_find_scale_space_extrema.restype = ctypes.c_int
        L.so_find_scale_space_extrema.argtypes = [fp, fp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_void_p, ctypes.c_int]
        L.so_calc_descriptors.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_int, fp, ctypes.c_int]
        L.so_sift.restype = ctypes.c_int
        L.so_sift.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)]
        L.so_free.argtypes = [ctypes.c_void_p]
        L.so_set_threads.argtypes = [ctypes.c_int]
        L.so_synth_image.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, fp]
        L.so_exp32f.argtypes = [fp, fp, ctypes.c_int]
        L.so_fast_atan2.argtypes = [fp, fp, fp, ctypes.c_int]
        L.so_magnitude32f.argtypes = [fp, fp, fp, ctypes.c_int]
        L.so_solve3.restype = ctypes.c_int
        L.so_solve3.argtypes = [fp, fp, fp]
        L.so_helper.argtypes = [ctypes.c_int, fp, fp, fp, ctypes.c_int]
        L.so_cv_round.restype = ctypes.c_int
        L.so_cv_round.argtypes = [ctypes.c_float]
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def octave_shapes(rows: int, cols: int, n_octaves: int = 5):
    out = []
    r, c = rows, cols
    for _ in range(n_octaves):
        out.append((r, c))
        r //= 2
        c //= 2
    return out


def split_planes(packed: np.ndarray, rows: int, cols: int, n_octaves: int, per: int):
    """Packed pyramid -> list of 2-D planes, index o*per + s."""
    planes, off = [], 0
    for (r, c) in octave_shapes(rows, cols, n_octaves):
        for _ in range(per):
            planes.append(packed[off:off + r * c].reshape(r, c))
            off += r * c
    return planes


def set_threads(n: int) -> None:
    lib().so_set_threads(int(n))


def gaussian_kernel(sigma: float) -> np.ndarray:
    w = int(np.floor(np.float32(3) * np.float32(sigma)))
    buf = np.zeros((2 * w + 1) ** 2, np.float32)
    ks = lib().so_gaussian_kernel(float(np.float32(sigma)), _fp(buf))
    return buf[:ks * ks].reshape(ks, ks)


def gaussian_blur(img: np.ndarray, sigma: float) -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    out = np.empty_like(img)
    lib().so_gaussian_blur(_fp(img), img.shape[0], img.shape[1], float(sigma), _fp(out))
    return out


def gaussian_blur_1d(img: np.ndarray, sigma: float) -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    out = np.empty_like(img)
    lib().so_gaussian_blur_1d(_fp(img), img.shape[0], img.shape[1], float(sigma), _fp(out))
    return out


def resize_nn(img: np.ndarray, drows: int, dcols: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    out = np.empty((drows, dcols), np.float32)
    lib().so_resize_nn(_fp(img), img.shape[0], img.shape[1], _fp(out), drows, dcols)
    return out


def _plane_total(rows, cols, n_octaves, per):
    return int(lib().so_pyramid_offsets(rows, cols, n_octaves, per, None))


def build_gaussian_pyramid(img: np.ndarray, n_octaves: int = 5) -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    r, c = img.shape
    out = np.empty(_plane_total(r, c, n_octaves, 5), np.float32)
    lib().so_build_gaussian_pyramid(_fp(img), r, c, n_octaves, _fp(out))
    return out


def fast_pyramid(img: np.ndarray, n_octaves: int = 5) -> np.ndarray:
    """The library's SIFT_FLAG_FAST separable pyramid in its exact operation
    order (agreement mode, not the reference's arithmetic), packed."""
    img = np.ascontiguousarray(img, np.float32)
    r, c = img.shape
    out = np.empty(_plane_total(r, c, n_octaves, 5), np.float32)
    lib().so_fast_pyramid(_fp(img), r, c, n_octaves, _fp(out))
    return out


def build_dog_pyramid(gpyr: np.ndarray, rows: int, cols: int, n_octaves: int = 5) -> np.ndarray:
    out = np.empty(_plane_total(rows, cols, n_octaves, 4), np.float32)
    lib().so_build_dog_pyramid(_fp(gpyr), rows, cols, n_octaves, _fp(out))
    return out


def find_scale_space_extrema(gpyr, dog, rows, cols, n_octaves=5) -> np.ndarray:
    cap = 1 << 14
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        n = lib().so_find_scale_space_extrema(_fp(gpyr), _fp(dog), rows, cols, n_octaves,
                                              kps.ctypes.data, cap)
        if n <= cap:
            return kps[:n].copy()
        cap = n


def calc_descriptors(gpyr, rows, cols, kps: np.ndarray, n_octaves=5, first_octave=0) -> np.ndarray:
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = np.zeros((len(kps), 128), np.float32)
    if len(kps):
        lib().so_calc_descriptors(_fp(gpyr), rows, cols, n_octaves, kps.ctypes.data, len(kps),
                                  _fp(out), first_octave)
    return out


def sift(img: np.ndarray, n_octaves: int = 5):
    """SIFT_NCL restated: returns (keypoints structured array, N x 128 float32)."""
    img = np.ascontiguousarray(img, np.float32)
    kp_p, d_p = ctypes.c_void_p(), ctypes.c_void_p()
    n = lib().so_sift(_fp(img), img.shape[0], img.shape[1], n_octaves,
                      ctypes.byref(kp_p), ctypes.byref(d_p))
    kps = np.zeros(n, KEYPOINT_DTYPE)
    desc = np.zeros((n, 128), np.float32)
    if n:
        ctypes.memmove(kps.ctypes.data, kp_p.value, n * 28)
        ctypes.memmove(desc.ctypes.data, d_p.value, n * 128 * 4)
    lib().so_free(kp_p)
    lib().so_free(d_p)
    return kps, desc


def synth_image(b: int, rows: int, cols: int) -> np.ndarray:
    out = np.empty((rows, cols), np.float32)
    lib().so_synth_image(int(b), rows, cols, _fp(out))
    return out


def exp32f(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    lib().so_exp32f(_fp(x), _fp(y), x.size)
    return y


def fast_atan2(y: np.ndarray, x: np.ndarray) -> np.ndarray:
    y = np.ascontiguousarray(y, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    lib().so_fast_atan2(_fp(y), _fp(x), _fp(o), x.size)
    return o


def magnitude(x: np.ndarray, y: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    o = np.empty_like(x)
    lib().so_magnitude32f(_fp(x), _fp(y), _fp(o), x.size)
    return o


def solve3(a: np.ndarray, b: np.ndarray):
    a = np.ascontiguousarray(a, np.float32).reshape(9)
    b = np.ascontiguousarray(b, np.float32).reshape(3)
    x = np.zeros(3, np.float32)
    ok = lib().so_solve3(_fp(a), _fp(b), _fp(x))
    return x, bool(ok)


def cv_round(v: float) -> int:
    return int(lib().so_cv_round(float(v)))


def helper(op: int, a: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
    """Same op codes as the library's sift_selftest_math."""
    a = np.ascontiguousarray(a, np.float32)
    bb = np.ascontiguousarray(b if b is not None else a, np.float32)
    out = np.empty_like(a)
    lib().so_helper(int(op), _fp(a), _fp(bb), _fp(out), a.size)
    return out
