"""Python host binding for libsift_hip.so (MI355X SIFT detect + compute).

Mirrors the reference API (canhld94/SIFT-GPU include/sift.hpp:36-67) with the
same function names and argument meaning, on numpy arrays, by calling the C ABI
declared in include/sift_hip.h through ctypes.  There is no CPU fallback: if
the HIP library cannot be loaded or no GPU is present, every call raises.

    kps, desc = SIFT_NCL(img)                     # src/sift.cpp:59-91
    dst = Gaussian_Blur(src, sigma)               # src/sift.cpp:123-153
    dst = Gaussian_Blur_1D(src, sigma)            # src/sift.cpp:170-217
    gpyr = buildGaussianPyramid(img, nOctaves)    # src/sift.cpp:229-263
    dog = buildDoGPyramid(gpyr, nOctaves)         # src/sift.cpp:265-283
    kps = findScaleSpaceExtrema(gpyr, dog, nOctaves)        # :547-577
    desc = calDescriptor(gpyr, kps, firstOctave)             # :733-753

Pyramids are lists of 2-D float32 planes indexed o*5+s (Gaussian) / o*4+s
(DoG).  Keypoints are numpy structured arrays laid out like cv::KeyPoint.

`Context` exposes the device-resident batch path used by bench.py; buffers are
torch tensors (PyTorch is used only for device memory and streams).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libsift_hip.so")

SIFT_OK, SIFT_E_INVALID, SIFT_E_HIP, SIFT_E_CAPACITY, SIFT_E_SIZE, SIFT_E_NOMEM = 0, -1, -2, -3, -4, -5
SIFT_MULTI_SELF_P2P = 0x100  # sift_multi_create: device 0's own records over RCCL too (tests)
SIFT_E_WORKSPACE = -6  # internal candidate workspace overflow: an error, never the sizing case
SIFT_FLAG_FAST, SIFT_FLAG_PROFILE, SIFT_FLAG_VERBOSE, SIFT_FLAG_NO_GRAPH = 0x1, 0x2, 0x4, 0x8
N_SCALES, N_DOG, DESC_LEN = 5, 4, 128

KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28


class SiftError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


class StageStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int), ("ms", ctypes.c_double),
                ("flops", ctypes.c_double), ("bytes", ctypes.c_double)]


_lib = None
_lib_lock = threading.Lock()


def build() -> str:
    """Compile libsift_hip.so (hipcc, gfx950) in-tree."""
    subprocess.run(["make", "-s", "-C", HERE, "-j8"], check=True)
    return LIB_PATH


def lib():
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built (run make -C {HERE}); no CPU fallback exists")
        L = ctypes.CDLL(LIB_PATH)
        vp, ip, fp, sz = ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_size_t
        pint = ctypes.POINTER(ctypes.c_int)
        sigs = {
            "sift_ctx_create": (ip, [ip, ip, ip, ip, ctypes.c_uint, ctypes.POINTER(vp)]),
            "sift_ctx_destroy": (ip, [vp]),
            "sift_last_error": (ctypes.c_char_p, [vp]),
            "sift_set_stream": (ip, [vp, vp]),
            "sift_get_stream": (vp, [vp]),
            "sift_set_flags": (ip, [vp, ctypes.c_uint]),
            "sift_set_octaves": (ip, [vp, ip]),
            "sift_sync": (ip, [vp]),
            "sift_set_candidate_capacity": (ip, [vp, ip]),
            "sift_version": (ctypes.c_char_p, []),
            "sift_graph_stats": (ip, [vp, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.POINTER(ctypes.c_longlong)]),
            "sift_octave_shapes": (ip, [ip, ip, ip, pint, pint]),
            "sift_packed_size": (sz, [ip, ip, ip, ip]),
            "sift_detect_compute": (ip, [vp, fp, ip, ip, sz, vp, fp, ip, pint]),
            "sift_detect_compute_batch": (ip, [vp, vp, ip, ip, ip, sz, sz, vp, vp, ip, vp]),
            "sift_copy_results": (ip, [vp, vp, fp, ip, pint]),
            "sift_synth_images": (ip, [vp, vp, ip, ip, ip, sz, sz, ip]),
            "sift_gaussian_blur": (ip, [vp, fp, ip, ip, ctypes.c_double, fp]),
            "sift_gaussian_blur_1d": (ip, [vp, fp, ip, ip, ctypes.c_double, fp]),
            "sift_build_gaussian_pyramid": (ip, [vp, fp, ip, ip, ip, fp]),
            "sift_build_dog_pyramid": (ip, [vp, fp, ip, ip, ip, fp]),
            "sift_find_scale_space_extrema": (ip, [vp, fp, fp, ip, ip, ip, vp, ip, pint]),
            "sift_calc_descriptors": (ip, [vp, fp, ip, ip, ip, vp, ip, fp, ip]),
            "sift_get_stage_stats": (ip, [vp, ctypes.POINTER(StageStat), ip, pint, ip]),
            "sift_selftest_math": (ip, [vp, ip, fp, fp, fp, ip]),
            "sift_knn_match_l1": (ip, [vp, fp, ip, fp, ip, ip, pint, fp]),
            "sift_bgr8_to_gray": (ip, [vp, vp, ip, ip, sz, ip, ip, fp]),
            "sift_find_homography": (ip, [fp, fp, ip, ctypes.c_double, ip, ctypes.c_double,
                                          ctypes.POINTER(ctypes.c_double), vp]),
            "sift_perspective_transform": (ip, [ctypes.POINTER(ctypes.c_double), fp, ip, fp]),
            "sift_bgr8_to_gray_device": (ip, [vp, vp, ip, ip, ip, sz, sz, ip, ip, vp, sz, sz]),
            "sift_knn_match_l1_device": (ip, [vp, vp, ip, vp, ip, ip, vp, vp]),
            "sift_multi_shard": (ip, [ip, ip, ip, pint, pint]),
            "sift_multi_merge_offsets": (ip, [ctypes.POINTER(pint), pint, ip, pint]),
            "sift_multi_create": (ip, [pint, ip, ip, ip, ip, ctypes.c_uint, ip, ip, ip, ctypes.POINTER(vp)]),
            "sift_multi_set_octaves": (ip, [vp, ip]),
            "sift_multi_set_flags": (ip, [vp, ctypes.c_uint]),
            "sift_multi_destroy": (ip, [vp]),
            "sift_multi_last_error": (ctypes.c_char_p, [vp]),
            "sift_multi_context": (vp, [vp, ip]),
            "sift_multi_step": (ip, [vp, ctypes.POINTER(vp), pint, ip, ip, sz, sz]),
            "sift_multi_flush": (ip, [vp]),
            "sift_multi_gathered": (ip, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), pint, ip, pint,
                                         ctypes.POINTER(ctypes.c_longlong)]),
            "sift_multi_stats": (ip, [vp, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.POINTER(ctypes.c_longlong)]),
            "sift_multi_rccl_version": (ip, []),
            "sift_multi_copy_gathered": (ip, [vp, vp, fp, ip, pint]),
        }
        optional = {"sift_graph_stats"}  # absent from older builds (A/B runs against a saved library)
        for name, (res, args) in sigs.items():
            if name in optional and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return L


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def octave_shapes(rows: int, cols: int, n_octaves: int = 5):
    out, r, c = [], rows, cols
    for _ in range(n_octaves):
        out.append((r, c))
        r //= 2
        c //= 2
    return out


def pack_planes(planes, rows, cols, n_octaves, per) -> np.ndarray:
    shapes = octave_shapes(rows, cols, n_octaves)
    if len(planes) < n_octaves * per:
        raise ValueError("too few planes")
    parts = []
    for o, (r, c) in enumerate(shapes):
        for s in range(per):
            p = np.ascontiguousarray(planes[o * per + s], np.float32)
            if p.shape != (r, c):
                raise ValueError(f"plane {o * per + s} has shape {p.shape}, octave shape is {(r, c)}")
            parts.append(p.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


def split_planes(packed: np.ndarray, rows, cols, n_octaves, per):
    planes, off = [], 0
    for (r, c) in octave_shapes(rows, cols, n_octaves):
        for _ in range(per):
            planes.append(packed[off:off + r * c].reshape(r, c))
            off += r * c
    return planes


class Context:
    """A device context (one HIP stream, workspace for max_rows x max_cols x max_batch)."""

    def __init__(self, max_rows: int, max_cols: int, max_batch: int = 1, device: int = 0,
                 flags: int = 0):
        self._L = lib()
        h = ctypes.c_void_p()
        rc = self._L.sift_ctx_create(device, max_rows, max_cols, max_batch, flags, ctypes.byref(h))
        if rc != SIFT_OK:
            raise SiftError("sift_ctx_create", rc, "could not create a device context (no GPU?)")
        self.h = h
        self.max_rows, self.max_cols, self.max_batch, self.device = max_rows, max_cols, max_batch, device

    def close(self):
        if getattr(self, "h", None):
            self._L.sift_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, fn, rc):
        if rc != SIFT_OK:
            raise SiftError(fn, rc, self._L.sift_last_error(self.h).decode())

    # ---- configuration --------------------------------------------------
    def set_flags(self, flags):
        self._check("sift_set_flags", self._L.sift_set_flags(self.h, flags))

    def set_octaves(self, n):
        self._check("sift_set_octaves", self._L.sift_set_octaves(self.h, n))

    def set_stream(self, stream_handle: int):
        self._check("sift_set_stream", self._L.sift_set_stream(self.h, ctypes.c_void_p(stream_handle)))

    def sync(self):
        self._check("sift_sync", self._L.sift_sync(self.h))

    def graph_stats(self):
        """(captures, in-place updates, instantiations) of the context's hipGraph cache."""
        v = [ctypes.c_longlong(0) for _ in range(3)]
        self._check("sift_graph_stats", self._L.sift_graph_stats(self.h, *[ctypes.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def set_candidate_capacity(self, per_image: int):
        self._check("sift_set_candidate_capacity", self._L.sift_set_candidate_capacity(self.h, per_image))

    # ---- host-memory API (reference names) ------------------------------
    def SIFT_NCL(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.float32)
        r, c = img.shape
        n = ctypes.c_int(0)
        rc = self._L.sift_detect_compute(self.h, _fp(img), r, c, c * 4, None, None, 0, ctypes.byref(n))
        if rc not in (SIFT_OK, SIFT_E_CAPACITY):
            self._check("sift_detect_compute", rc)
        kps = np.zeros(n.value, KEYPOINT_DTYPE)
        desc = np.zeros((n.value, DESC_LEN), np.float32)
        if n.value:
            rc = self._L.sift_copy_results(self.h, kps.ctypes.data, _fp(desc), n.value, ctypes.byref(n))
            self._check("sift_copy_results", rc)
        return kps, desc

    def Gaussian_Blur(self, src: np.ndarray, sigma: float) -> np.ndarray:
        src = np.ascontiguousarray(src, np.float32)
        dst = np.empty_like(src)
        self._check("sift_gaussian_blur",
                    self._L.sift_gaussian_blur(self.h, _fp(src), src.shape[0], src.shape[1], float(sigma), _fp(dst)))
        return dst

    def Gaussian_Blur_1D(self, src: np.ndarray, sigma: float) -> np.ndarray:
        src = np.ascontiguousarray(src, np.float32)
        dst = np.empty_like(src)
        self._check("sift_gaussian_blur_1d",
                    self._L.sift_gaussian_blur_1d(self.h, _fp(src), src.shape[0], src.shape[1], float(sigma), _fp(dst)))
        return dst

    def buildGaussianPyramid(self, image: np.ndarray, nOctaves: int = 5):
        image = np.ascontiguousarray(image, np.float32)
        r, c = image.shape
        out = np.empty(self._L.sift_packed_size(r, c, nOctaves, N_SCALES), np.float32)
        self._check("sift_build_gaussian_pyramid",
                    self._L.sift_build_gaussian_pyramid(self.h, _fp(image), r, c, nOctaves, _fp(out)))
        return split_planes(out, r, c, nOctaves, N_SCALES)

    def buildDoGPyramid(self, gpyr, nOctaves: int = 5):
        r, c = gpyr[0].shape
        g = pack_planes(gpyr, r, c, nOctaves, N_SCALES)
        out = np.empty(self._L.sift_packed_size(r, c, nOctaves, N_DOG), np.float32)
        self._check("sift_build_dog_pyramid",
                    self._L.sift_build_dog_pyramid(self.h, _fp(g), r, c, nOctaves, _fp(out)))
        return split_planes(out, r, c, nOctaves, N_DOG)

    def findScaleSpaceExtrema(self, gpyr, dogpyr, nOctaves: int = 5) -> np.ndarray:
        r, c = gpyr[0].shape
        g = pack_planes(gpyr, r, c, nOctaves, N_SCALES)
        d = pack_planes(dogpyr, r, c, nOctaves, N_DOG)
        n = ctypes.c_int(0)
        rc = self._L.sift_find_scale_space_extrema(self.h, _fp(g), _fp(d), r, c, nOctaves, None, 0, ctypes.byref(n))
        if rc not in (SIFT_OK, SIFT_E_CAPACITY):
            self._check("sift_find_scale_space_extrema", rc)
        kps = np.zeros(n.value, KEYPOINT_DTYPE)
        if n.value:
            rc = self._L.sift_copy_results(self.h, kps.ctypes.data, None, n.value, ctypes.byref(n))
            self._check("sift_copy_results", rc)
        return kps

    def calDescriptor(self, gpyr, keypoints: np.ndarray, firstOctave: int = 0) -> np.ndarray:
        r, c = gpyr[0].shape
        n_oct = len(gpyr) // N_SCALES
        g = pack_planes(gpyr, r, c, n_oct, N_SCALES)
        kps = np.ascontiguousarray(keypoints, KEYPOINT_DTYPE)
        desc = np.zeros((len(kps), DESC_LEN), np.float32)
        self._check("sift_calc_descriptors",
                    self._L.sift_calc_descriptors(self.h, _fp(g), r, c, n_oct, kps.ctypes.data, len(kps),
                                                  _fp(desc), firstOctave))
        return desc

    def bgr8_to_gray(self, bgr: np.ndarray, out_rows: int | None = None, out_cols: int | None = None):
        """readImage's conversion (src/main.cpp:83-85) of decoded BGR bytes:
        optional INTER_LINEAR resize, COLOR_RGB2GRAY on BGR, CV_32F."""
        bgr = np.ascontiguousarray(bgr, np.uint8)
        if bgr.ndim != 3 or bgr.shape[2] != 3:
            raise ValueError("expected an H x W x 3 uint8 BGR image")
        r, c = bgr.shape[:2]
        orows, ocols = out_rows or r, out_cols or c
        gray = np.empty((orows, ocols), np.float32)
        self._check("sift_bgr8_to_gray",
                    self._L.sift_bgr8_to_gray(self.h, bgr.ctypes.data, r, c, c * 3, orows, ocols, _fp(gray)))
        return gray

    def bgr8_to_gray_device(self, src_ptr: int, batch: int, rows: int, cols: int, row_stride: int,
                            img_stride: int, out_rows: int, out_cols: int, dst_ptr: int, out_row_stride: int,
                            out_img_stride: int):
        self._check("sift_bgr8_to_gray_device",
                    self._L.sift_bgr8_to_gray_device(self.h, ctypes.c_void_p(src_ptr), batch, rows, cols,
                                                     row_stride, img_stride, out_rows, out_cols,
                                                     ctypes.c_void_p(dst_ptr), out_row_stride, out_img_stride))

    def knnMatch(self, query: np.ndarray, train: np.ndarray, k: int = 2):
        """BFMatcher(NORM_L1).knnMatch as arrays (src/main.cpp:25-27): idx, dist
        [n_query, k]; idx -1 / dist +inf where there are fewer than k train rows."""
        q = np.ascontiguousarray(query, np.float32).reshape(-1, DESC_LEN)
        t = np.ascontiguousarray(train, np.float32).reshape(-1, DESC_LEN)
        idx = np.empty((len(q), k), np.int32)
        dist = np.empty((len(q), k), np.float32)
        self._check("sift_knn_match_l1",
                    self._L.sift_knn_match_l1(self.h, _fp(q), len(q), _fp(t), len(t), k,
                                              idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _fp(dist)))
        return idx, dist

    def knn_match_device(self, query_ptr: int, n_query: int, train_ptr: int, n_train: int, k: int,
                         idx_ptr: int, dist_ptr: int):
        """Device-pointer form, enqueued on the context stream (no sync)."""
        self._check("sift_knn_match_l1_device",
                    self._L.sift_knn_match_l1_device(self.h, ctypes.c_void_p(query_ptr), n_query,
                                                     ctypes.c_void_p(train_ptr), n_train, k,
                                                     ctypes.c_void_p(idx_ptr), ctypes.c_void_p(dist_ptr)))

    # ---- device batch API ------------------------------------------------
    def synth_images(self, out_ptr: int, batch: int, rows: int, cols: int, row_stride: int,
                     img_stride: int, seed_base: int = 0):
        self._check("sift_synth_images",
                    self._L.sift_synth_images(self.h, ctypes.c_void_p(out_ptr), batch, rows, cols,
                                              row_stride, img_stride, seed_base))

    def detect_compute_batch(self, imgs_ptr: int, batch: int, rows: int, cols: int, row_stride: int,
                             img_stride: int, kpts_ptr: int, desc_ptr: int, kp_cap: int, offs_ptr: int):
        self._check("sift_detect_compute_batch",
                    self._L.sift_detect_compute_batch(self.h, ctypes.c_void_p(imgs_ptr), batch, rows, cols,
                                                      row_stride, img_stride, ctypes.c_void_p(kpts_ptr),
                                                      ctypes.c_void_p(desc_ptr), kp_cap,
                                                      ctypes.c_void_p(offs_ptr)))

    def selftest_math(self, op: int, a: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
        a = np.ascontiguousarray(a, np.float32)
        bb = np.ascontiguousarray(b if b is not None else a, np.float32)
        out = np.empty_like(a)
        self._check("sift_selftest_math",
                    self._L.sift_selftest_math(self.h, op, _fp(a), _fp(bb), _fp(out), a.size))
        return out

    def stage_stats(self, reset: bool = True):
        buf = (StageStat * 32)()
        n = ctypes.c_int(0)
        self._check("sift_get_stage_stats",
                    self._L.sift_get_stage_stats(self.h, buf, 32, ctypes.byref(n), int(reset)))
        return {buf[i].name.decode(): dict(launches=buf[i].launches, ms=buf[i].ms, flops=buf[i].flops,
                                           bytes=buf[i].bytes) for i in range(n.value)}


def multi_shard(batch: int, n_devices: int, index: int) -> tuple[int, int]:
    """(first, count) of device `index`'s contiguous shard (sift_multi_shard)."""
    f, c = ctypes.c_int(0), ctypes.c_int(0)
    rc = lib().sift_multi_shard(batch, n_devices, index, ctypes.byref(f), ctypes.byref(c))
    if rc != SIFT_OK:
        raise SiftError("sift_multi_shard", rc, "bad arguments")
    return f.value, c.value


def multi_merge_offsets(shard_offsets) -> np.ndarray:
    """Global per-image offsets from each shard's own (sift_multi_merge_offsets)."""
    arrs = [np.ascontiguousarray(o, np.int32) for o in shard_offsets]
    pint = ctypes.POINTER(ctypes.c_int)
    ptrs = (pint * len(arrs))(*[a.ctypes.data_as(pint) for a in arrs])
    counts = np.array([len(a) - 1 for a in arrs], np.int32)
    out = np.zeros(int(counts.sum()) + 1, np.int32)
    rc = lib().sift_multi_merge_offsets(ptrs, counts.ctypes.data_as(pint), len(arrs), out.ctypes.data_as(pint))
    if rc != SIFT_OK:
        raise SiftError("sift_multi_merge_offsets", rc, "bad arguments")
    return out


class MultiContext:
    """Multi-GPU batch mode (sift_multi_*): one context + stream per device,
    contiguous image shards, the keypoint records (and optionally the
    descriptors) gathered to devices[0] over RCCL one step behind."""

    def __init__(self, devices, max_rows: int, max_cols: int, max_batch_per_device: int, kp_cap_per_device: int,
                 flags: int = 0, gather_desc: bool = False, streams_per_device: int = 0):
        self._L = lib()
        self.devices = list(devices)
        dv = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        rc = self._L.sift_multi_create(dv, len(self.devices), max_rows, max_cols, max_batch_per_device, flags,
                                       streams_per_device, kp_cap_per_device, int(gather_desc), ctypes.byref(h))
        if rc != SIFT_OK:
            raise SiftError("sift_multi_create", rc, "could not create the multi-GPU context (see stderr)")
        self.h = h
        self.gather_desc = gather_desc

    def close(self):
        if getattr(self, "h", None):
            self._L.sift_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, fn, rc):
        if rc != SIFT_OK:
            raise SiftError(fn, rc, self._L.sift_multi_last_error(self.h).decode())

    def context_handle(self, index: int):
        return self._L.sift_multi_context(self.h, index)

    def set_octaves(self, n: int):
        self._check("sift_multi_set_octaves", self._L.sift_multi_set_octaves(self.h, n))

    def set_flags(self, flags: int):
        self._check("sift_multi_set_flags", self._L.sift_multi_set_flags(self.h, flags))

    def synth_images(self, index: int, out_ptr: int, batch: int, rows: int, cols: int, row_stride: int,
                     img_stride: int, seed_base: int = 0):
        rc = self._L.sift_synth_images(ctypes.c_void_p(self.context_handle(index)), ctypes.c_void_p(out_ptr), batch,
                                       rows, cols, row_stride, img_stride, seed_base)
        self._check("sift_synth_images", rc)

    def step(self, img_ptrs, counts, rows: int, cols: int, row_stride: int, img_stride: int):
        n = len(self.devices)
        ptrs = (ctypes.c_void_p * n)(*[ctypes.c_void_p(p) for p in img_ptrs])
        cnt = (ctypes.c_int * n)(*counts)
        self._check("sift_multi_step", self._L.sift_multi_step(self.h, ptrs, cnt, rows, cols, row_stride, img_stride))

    def flush(self):
        self._check("sift_multi_flush", self._L.sift_multi_flush(self.h))

    def gathered(self, offsets_cap: int):
        """(device pointer to the records, to the descriptors or None, global
        offsets as numpy, step index) of the last gathered step."""
        k, d = ctypes.c_void_p(), ctypes.c_void_p()
        offs = np.zeros(offsets_cap, np.int32)
        bt, st = ctypes.c_int(0), ctypes.c_longlong(0)
        self._check("sift_multi_gathered",
                    self._L.sift_multi_gathered(self.h, ctypes.byref(k), ctypes.byref(d),
                                                offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), offsets_cap,
                                                ctypes.byref(bt), ctypes.byref(st)))
        return k.value, d.value, offs[:bt.value + 1].copy(), st.value

    def copy_gathered(self):
        """Host copies (keypoints, descriptors or None) of the last gathered step."""
        n = ctypes.c_int(0)
        rc = self._L.sift_multi_copy_gathered(self.h, None, None, 0, ctypes.byref(n))
        if rc not in (SIFT_OK, SIFT_E_CAPACITY):
            self._check("sift_multi_copy_gathered", rc)
        kps = np.zeros(n.value, KEYPOINT_DTYPE)
        desc = np.zeros((n.value, DESC_LEN), np.float32) if self.gather_desc else None
        if n.value:
            self._check("sift_multi_copy_gathered",
                        self._L.sift_multi_copy_gathered(self.h, kps.ctypes.data,
                                                         _fp(desc) if desc is not None else None, n.value,
                                                         ctypes.byref(n)))
        return kps, desc

    def stats(self):
        v = [ctypes.c_longlong(0) for _ in range(3)]
        self._check("sift_multi_stats", self._L.sift_multi_stats(self.h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("steps", "records", "transfers"), (x.value for x in v)))


def rccl_version() -> int:
    return lib().sift_multi_rccl_version()


# ---- module-level API with the reference's names (one shared context) -------
_default = None


def _ctx(rows, cols):
    global _default
    if _default is None or rows > _default.max_rows or cols > _default.max_cols:
        mr = max(rows, _default.max_rows if _default else 0)
        mc = max(cols, _default.max_cols if _default else 0)
        if _default is not None:
            _default.close()
        _default = Context(mr, mc, 1, int(os.environ.get("SIFT_HIP_DEVICE", "0")))
    return _default


def SIFT_NCL(image):
    return _ctx(*image.shape).SIFT_NCL(image)


def Gaussian_Blur(src, sigma):
    return _ctx(*src.shape).Gaussian_Blur(src, sigma)


def Gaussian_Blur_1D(src, sigma):
    return _ctx(*src.shape).Gaussian_Blur_1D(src, sigma)


def buildGaussianPyramid(image, nOctaves=5):
    return _ctx(*image.shape).buildGaussianPyramid(image, nOctaves)


def buildDoGPyramid(gpyr, nOctaves=5):
    return _ctx(*gpyr[0].shape).buildDoGPyramid(gpyr, nOctaves)


def findScaleSpaceExtrema(gpyr, dogpyr, nOctaves=5):
    return _ctx(*gpyr[0].shape).findScaleSpaceExtrema(gpyr, dogpyr, nOctaves)


def calDescriptor(gpyr, keypoints, firstOctave=0):
    return _ctx(*gpyr[0].shape).calDescriptor(gpyr, keypoints, firstOctave)


# ---- image front end -------------------------------------
def imread(filename) -> np.ndarray:
    """cv::imread(filename) layout: H x W x 3 uint8 BGR (decoded with PIL)."""
    from PIL import Image
    rgb = np.asarray(Image.open(filename).convert("RGB"), np.uint8)
    return np.ascontiguousarray(rgb[..., ::-1])


def readImage(filename_or_bgr, resized: bool):
    """src/main.cpp:79-87 -> (img, gray): gray is the CV_32F plane SIFT_NCL
    takes (960 x 960 when resized), produced on the GPU (frontend.hip); img is
    the decoded BGR image (the reference keeps the resized copy, which only its
    drawMatches uses -- not produced here)."""
    bgr = imread(filename_or_bgr) if isinstance(filename_or_bgr, (str, os.PathLike)) else \
        np.ascontiguousarray(filename_or_bgr, np.uint8)
    rows, cols = (960, 960) if resized else bgr.shape[:2]
    gray = _ctx(rows, cols).bgr8_to_gray(bgr, rows, cols)
    return bgr, gray


# ---- matcher: the reference application's consumer ------
class DMatch:
    """cv::DMatch fields (queryIdx, trainIdx, imgIdx, distance)."""
    __slots__ = ("queryIdx", "trainIdx", "imgIdx", "distance")

    def __init__(self, queryIdx, trainIdx, imgIdx, distance):
        self.queryIdx, self.trainIdx, self.imgIdx, self.distance = queryIdx, trainIdx, imgIdx, distance

    def __repr__(self):
        return f"DMatch({self.queryIdx}, {self.trainIdx}, {self.imgIdx}, {self.distance!r})"


NORM_L1 = 2  # cv::NORM_L1


class BFMatcher:
    """`cv::BFMatcher(NORM_L1)` as the reference uses it (src/main.cpp:25-27):
    knnMatch(queryDescriptors, trainDescriptors, k) -> per query a list of up to
    k DMatch, nearest first.  Only NORM_L1 float descriptors, k in (1, 2), no
    masks / crossCheck (the reference uses none)."""

    def __init__(self, normType: int = NORM_L1, crossCheck: bool = False, ctx: Context | None = None):
        if normType != NORM_L1 or crossCheck:
            raise ValueError("only BFMatcher(NORM_L1) without crossCheck is implemented")
        self._ctx = ctx

    def knnMatch(self, queryDescriptors, trainDescriptors, k: int = 2):
        ctx = self._ctx or _ctx(1, 1)
        idx, dist = ctx.knnMatch(queryDescriptors, trainDescriptors, k)
        return [[DMatch(i, int(idx[i, j]), 0, float(dist[i, j])) for j in range(k) if idx[i, j] >= 0]
                for i in range(len(idx))]


def ratio_test(matches, ratio: float = 0.86):
    """src/main.cpp:28-40: keep m1 where m1.distance <= ratio * m2.distance
    (a query with fewer than two matches is skipped)."""
    return [m[0] for m in matches if len(m) >= 2 and m[0].distance <= ratio * m[1].distance]


# ---- homography: src/main.cpp:44-62 ------------------------
RANSAC = 8  # cv::RANSAC


def findHomography(srcPoints, dstPoints, method: int = RANSAC, ransacReprojThreshold: float = 3.0,
                   mask=None, maxIters: int = 2000, confidence: float = 0.995):
    """cv::findHomography(obj, scene, RANSAC) -> (H 3x3 float64 or None, inlier mask).
    Host code in the library (homography.hip); None where OpenCV returns an empty Mat."""
    if method != RANSAC:
        raise ValueError("only RANSAC is implemented (the reference uses RANSAC)")
    src = np.ascontiguousarray(srcPoints, np.float32).reshape(-1, 2)
    dst = np.ascontiguousarray(dstPoints, np.float32).reshape(-1, 2)
    if len(src) != len(dst):
        raise ValueError("point counts differ")
    H = np.zeros(9, np.float64)
    m = np.zeros(max(len(src), 1), np.uint8)
    rc = lib().sift_find_homography(_fp(src), _fp(dst), len(src), float(ransacReprojThreshold), int(maxIters),
                                    float(confidence), H.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                    m.ctypes.data)
    if rc != SIFT_OK:
        return None, np.zeros(len(src), np.uint8)
    return H.reshape(3, 3), m[:len(src)]


def perspectiveTransform(points, H):
    """cv::perspectiveTransform for Point2f with a 3x3 double H."""
    pts = np.ascontiguousarray(points, np.float32).reshape(-1, 2)
    Hd = np.ascontiguousarray(H, np.float64).reshape(9)
    out = np.empty_like(pts)
    rc = lib().sift_perspective_transform(Hd.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), _fp(pts), len(pts),
                                          _fp(out))
    if rc != SIFT_OK:
        raise SiftError("sift_perspective_transform", rc, "bad argument")
    return out
