"""Shared fixtures.  `-m "not gpu"` runs the oracle, host-logic, ABI-export and
distributed (gloo) tests on CPU; `-m gpu` runs the HIP parity tests through the
C ABI on an MI355X."""
import hashlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sift-gpu_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (HIP) -- parity tests")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def siftgpu():
    # torch first: its bundled HIP runtime (soname libamdhip64.so.7) is then the
    # one process-wide runtime that libsift_hip.so binds to as well.
    import torch  # noqa: F401
    import siftgpu as S
    S.build()
    return S


@pytest.fixture(scope="session")
def ctx(siftgpu):
    """One device context big enough for every parity case (1080p, batch 4)."""
    c = siftgpu.Context(1080, 1920, 4, device=0)
    yield c
    c.close()


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def read_pgm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    assert parts[0] == b"P5"
    w, h = int(parts[1]), int(parts[2])
    return np.frombuffer(parts[4][:w * h], np.uint8).reshape(h, w)


def book_image():
    return read_pgm(os.path.join(GOLDEN, "book_gray.pgm")).astype(np.float32)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def kp_bytes(kps) -> np.ndarray:
    return np.ascontiguousarray(kps).view(np.uint8).reshape(len(kps), 28)


def assert_bits_equal(a, b, what=""):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    assert a.shape == b.shape, f"{what}: shape {a.shape} != {b.shape}"
    if a.tobytes() != b.tobytes():
        av = a.view(np.uint8).reshape(-1)
        bv = b.view(np.uint8).reshape(-1)
        nbad = int(np.count_nonzero(av != bv))
        if a.dtype == np.float32:
            diff = np.abs(a.astype(np.float64) - b.astype(np.float64))
            idx = np.unravel_index(int(np.argmax(diff)), a.shape)
            raise AssertionError(f"{what}: {nbad} bytes differ; max |diff| {diff.max():.3g} at {idx}")
        raise AssertionError(f"{what}: {nbad} bytes differ")
