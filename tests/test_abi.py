"""CPU tests of the drop-in boundary: the C-ABI library builds for gfx950,
loads, and exports every symbol include/sift_hip.h declares; the C++ shim
exports the reference's eight sift.hpp functions and compiles reference-style
caller code; host-only layout helpers agree with the oracle.  No GPU compute."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "sift_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sift_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_api():
    syms = declared_symbols()
    for must in ["sift_ctx_create", "sift_detect_compute", "sift_detect_compute_batch",
                 "sift_gaussian_blur", "sift_gaussian_blur_1d", "sift_build_gaussian_pyramid",
                 "sift_build_dog_pyramid", "sift_find_scale_space_extrema", "sift_calc_descriptors",
                 "sift_last_error", "sift_sync"]:
        assert must in syms


def test_library_exports_every_declared_symbol(siftgpu):
    L = ctypes.CDLL(siftgpu.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, f"not exported: {missing}"


def test_library_is_gfx950_code_object(siftgpu):
    data = open(siftgpu.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data      # the offload bundle id


def test_shim_exports_reference_api(siftgpu):
    shim = os.path.join(PKG, "lib", "libsift_shim.so")
    assert os.path.exists(shim)
    syms = subprocess.run(["nm", "-DC", shim], capture_output=True, text=True, check=True).stdout
    for fn in ["SIFT_NCL(", "Gaussian_Blur(", "Gaussian_Blur_1D(", "buildGaussianPyramid(",
               "buildDoGPyramid(", "findScaleSpaceExtrema(", "calDescriptor(", "SITF_BuildIn_OpenCV("]:
        assert re.search(r" T " + re.escape(fn), syms), fn


def test_reference_style_caller_compiles(tmp_path, siftgpu):
    """A caller written against the reference header (src/main.cpp's use of
    SIFT_NCL and the sub-modules) compiles and links unchanged."""
    src = os.path.join(ROOT, "tests", "cpp", "sift_cli.cpp")
    exe = tmp_path / "sift_cli"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), src, "-o", str(exe),
                    "-L", os.path.join(PKG, "lib"), "-lsift_shim", "-lsift_hip",
                    f"-Wl,-rpath,{os.path.join(PKG, 'lib')}"], check=True)
    assert exe.exists()


@pytest.mark.parametrize("openmp", [False, True])
def test_main_shaped_caller_compiles_with_header_only(tmp_path, siftgpu, openmp):
    """A src/main.cpp-shaped caller that includes only sift.hpp and uses
    std::cout, gettimeofday and omp_get_max_threads through it (the reference
    header's transitive includes, include/sift.hpp:11-26) compiles and links
    in compat mode (no OpenCV)."""
    src = os.path.join(ROOT, "tests", "cpp", "main_shape.cpp")
    exe = tmp_path / "main_shape"
    cmd = ["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), src, "-o", str(exe),
           "-L", os.path.join(PKG, "lib"), "-lsift_shim", "-lsift_hip", f"-Wl,-rpath,{os.path.join(PKG, 'lib')}"]
    if openmp:
        cmd.insert(1, "-fopenmp")
    subprocess.run(cmd, check=True)
    assert exe.exists()


def build_multi_gpu_host(out_path):
    """tests/cpp/multi_gpu.cpp: a C++ host driving configs[3] through the C
    ABI's sift_multi_* (g++ + the HIP runtime API, no hipcc)."""
    src = os.path.join(ROOT, "tests", "cpp", "multi_gpu.cpp")
    subprocess.run(["g++", "-O1", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
                    "-I", "/opt/rocm/include", src, "-o", str(out_path), "-L", os.path.join(PKG, "lib"),
                    "-lsift_hip", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{os.path.join(PKG, 'lib')}",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return out_path


def test_multi_gpu_host_compiles(tmp_path, siftgpu):
    assert build_multi_gpu_host(tmp_path / "multi_gpu").exists()


def test_ctx_create_fails_cleanly_without_gpu(siftgpu):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    L = siftgpu.lib()
    h = ctypes.c_void_p()
    rc = L.sift_ctx_create(0, 64, 64, 1, 0, ctypes.byref(h))
    assert rc != 0 and not h.value
    with pytest.raises(siftgpu.SiftError):
        siftgpu.Context(64, 64)


@pytest.mark.parametrize("shape", [(1080, 1920), (300, 210), (203, 157), (4320, 7680)])
def test_layout_helpers_match_oracle(siftgpu, oracle, shape):
    L = siftgpu.lib()
    r, c = shape
    orow = (ctypes.c_int * 5)()
    ocol = (ctypes.c_int * 5)()
    assert L.sift_octave_shapes(r, c, 5, orow, ocol) == 0
    assert list(zip(orow, ocol)) == oracle.octave_shapes(r, c, 5)
    for per in (5, 4):
        assert L.sift_packed_size(r, c, 5, per) == oracle.lib().so_pyramid_offsets(r, c, 5, per, None)


def test_pack_split_roundtrip(siftgpu):
    rng = np.random.default_rng(0)
    planes = [rng.random(s, dtype=np.float32) for (s) in
              [sh for sh in siftgpu.octave_shapes(37, 53, 3) for _ in range(5)]]
    packed = siftgpu.pack_planes(planes, 37, 53, 3, 5)
    back = siftgpu.split_planes(packed, 37, 53, 3, 5)
    assert all(np.array_equal(a, b) for a, b in zip(planes, back))
    with pytest.raises(ValueError):
        siftgpu.pack_planes(planes[:-1], 37, 53, 3, 5)


def test_ctx_create_rejects_planes_over_2g_elements(siftgpu):
    """descriptor.hip gathers with 32-bit element offsets inside a plane:
    an octave-0 plane of 2^31 or more elements is refused up front
    (SIFT_E_SIZE), before any device call."""
    L = siftgpu.lib()
    h = ctypes.c_void_p()
    assert L.sift_ctx_create(0, 46341, 46352, 1, 0, ctypes.byref(h)) == siftgpu.SIFT_E_SIZE and not h.value
    assert L.sift_ctx_create(0, 1 << 16, 1 << 15, 1, 0, ctypes.byref(h)) == siftgpu.SIFT_E_SIZE
