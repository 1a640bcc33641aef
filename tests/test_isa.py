"""Static ISA guards (CPU; hipcc cross-compiles gfx950 assembly): properties
of the compiled kernels that bit-exactness or speed rests on and that only
large GPU runs would otherwise notice."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tool):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_orientation_steps_stay_ordered():
    """orient_slots_kernel: the 8 read-modify-write steps of each sample batch
    in step order, each step's LDS accesses inside its own exec-masked block
    (src/sift.cpp:429-437 ordering)."""
    out = _run("check_orient_isa.py")
    lines = [l for l in out.splitlines() if "ordered steps" in l]
    # orient_slots_kernel<2> (batches and images above 4 Mpx)
    assert len(lines) == 1 and "orient_slots_kernelILi2E" in lines[0], out
    assert all(l.endswith("0 violations") and not l.split(": ")[1].startswith("0 run") for l in lines), out


def test_orientation_checker_fails_without_the_barrier(tmp_path):
    """The guard itself: orient_slots_kernel compiled with plain `q == jj`
    steps (round 3's form) must be rejected."""
    src = open(os.path.join(ROOT, "sift-gpu_amd", "csrc", "detect.hip")).read()
    a = src.index("void orient_slots_kernel(")
    b = src.index("bool one_image_variants(", a)
    old = ("        int qv = q;\n"
           "        asm volatile(\"; orient step %1\" : \"+v\"(qv) : \"n\"(jj) : \"memory\");\n"
           "        if (qv == jj) {")
    assert old in src[a:b]
    mutated = src[:a] + src[a:b].replace(old, "        if (q == jj) {") + src[b:]
    (tmp_path / "detect.hip").write_text(mutated)
    for h in ("common.hpp", "gauss_host.hpp"):
        (tmp_path / h).write_text(open(os.path.join(ROOT, "sift-gpu_amd", "csrc", h)).read())
    asm = tmp_path / "detect.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                           "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include"),
                           "-I" + os.path.join(ROOT, "sift-gpu_amd", "build"), "--cuda-device-only", "-S",
                           str(tmp_path / "detect.hip"), "-o", str(asm)], stderr=subprocess.DEVNULL, timeout=600)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_orient_isa.py"), str(asm)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 1 and "orient_slots_kernelILi2EEEvNS_7RefArgsE: no \"; orient step\" markers" in r.stdout, \
        r.stdout


def test_fast_pyramid_vmcnt_accounting():
    """pyr_pc_kernel: no spills or scratch (vector-memory ops its hand-counted
    vmcnt waits do not know about), only the producer's expected waits, one
    s_barrier (the LDS counters' initialisation) and the register transposes."""
    out = _run("check_pc_isa.py")
    assert out.count(" 0 violations") == 2, out
