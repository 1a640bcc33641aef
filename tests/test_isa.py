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
    assert "run(s) of 8 ordered steps, 0 violations" in out


def test_fast_pyramid_prefetch_untouched():
    """pyr_fast_kernel: the untracked prefetch registers are not touched before
    their explicit vmcnt wait."""
    out = _run("check_prefetch_isa.py")
    assert " 0 violations" in out
