"""bench.py must print its one JSON line even when an optional leg fails
(a late-leg failure cost the driver's only bench record).  CPU
test: the device legs are replaced by canned results, one leg raises."""
import json
import subprocess
import sys
import types

import pytest

import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _stats():
    st = {"blur_octave_sym": {"ms": 40.0, "flops": 4e13, "bytes": 4e9, "launches": 16},
          "blur_octave": {"ms": 2.0, "flops": 2e11, "bytes": 1e8, "launches": 4},
          "descriptor": {"ms": 30.0, "flops": 0, "bytes": 0, "launches": 4}}
    return st


@pytest.fixture()
def bench(monkeypatch):
    import torch
    import bench as B
    monkeypatch.setattr(torch.cuda, "set_device", lambda *a, **k: None)

    class FakeEnv:
        def __init__(self, a, world, rank):
            self.B, self.R, self.C, self.S = a.batch, a.rows, a.cols, 2
            self.rank, self.world = rank, world

        def close(self):
            pass
    monkeypatch.setattr(B, "Env", FakeEnv)
    monkeypatch.setattr(B, "run_exact", lambda env: {"exact": (0.1, {}, 800000.0), "prof": (0.12, _stats(), 0.0),
                                                     "verified": [0, 31, 63], "failed": [], "gather": None})
    monkeypatch.setattr(B, "cpu_baseline", lambda r, c, threads=1, min_seconds=0.0: {"value": 0.6, "unit": "Mpix/s", "cores": threads,
                                                                    "kind": "port", "keypoints_per_s": 4000.0,
                                                                    "sample": "canned"})
    monkeypatch.setattr(B, "cpu_baseline_parallel", lambda r, c, w: None)
    return B


def _run(B, monkeypatch, capsys, argv):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    B.main()
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


def test_line_survives_failing_legs(bench, monkeypatch, capsys):
    def boom(*a, **k):
        raise RuntimeError("leg exploded")
    monkeypatch.setattr(bench, "run_fast", boom)
    monkeypatch.setattr(bench, "run_match", boom)
    monkeypatch.setattr(bench, "single_image_leg", boom)
    monkeypatch.setattr(bench, "eightk_leg", boom)
    monkeypatch.setattr(bench, "c_abi_multi_leg", boom)
    out = _run(bench, monkeypatch, capsys, [])
    assert out["value"] > 0 and out["unit"] == "Mpix/s" and out["n_gpus"] == 1
    assert out["roofline"]["kernel"] == "blur_sym_kernel" and out["roofline"]["frac"] > 0
    assert out["cpu_baseline"]["value"] == 0.6 and "speedup_vs_cpu_1thread" in out
    for block in ("fast_mode", "match", "single_image", "image_8k", "c_abi_multi"):
        assert "leg exploded" in out[block]["error"]
    assert set(out["leg_errors"]) == {"fast", "match", "single", "eightk", "multi"}


def test_line_survives_failing_cpu_leg(bench, monkeypatch, capsys):
    def boom(*a, **k):
        raise TimeoutError("cpu leg hung")
    monkeypatch.setattr(bench, "cpu_baseline_parallel", boom)
    for leg in ("run_fast", "run_match", "single_image_leg", "eightk_leg", "c_abi_multi_leg"):
        monkeypatch.setattr(bench, leg, lambda *a, **k: None)
    out = _run(bench, monkeypatch, capsys, [])
    assert out["value"] > 0 and out["cpu_baseline"]["value"] == 0.6
    assert "cpu_baseline_gpu_share" not in out and "cpu leg hung" in out["leg_errors"]["cpu_baseline_gpu_share"]


def _quiet_legs(B, monkeypatch):
    for leg in ("run_fast", "run_match", "single_image_leg", "eightk_leg", "c_abi_multi_leg"):
        monkeypatch.setattr(B, leg, lambda *a, **k: None)


def test_gpus_n_launches_ranks_as_child(bench, monkeypatch):
    """--gpus N > 1 without WORLD_SIZE: torch.distributed.run as a child
    process with the same arguments; its exit code is ours."""
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, **kw):
        seen["cmd"] = cmd
        return Done()
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(bench, "Env", lambda *a, **k: pytest.fail("the launcher touched the GPU"))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3", "--warmup", "1"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert any(c.startswith("--master-port=") and int(c.split("=")[1]) > 0 for c in cmd)
    i = [k for k, c in enumerate(cmd) if c.endswith("bench.py")][0]
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]


def test_gpus_mismatch_fails(bench, monkeypatch):
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code not in (0, None) and "WORLD_SIZE=2" in str(ex.value.code)


def test_gpus_more_than_devices_fails(bench, monkeypatch):
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(bench.subprocess, "run", lambda *a, **k: pytest.fail("launched with too few devices"))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code not in (0, None) and "only 1" in str(ex.value.code)


def test_shared_gpu_rehearsal_launches_past_the_device_count(bench, monkeypatch):
    """SIFT_BENCH_SHARE_GPU=1: --gpus 2 on a one-device box still launches two
    ranks (the rehearsal of the N > 1 path); without it the same call fails."""
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("SIFT_BENCH_SHARE_GPU", "1")
    monkeypatch.setenv("SIFT_BENCH_DIST_BACKEND", "gloo")
    seen = {}

    def fake_run(cmd, env=None, **k):
        seen["cmd"] = cmd
        return subprocess.CompletedProcess(cmd, 0)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0 and "--nproc-per-node=2" in seen["cmd"]
    assert bench.dist_backend() == "gloo" and bench.check_world(bench.parse()) is None
    monkeypatch.setenv("SIFT_BENCH_SHARE_GPU", "0")
    assert bench.dist_backend() == "nccl"


def test_line_carries_world_and_launcher(bench, monkeypatch, capsys):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    _quiet_legs(bench, monkeypatch)
    out = _run(bench, monkeypatch, capsys, ["--no-cpu-baseline"])
    assert out["distributed"] == {"world_size": 1, "backend": None, "launcher": "none"}
    keys = list(out)
    assert keys.index("output_verified") < keys.index("value") < 4


def test_failed_output_check_fails_the_run(bench, monkeypatch, capsys):
    """the line is printed, then rc != 0."""
    _quiet_legs(bench, monkeypatch)
    monkeypatch.setattr(bench, "run_exact", lambda env: {"exact": (0.1, {}, 800000.0),
                                                         "prof": (0.12, _stats(), 0.0),
                                                         "verified": [0, 63], "failed": [31], "gather": None})
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-cpu-baseline"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 4
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    out = json.loads(lines[0])
    assert out["output_verified"] is False and out["output_failed_seeds"] == [31]


def test_unverified_without_failures_fails_the_run(bench, monkeypatch, capsys):
    _quiet_legs(bench, monkeypatch)
    monkeypatch.setattr(bench, "run_exact", lambda env: {"exact": (0.1, {}, 800000.0),
                                                         "prof": (0.12, _stats(), 0.0),
                                                         "verified": [], "failed": [], "gather": None})
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-cpu-baseline"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 4


def test_gpu_error_flag_by_exception_type(bench, monkeypatch, capsys):
    """exit 3 on a device error only, not on any message holding
    the letters 'hip' (a 'chip' in a CPU leg's message must not count)."""
    import siftgpu
    monkeypatch.setattr(bench, "GPU_ERROR_LEGS", set())
    _quiet_legs(bench, monkeypatch)

    def chip(*a, **k):
        raise RuntimeError("relationship with the chip went wrong")
    monkeypatch.setattr(bench, "single_image_leg", chip)
    out = _run(bench, monkeypatch, capsys, ["--no-cpu-baseline"])
    assert "chip" in out["leg_errors"]["single"]

    def hip(*a, **k):
        raise siftgpu.SiftError("sift_sync", siftgpu.SIFT_E_HIP, "illegal address")
    monkeypatch.setattr(bench, "single_image_leg", hip)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-cpu-baseline"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 3


def test_line_survives_failing_block(bench, monkeypatch, capsys):
    """A leg that returns but whose block cannot be built (missing stage)."""
    monkeypatch.setattr(bench, "run_fast", lambda env: ((0.05, {}, 1.0), None))
    for leg in ("run_match", "single_image_leg", "eightk_leg", "c_abi_multi_leg"):
        monkeypatch.setattr(bench, leg, lambda *a, **k: None)
    out = _run(bench, monkeypatch, capsys, ["--no-cpu-baseline"])
    assert out["value"] > 0 and "error" in out["fast_mode"]


def test_launcher_cpu_legs_reach_rank0_line(bench, monkeypatch, capsys, tmp_path):
    """at N > 1 the launching parent measures the CPU legs
    before any rank exists and rank 0 merges them; the gather is labelled by
    the backend that carried it (a gloo rehearsal never claims RCCL)."""
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    seen = {}
    fake_env = bench.Env

    def fake_run(cmd, env=None, **k):
        seen["path"] = env[bench.CPU_JSON_ENV]
        with open(seen["path"]) as f:
            seen["payload"] = json.load(f)
        return subprocess.CompletedProcess(cmd, 0)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(bench, "Env", lambda *a, **k: pytest.fail("the launcher touched the GPU"))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0
    assert seen["payload"]["cpu"]["cpu_baseline"]["value"] == 0.6
    assert not os.path.exists(seen["path"])   # the parent cleans up after the child

    # rank 0 of the child: reads the parent's file, runs no CPU leg itself
    monkeypatch.setattr(bench, "Env", fake_env)
    cpu_file = tmp_path / "cpu.json"
    bench.save_cpu_legs(seen["payload"]["cpu"], {"cpu_baseline_gpu_share": "canned failure"}, str(cpu_file))
    monkeypatch.setattr(bench, "cpu_baseline", lambda *a, **k: pytest.fail("rank 0 re-ran the CPU leg"))
    _quiet_legs(bench, monkeypatch)
    gather = {"backend": "gloo", "world_size": 2}
    monkeypatch.setattr(bench, "run_exact", lambda env: {"exact": (0.1, {}, 800000.0),
                                                         "prof": (0.12, _stats(), 0.0),
                                                         "verified": [0, 31, 63], "failed": [],
                                                         "gather": gather})
    monkeypatch.setattr(bench.dist, "init_process_group", lambda *a, **k: None)
    monkeypatch.setattr(bench.dist, "destroy_process_group", lambda *a, **k: None)
    monkeypatch.setattr(bench.dist, "get_backend", lambda *a, **k: "gloo")
    for k, v in (("WORLD_SIZE", "2"), ("RANK", "0"), ("LOCAL_RANK", "0"), (bench.CPU_JSON_ENV, str(cpu_file)),
                 ("SIFT_BENCH_SHARE_GPU", "1"), ("SIFT_BENCH_DIST_BACKEND", "gloo")):
        monkeypatch.setenv(k, v)
    out = _run(bench, monkeypatch, capsys, ["--gpus", "2"])
    assert out["n_gpus"] == 2 and out["cpu_baseline"]["value"] == 0.6
    assert out["speedup_vs_cpu_1thread"]["Mpix/s"] > 0
    assert out["leg_errors"]["cpu_baseline_gpu_share"] == "canned failure"
    par = out["config"]["parallelism"]
    assert "gloo" in par and "not RCCL" in par and out["distributed"]["backend"] == "gloo"

    # the same rank under an outside launcher (no parent file): rank 0 measures
    monkeypatch.delenv(bench.CPU_JSON_ENV)
    monkeypatch.setattr(bench, "cpu_baseline", lambda r, c, threads=1, min_seconds=0.0: {
        "value": 0.7, "unit": "Mpix/s", "cores": threads, "kind": "port", "keypoints_per_s": 4100.0,
        "sample": "canned"})
    gather["backend"] = "nccl"
    out = _run(bench, monkeypatch, capsys, ["--gpus", "2"])
    assert out["cpu_baseline"]["value"] == 0.7 and "RCCL" in out["config"]["parallelism"]
