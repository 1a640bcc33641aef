"""bench.py must print its one JSON line even when an optional leg fails
(a late-leg failure cost the driver's only bench record).  CPU
test: the device legs are replaced by canned results, one leg raises."""
import json
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
    monkeypatch.setattr(B, "cpu_baseline", lambda r, c, threads=1: {"value": 0.6, "unit": "Mpix/s", "cores": threads,
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
    out = _run(bench, monkeypatch, capsys, [])
    assert out["value"] > 0 and out["unit"] == "Mpix/s" and out["n_gpus"] == 1
    assert out["roofline"]["kernel"] == "blur_sym_kernel" and out["roofline"]["frac"] > 0
    assert out["cpu_baseline"]["value"] == 0.6 and "speedup_vs_cpu_1thread" in out
    for block in ("fast_mode", "match", "single_image", "image_8k"):
        assert "leg exploded" in out[block]["error"]
    assert set(out["leg_errors"]) == {"fast", "match", "single", "eightk"}


def test_line_survives_failing_cpu_leg(bench, monkeypatch, capsys):
    def boom(*a, **k):
        raise TimeoutError("cpu leg hung")
    monkeypatch.setattr(bench, "cpu_baseline_parallel", boom)
    for leg in ("run_fast", "run_match", "single_image_leg", "eightk_leg"):
        monkeypatch.setattr(bench, leg, lambda *a, **k: None)
    out = _run(bench, monkeypatch, capsys, [])
    assert out["value"] > 0 and out["cpu_baseline"]["value"] == 0.6
    assert "cpu_baseline_gpu_share" not in out and "cpu leg hung" in out["leg_errors"]["cpu_baseline_gpu_share"]


def test_line_survives_failing_block(bench, monkeypatch, capsys):
    """A leg that returns but whose block cannot be built (missing stage)."""
    monkeypatch.setattr(bench, "run_fast", lambda env: ((0.05, {}, 1.0), None))
    for leg in ("run_match", "single_image_leg", "eightk_leg"):
        monkeypatch.setattr(bench, leg, lambda *a, **k: None)
    out = _run(bench, monkeypatch, capsys, ["--no-cpu-baseline"])
    assert out["value"] > 0 and "error" in out["fast_mode"]
