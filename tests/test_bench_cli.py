"""bench.py's argument handling (no GPU): presets, the workload name the
line carries, and the preset-dependent spin-up / timed-step defaults."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _parse(monkeypatch, *args):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", *args])
    return bench.parse()


def test_presets_and_workload_names(monkeypatch):
    import bench
    a = _parse(monkeypatch)
    assert (a.config, a.gaussians, a.width, a.height) == ("C3", 1_000_000, 1920, 1080)
    assert (a.steps, a.spinup_steps) == (30, 50)  # the headline defaults
    assert bench.workload_name(a.gaussians, a.width, a.height) == "C3"
    a = _parse(monkeypatch, "--config", "C1")
    assert (a.gaussians, a.width, a.height, a.steps, a.spinup_steps) == (5_000, 256, 256, 500, 1000)
    assert bench.workload_name(a.gaussians, a.width, a.height) == "C1"
    a = _parse(monkeypatch, "--config", "C2", "--steps", "7", "--spinup-steps", "3", "--gaussians", "1234")
    assert (a.steps, a.spinup_steps, a.gaussians, a.width) == (7, 3, 1234, 800)
    assert bench.workload_name(a.gaussians, a.width, a.height) == "custom"
    for name, (n, w, h) in bench.CONFIGS.items():
        assert bench.workload_name(n, w, h) == name
