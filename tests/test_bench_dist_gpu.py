"""The N > 1 bench line's all-reduce numbers: bench.py run as
the driver runs it, at C1 with a few steps -- world size 1 through the
native RCCL communicator (--force-dist: the collective path of an 8-GPU run,
one rank), and two gloo ranks sharing the box's one GPU (the collectives go
through torch.distributed: not timeable on the GPU, reported as such).
Either way the line carries gpu_us_per_step and exposed_frac."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--config", "C1", "--steps", "8", "--warmup", "2", "--spinup-steps", "3", "--diag-steps", "2",
        "--no-cpu-baseline"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(out: str) -> dict:
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def test_bench_world1_native_rccl(cuda):
    env = _env()
    env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, "bench.py", "--force-dist"] + ARGS, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    ar = _line(p.stdout)["allreduce"]
    assert ar["native"] is True and ar["rccl_nranks"] == 1
    assert ar["collectives_per_step"] == 1  # one range at world size 1 (overlap_chunks)
    assert ar["gpu_us_per_step"] > 0
    assert 0.0 <= ar["exposed_frac"] < 1.0
    assert ar["ms_per_step_no_collective"] > 0


def test_bench_two_gloo_ranks(cuda):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--dist-backend", "gloo"] + ARGS
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = _line(p.stdout)
    assert line["n_gpus"] == 2
    ar = line["allreduce"]
    assert ar["native"] is False
    assert ar["gpu_us_per_step"] is None and "torch.distributed" in ar["gpu_us_note"]
    assert 0.0 <= ar["exposed_frac"] < 1.0
