"""bench.py's rank plumbing (CPU): `bench.py --gpus N` without a launcher starts N rank
processes itself (torch.distributed.run as a child, before anything touches a GPU) and
relays rank 0's line; under a launcher WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def test_world_plan():
    assert bench.world_plan(1, {}) == ("single", 1)
    assert bench.world_plan(8, {}) == ("launch", 8)
    assert bench.world_plan(2, {"WORLD_SIZE": "2"}) == ("rank", 2)
    assert bench.world_plan(1, {"WORLD_SIZE": "1"}) == ("rank", 1)
    with pytest.raises(SystemExit):
        bench.world_plan(2, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.world_plan(1, {"WORLD_SIZE": "8"})
    with pytest.raises(SystemExit):
        bench.world_plan(0, {})


def test_launcher_cmd_passes_arguments_through():
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "7"], 4, 12345)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=12345" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"]
    assert os.path.basename(cmd[-5]) == "bench.py"


def test_bench_gpus_2_starts_two_ranks():
    """The real path: `python bench.py --gpus 2` with no launcher runs two ranks (gloo on CPU
    here) and prints rank 0's line with n_gpus 2."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                         capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["rank_sum"] == 3 and rec["local_ranks"] == "2"


def test_bench_refuses_world_size_mismatch():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                         capture_output=True, text=True, timeout=120, env=_env(WORLD_SIZE="1", RANK="0"), cwd=ROOT)
    assert out.returncode != 0
    assert "WORLD_SIZE=1" in out.stderr and "--gpus 2" in out.stderr
