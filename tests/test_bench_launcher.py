"""CPU: bench.py's multi-GPU entry point.  `python bench.py --gpus N`
without a torch.distributed environment must start N ranks as a child process (the
driver's own `torch.distributed.run` form), and every rank must refuse a world size
that differs from --gpus."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launcher_command_is_the_drivers_form():
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "5", "--warmup", "2"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5", "--warmup", "2"]


def test_world_size_mismatch_refused():
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 4"):
        bench.check_world(2, 4)
    bench.check_world(4, 4)


def test_rank_refuses_mismatch_before_touching_the_gpu():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--no-cpu-baseline"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr


def test_parent_forwards_child_exit_code(monkeypatch):
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    assert "--nproc-per-node=2" in seen["cmd"]
