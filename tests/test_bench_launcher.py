"""bench.py's own rank launcher (CPU): `python bench.py --gpus N` with no WORLD_SIZE starts N
ranks through torch.distributed.run (light_training/launch.py:81-112 re-launches the same way);
as a rank, or with N = 1, it does not relaunch."""
import os
import sys
from types import SimpleNamespace

import bench


def test_launcher_cmd_shape():
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "7"], 4, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29555"
    j = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[j + 1:] == ["--gpus", "4", "--steps", "7"]


def test_no_relaunch_as_rank_or_single_gpu(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch_ranks(SimpleNamespace(gpus=2)) is None
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.maybe_launch_ranks(SimpleNamespace(gpus=1)) is None


def test_relaunch_runs_child(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 3
    import subprocess
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    assert bench.maybe_launch_ranks(SimpleNamespace(gpus=8)) == 3
    assert "--nproc-per-node=8" in seen["cmd"] and seen["cmd"][-2:] == ["--gpus", "8"]


def test_stamp_marks_rehearsal(monkeypatch):
    monkeypatch.setenv("WF_BENCH_BACKEND", "gloo")
    out = bench._stamp({}, SimpleNamespace(devices=1), 2)
    assert out["devices"] == 1 and "2 ranks on 1 GPU" in out["rehearsal"]
    assert "rehearsal" not in bench._stamp({}, SimpleNamespace(devices=8), 8)
