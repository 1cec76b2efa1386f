"""bench.py's N > 1 path (the driver's 2/4/8-GPU scaling runs) rehearsed on the one GPU of the
test box: `python bench.py --gpus 2` exactly as the driver types it -- bench.py starts the two
ranks itself (torch.distributed.run as a child) -- over the gloo backend (WF_BENCH_BACKEND=gloo;
RCCL itself needs distinct GPUs), both on cuda:0.  Each rank builds the encoder, captures its HIP graph, replays it
between the barriers, the MAX of the ranks' times is all-reduced, and rank 0 alone prints the
one JSON line -- with n_gpus = 2 and the whole-job volume count (2 ranks x B x steps)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_one_line():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    env = dict(os.environ, WF_BENCH_BACKEND="gloo", PYTHONPATH=REPO)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--batch", "2", "--parity", "0", "--cpu-baseline", "0", "--op-timers", "0"]
    p = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4
    assert out["devices"] == 1 and "rehearsal" in out  # both ranks folded onto cuda:0
    assert out["config"]["global_batch"] == 4 and out["config"]["per_gpu_batch"] == 2
    assert out["value"] > 0
    # value = all ranks' volumes / the slowest rank's time
    assert abs(out["value"] - 2 * 2 * 4 / (out["ms_per_step"] * 4 / 1e3)) < 1e-6 * out["value"]
