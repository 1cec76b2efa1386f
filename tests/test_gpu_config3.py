"""Config 3 at its own geometry (VERDICT r3 missing #2): the BraTS 240 x 240 x 155 x 4 case
through the sharded sliding-window path, against what the REFERENCE produced for the same case
(tests/golden/gen_config3_fixture.py: the vendored MONAI's SlidingWindowInferer over the
reference Waveformer, roi 128^3, sw_batch 2, overlap 0.5, gaussian; monai/inferers/utils.py:
216-299, 4_predict.py:199-205).

Two gloo ranks share the one GPU (tests/sw_worker.py, spawned before this process touches the
GPU); the 18 windows are dealt round-robin, all-gathered and stitched on every rank.  Checks:
  * Dice of the argmax labels (TC / WT / ET) against the reference's labels >= 1 - 1e-3
    (north_star's bar);
  * the logits' summary against the reference's: sqrt(sum of squares) within 2e-4 relative and
    the strided sample within rel-L2 2e-4 (the bf16x3 path's full-model tolerance is 1e-4 per
    tensor; the sample is dominated by low-margin voxels);
  * both ranks stitched bit-identical cases.
"""
import json
import math
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))
from gen_config3_fixture import unpack_labels  # noqa: E402

from tests import cases as C  # noqa: E402

FIX = os.path.join(HERE, "golden", "config3_fixture.npz")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("exchange", ["allgather", "allreduce"])
def test_config3_sharded_sliding_window_vs_reference(tmp_path, exchange):
    """exchange: the per-round all-gather of window logits + stitch on every rank, or (SURVEY
    8e's alternative) each rank's partial stitch + one all-reduce + divide."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    fx = np.load(FIX)
    world = 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE=str(world), PYTHONPATH=REPO, WF_SW_EXCHANGE=exchange)
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "sw_worker.py"),
                                       str(tmp_path)], env=e, cwd=REPO, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=300)
            logs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    reps = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(world)]
    shape = tuple(int(v) for v in fx["c3__shape"])
    for rep in reps:
        assert tuple(rep["shape"]) == shape
    sums = reps[0]["all_rank_sums"]
    assert all(s == sums[0] for s in sums), sums
    s0 = np.load(tmp_path / "sample_0.npy")
    assert np.array_equal(s0, np.load(tmp_path / "sample_1.npy"))
    ref = fx["c3__sum"]
    assert abs(math.sqrt(reps[0]["sum"][1]) / math.sqrt(ref[1]) - 1) <= 2e-4
    assert C.rel_l2(torch.from_numpy(s0), torch.from_numpy(fx["c3__sample"])) <= 2e-4
    lab = torch.from_numpy(np.load(tmp_path / "labels.npy")).long()
    want = torch.from_numpy(unpack_labels(fx["c3_labels_packed"], tuple(fx["c3_labels_shape"]))).long()
    assert lab.shape == want.shape
    d = [C.dice(a, b) for a, b in zip(C.brats_regions(lab), C.brats_regions(want))]
    assert min(d) >= 1 - 1e-3, d
