"""Config 4 under DistributedDataParallel as the reference trainer builds it
(light_training/trainer.py:353-358: convert_sync_batchnorm + DDP(find_unused_parameters=True)).

Two gloo ranks on the one GPU (tests/ddp_worker.py) train two AdamW steps of the 32^3 x 4
Waveformer through the custom autograd Functions, one sample each.  Rank 0 recomputes both
steps' gradients on un-wrapped models (step 2 from DDP's own post-AdamW parameters): "accum" /
"accum2" = one B = 1 pass per sample, accumulated (what the all-reduce sums), "concat" = one
pass over the concatenated batch.  Checked here:
  * every parameter that gets a gradient in the single-process runs gets one under DDP, and no
    other (DDP's unused-parameter search agrees with autograd), at both steps -- step 2 is
    where a reducer that missed a parameter would fail;
  * DDP's averaged gradients equal every single-process reference to rel-L2 <= 1e-2 per
    tensor, and DDP's worst deviation from "accum" is within 4x the run-to-run noise of the
    single-process computation itself (|accum - accum2|).  That noise is not zero: the
    attention backward's dQ / dBias and the decoder conv's split-K sums are fp32 atomics, and
    the decoder's InstanceNorms on 2^3..16^3 maps amplify their rounding through the backward
    (measured: noise 1.8e-3, DDP vs accum 2.4e-3, vs concat 3.1e-3 worst tensor).  A DDP
    error (a missed bucket, a sum instead of a mean) is O(1).
  Gradients whose true value is 0 (conv biases ahead of a non-affine InstanceNorm) are
  rounding noise on every side and are compared against 1e-6 of the largest gradient norm.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


# rel-L2 bars per tensor against each single-process reference (see module docstring)
BARS = {"accum": 1e-2, "accum2": 1e-2, "concat": 1e-2}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ddp_two_ranks_match_single_process(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    world = 2
    out = tmp_path / "ddp.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE=str(world), PYTHONPATH=REPO)
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "ddp_worker.py"),
                                       str(out)], env=e, cwd=REPO, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=240)
            logs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    report = json.loads(out.read_text())
    assert len(report["steps"]) == 2
    worst = {}
    bad = []
    for step, rows in enumerate(report["steps"]):
        for mode in report["modes"]:
            none_mismatch = [k for k, r in rows.items() if r[mode + "_none"] != r["ddp_none"]]
            assert not none_mismatch, (step, mode, none_mismatch)
        with_grad = {k: r for k, r in rows.items() if not r["ddp_none"]}
        assert len(with_grad) > 200, (step, len(with_grad))
        big = max(r["norm"] for r in with_grad.values())
        for k, r in with_grad.items():
            for mode in list(BARS) + ["noise"]:
                if r["norm"] < 1e-6 * big:  # true gradient 0: noise on every side
                    if not r[mode] <= 1e-6 * big:
                        bad.append((step, mode, k, r[mode]))
                    continue
                e = r[mode] / r["norm"]
                worst[mode] = max(worst.get(mode, 0.0), e)
                # a tensor whose own single-process run-to-run noise is already a large part
                # of the bar (stage-4 biases summed over a handful of positions) is held to 4x
                # that noise instead
                bar = max(BARS[mode], 4 * r["noise"] / r["norm"]) if mode in BARS else None
                if mode in BARS and not e <= bar:
                    bad.append((step, mode, k, e, r["noise"] / r["norm"]))
    print("DDP vs single-process, worst rel-L2 per reference:", worst)
    assert not bad, bad[:8]
    # DDP adds nothing beyond the run-to-run noise of the single-process computation
    assert worst["accum"] <= 4 * worst["noise"] + 1e-6, worst
