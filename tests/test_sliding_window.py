"""CPU: sliding-window inference and flip-TTA (config 3) -- the oracle against fixtures made by
the reference's own MONAI / Predictor (tests/golden/gen_sliding_window_fixtures.py), and the
product's host logic (window enumeration, padding, round-robin sharding, per-round gather
layout) on CPU tensors with the oracle standing in for the two HIP kernels, single-process
and over gloo process groups of 2 and 3 ranks."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from gen_sliding_window_fixtures import CASES, TTA, toy_predictor  # noqa: E402

from oracle import ref_sliding_window as RS  # noqa: E402
from oracle.weight_rule import seeded_randn  # noqa: E402
from waveformer_amd import inferers  # noqa: E402

FIX = np.load(os.path.join(HERE, "golden", "sw_fixtures.npz"))


def _fx(k):
    return torch.from_numpy(np.array(FIX[k]))


def _cpu_map(roi, mode, sigma_scale, device=None):
    return RS.importance_map(roi, mode, sigma_scale)


@pytest.mark.parametrize("roi", [(16, 16, 16), (12, 12, 12), (12, 20, 8)])
def test_oracle_importance_map_matches_reference(roi):
    got = RS.importance_map(roi, "gaussian", (0.125,) * 3)
    assert torch.equal(got, _fx("imap_gauss_" + "x".join(map(str, roi))))


def test_oracle_importance_map_128():
    got = RS.importance_map((128,) * 3, "gaussian", (0.125,) * 3)[::3, ::3, ::3]
    assert torch.equal(got.contiguous(), _fx("imap_gauss_128x128x128_s3"))


def test_brats_geometry():
    """config 3: 240 x 240 x 155 with roi 128, overlap 0.5 -> starts 0/64/112 and 0/27."""
    img, roi = (240, 240, 155), (128, 128, 128)
    st = inferers.dense_patch_starts(img, roi, inferers.scan_interval(img, roi, (0.5,) * 3))
    assert st == [[0, 64, 112], [0, 64, 112], [0, 27]]
    win = [(z, y, x) for z in st[0] for y in st[1] for x in st[2]]
    assert np.array_equal(np.array(win), FIX["brats_window_starts"])
    assert RS.window_starts(img, roi, (0.5,) * 3) == st
    # 18 windows over 8 ranks, sw_batch 2: 2 rounds of 2 slots (3,3,2,2,2,2,2,2 live)
    assert inferers.shard_plan(18, 8, 2) == (2, 4)
    live = [sum(1 for j in range(4) if r + j * 8 < 18) for r in range(8)]
    assert live == [3, 3, 2, 2, 2, 2, 2, 2]
    # with 8-way TTA: 144 windows -> exactly 18 per rank
    assert inferers.shard_plan(144, 8, 2) == (9, 18)


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference(name):
    shape, seed, roi, sb, ov, mode = CASES[name]
    y = RS.sliding_window_inference(seeded_randn(shape, seed), roi, sb, toy_predictor,
                                    overlap=ov, mode=mode)
    assert torch.equal(y, _fx(name + "_y"))


def test_oracle_tta_matches_reference():
    name, shape, seed, roi, sb, ov, mode, axes = TTA
    x = seeded_randn(shape, seed)
    y = RS.mirror_and_predict(
        x, lambda v: RS.sliding_window_inference(v, roi, sb, toy_predictor, overlap=ov,
                                                 mode=mode), axes)
    assert torch.equal(y, _fx(name + "_y"))


def _product(x, roi, sb, ov, mode, group=None, exchange="allgather"):
    return inferers.sliding_window_inference(x, roi, sb, toy_predictor, overlap=ov, mode=mode,
                                             process_group=group, stitch=RS.stitch,
                                             weight_map_fn=_cpu_map, exchange=exchange,
                                             partial_stitch=RS.stitch_partial,
                                             normalize=RS.normalize)


@pytest.mark.parametrize("name", sorted(CASES))
def test_host_logic_single_process(name):
    shape, seed, roi, sb, ov, mode = CASES[name]
    y = _product(seeded_randn(shape, seed), roi, sb, ov, mode)
    assert torch.equal(y, _fx(name + "_y"))


@pytest.mark.parametrize("name", sorted(CASES))
def test_host_logic_allreduce_single_process(name):
    """The all-reduce exchange on one process: each window's weighted sum and weight in window
    order, then one division -- bitwise the reference's accumulation."""
    shape, seed, roi, sb, ov, mode = CASES[name]
    y = _product(seeded_randn(shape, seed), roi, sb, ov, mode, exchange="allreduce")
    assert torch.equal(y, _fx(name + "_y"))


def test_host_logic_tta():
    name, shape, seed, roi, sb, ov, mode, axes = TTA
    inf = inferers.SlidingWindowInferer(roi, sw_batch_size=sb, overlap=ov, mode=mode)
    x = seeded_randn(shape, seed)
    # TTA passes batched as one window set; CPU stand-ins for the stitch / merge kernels
    orig = inferers.ops.sliding_window_stitch, inferers.ops.importance_map
    try:
        inferers.ops.sliding_window_stitch, inferers.ops.importance_map = RS.stitch, _cpu_map
        y = inferers.maybe_mirror_and_predict(x, toy_predictor, inf, axes, merge=RS.tta_merge)
    finally:
        inferers.ops.sliding_window_stitch, inferers.ops.importance_map = orig
    assert torch.equal(y, _fx(name + "_y"))
    assert inferers.mirror_passes(axes) == [(), (2,), (3,), (4,), (2, 3), (2, 4), (3, 4),
                                            (2, 3, 4)]
    assert inferers.mirror_passes([0, 2]) == [(), (2,), (4,), (2, 4)]


def test_unsupported_options_raise():
    x = torch.zeros(1, 1, 8, 8, 8)
    with pytest.raises(NotImplementedError):
        inferers.sliding_window_inference(x, (4, 4, 4), 1, toy_predictor, buffer_steps=2)
    with pytest.raises(ValueError):
        inferers.sliding_window_inference(x, (4, 4, 4), 1, toy_predictor, overlap=1.0)
    with pytest.raises(NotImplementedError):
        inferers.sliding_window_inference(x, (4, 4, 4), 1, lambda v: v[:, :, ::2],
                                          stitch=RS.stitch, weight_map_fn=_cpu_map)


def _dist_worker(rank, world, port, names, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for name in names:
            shape, seed, roi, sb, ov, mode = CASES[name]
            y = _product(seeded_randn(shape, seed), roi, sb, ov, mode, dist.group.WORLD)
            res[name] = bool(torch.equal(y, _fx(name + "_y")))
            # the all-reduce exchange: the ranks' partial sums meet in rank order
            y2 = _product(seeded_randn(shape, seed), roi, sb, ov, mode, dist.group.WORLD,
                          exchange="allreduce")
            ref = _fx(name + "_y")
            res[name + "_allreduce"] = bool(((y2 - ref).norm() / ref.norm()).item() <= 1e-6)
        # fewer windows than ranks (ranks without windows agree on C via all_reduce)
        x = seeded_randn((1, 1, 10, 10, 10), 5)
        y = _product(x, (10, 10, 10), 1, 0.5, "gaussian", dist.group.WORLD)
        ref = RS.sliding_window_inference(x, (10, 10, 10), 1, toy_predictor, 0.5, "gaussian")
        res["one_window"] = bool(torch.equal(y, ref))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + world
    names = sorted(CASES)
    ps = [ctx.Process(target=_dist_worker, args=(r, world, port, names, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, res in out:
        assert all(res.values()), (rank, res)
