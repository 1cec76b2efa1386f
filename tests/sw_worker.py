"""One rank of the config-3 check (tests/test_gpu_config3.py starts WORLD_SIZE of these before
any GPU call of its own).

The BraTS-shaped 1 x 4 x 240 x 240 x 155 case of tests/golden/gen_config3_fixture.py through
waveformer_amd.inferers.SlidingWindowInferer(roi 128^3, sw_batch 2, overlap 0.5, 'gaussian',
process_group=WORLD) -- 4_predict.py:199-205 -- over the HIP Waveformer with the same rule
weights: the 18 windows are dealt round-robin over the ranks, each round's window logits are
all-gathered (async, overlapping the next round's forward), and every rank stitches the whole
case.  All ranks share cuda:0 of the one GPU box over gloo, so this exercises the sharding,
the exchange and the stitch, not the transport.  Each rank writes its stitched logits'
summary (sum, sum of squares, seeded dot, strided sample) and rank 0 its argmax labels.
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    out_dir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", init_method="env://")
    import waveformer_amd.network_models as NM
    from waveformer_amd import inferers
    from oracle.weight_rule import rule_state_dict, seeded_randn
    from tests import cases as C
    from gen_config3_fixture import MODEL_KW, OVERLAP, ROI, SEED, SHAPE, SW_BATCH

    torch.cuda.set_device(0)
    model = NM.Waveformer(**MODEL_KW)
    model.load_state_dict(rule_state_dict(model.state_dict()), strict=True)
    model = model.eval().cuda()
    x = seeded_randn(SHAPE, SEED).cuda()
    inf = inferers.SlidingWindowInferer(ROI, sw_batch_size=SW_BATCH, overlap=OVERLAP,
                                        mode="gaussian", process_group=dist.group.WORLD)
    with torch.no_grad():
        y = inf(x, model)
    torch.cuda.synchronize()
    sums, sample = C.summary(y)
    rep = {"rank": rank, "world": world, "shape": list(y.shape), "sum": sums.tolist()}
    np.save(os.path.join(out_dir, f"sample_{rank}.npy"), sample.numpy())
    if rank == 0:
        np.save(os.path.join(out_dir, "labels.npy"), y.argmax(1).to(torch.uint8).cpu().numpy())
    # the stitched case must be identical on every rank (same gathered logits, same kernel)
    h = torch.tensor([float(y.double().sum()), float((y.double() ** 2).sum())], dtype=torch.float64)
    hs = [torch.zeros_like(h) for _ in range(world)]
    dist.all_gather(hs, h)
    rep["all_rank_sums"] = [t.tolist() for t in hs]
    json.dump(rep, open(os.path.join(out_dir, f"rank{rank}.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
