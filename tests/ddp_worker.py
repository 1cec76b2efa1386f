"""One rank of the config-4 DDP check (tests/test_gpu_ddp.py starts WORLD_SIZE of these).

The reference trainer wraps the model exactly so (light_training/trainer.py:353-358):
SyncBatchNorm.convert_sync_batchnorm, then DistributedDataParallel(device_ids=[local_rank],
output_device=local_rank, find_unused_parameters=True).  Every rank runs on cuda:0 of the one
GPU box; the process group is gloo (it all-reduces CUDA tensors), so the test exercises DDP's
reducer, bucketing and unused-parameter search around the custom autograd Functions, not the
transport.

Each rank trains two steps (DiceCE, AdamW 1e-4: 3_train.py:72, :96-102) of the 32^3 x 4
Waveformer on its own sample.  DropPath is live (train mode, drop_path_rate 0.1) with its
per-sample factors pinned to a function of (call, global sample index), so rank 0 can replay
the same two steps on un-wrapped models: "concat" = one pass over the concatenated batch
(DiceCE with batch=False is the mean of the per-sample losses, so DDP's averaged gradients must
equal its gradients), "accum" / "accum2" = one pass per sample with the gradients accumulated
(what DDP's all-reduce computes, twice, to expose run-to-run noise).  The second step starts
every reference from the DDP model's own parameters after its AdamW step: AdamW's first update
is lr * sign(g) per element, so gradient noise on near-zero elements moves independent runs
apart by 2 lr in random directions, and their step-2 gradients would differ by a few percent
for that reason alone (measured 4%).  Rank 0 writes the per-parameter |g_ddp - g_ref|,
|g_ref| and |g_accum - g_accum2| to the JSON file named on the command line.
"""
import json
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

KEEP = 0.9
PATTERN = (1 / KEEP, 0.0, 1 / KEEP, 1 / KEEP, 0.0)


def main():
    out_path = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from waveformer_amd import _lib
    _lib.load()
    import waveformer_amd.network_models as NM
    from waveformer_amd.losses import DiceCELoss
    from waveformer_amd.network_models.wave_helper import DropPath
    from oracle.weight_rule import rule_state_dict, seeded_randn

    state = {"call": 0, "samples": [rank]}

    def pinned(self, batch, device):
        assert batch == len(state["samples"])
        k = state["call"]
        state["call"] += 1
        return torch.tensor([PATTERN[(k + g) % len(PATTERN)] for g in state["samples"]],
                            device=device)

    DropPath.sample_scale = pinned

    def make():
        m = NM.Waveformer(img_size=(32,) * 3, in_chans=4, out_chans=4, depths=[2, 2, 2, 2],
                          feat_size=[48, 96, 192, 384], num_heads=[3, 6, 12, 24],
                          drop_path_rate=1 - KEEP)
        m.load_state_dict(rule_state_dict(m.state_dict()), strict=True)
        return m.train().to(dev)

    x_all = seeded_randn((world, 4, 32, 32, 32), 61).to(dev)
    y_all = (seeded_randn((world, 1, 32, 32, 32), 62).abs() * 1.7).long().clamp_(0, 3).to(dev)
    loss_fn = DiceCELoss(to_onehot_y=True, softmax=True)

    model = make()
    model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], output_device=0,
                                                    find_unused_parameters=True)
    opt = torch.optim.AdamW(ddp.parameters(), lr=1e-4)
    ddp_grads = []
    after_step1 = None
    for step in range(2):
        if step == 1:
            after_step1 = {k: v.detach().clone() for k, v in model.state_dict().items()}
        state["call"] = 0
        opt.zero_grad(set_to_none=True)
        loss = loss_fn(ddp(x_all[rank:rank + 1]), y_all[rank:rank + 1])
        loss.backward()
        ddp_grads.append({k: (None if p.grad is None else p.grad.detach().clone())
                          for k, p in model.named_parameters()})
        opt.step()
    torch.cuda.synchronize()
    dist.barrier()

    if rank == 0:
        report = {"steps": [], "modes": ["concat", "accum", "accum2"]}
        refs = {}
        for mode in report["modes"]:
            ref = make()
            grads = []
            for step in range(2):
                if step == 1:  # step 2 from DDP's own post-AdamW parameters (see below)
                    ref.load_state_dict(after_step1)
                ref.zero_grad(set_to_none=True)
                if mode == "concat":  # one pass over the concatenated batch
                    state["call"], state["samples"] = 0, list(range(world))
                    loss_fn(ref(x_all), y_all).backward()
                else:                 # one pass per sample, gradients accumulated (DDP's sum)
                    for r in range(world):
                        state["call"], state["samples"] = 0, [r]
                        (loss_fn(ref(x_all[r:r + 1]), y_all[r:r + 1]) / world).backward()
                grads.append({k: (None if p.grad is None else p.grad.detach().clone())
                              for k, p in ref.named_parameters()})
            refs[mode] = grads
        for step in range(2):
            rows = {}
            for k, g_ddp in ddp_grads[step].items():
                r = {"ddp_none": g_ddp is None}
                for mode in report["modes"]:
                    g_ref = refs[mode][step][k]
                    r[mode + "_none"] = g_ref is None
                    if g_ref is not None and g_ddp is not None:
                        r[mode] = (g_ddp.double() - g_ref.double()).norm().item()
                        r["norm"] = g_ref.double().norm().item()
                a, b = refs["accum"][step][k], refs["accum2"][step][k]
                if a is not None and b is not None:  # run-to-run noise of the same computation
                    r["noise"] = (a.double() - b.double()).norm().item()
                rows[k] = r
            report["steps"].append(rows)
        with open(out_path, "w") as f:
            json.dump(report, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
