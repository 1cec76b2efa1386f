"""Probe: can two ranks on ONE MI355X run an RCCL (backend 'nccl') all-reduce / all-gather?
torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_probe.py"""
import os
import time

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1 << 20,), float(rank + 1), device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
ok = bool((x == sum(range(1, world + 1))).all())
g = torch.empty(world * 1024, device="cuda")
dist.all_gather_into_tensor(g, torch.full((1024,), float(rank), device="cuda"))
torch.cuda.synchronize()
ok2 = all(bool((g[r * 1024:(r + 1) * 1024] == r).all()) for r in range(world))
n = 64 << 20
big = torch.ones(n // 4, device="cuda")
dist.barrier()
t0 = time.perf_counter()
for _ in range(5):
    dist.all_reduce(big)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 5
if rank == 0:
    print(f"RCCL_PROBE world={world} allreduce_ok={ok} allgather_ok={ok2} "
          f"64MB allreduce {dt * 1e3:.2f} ms", flush=True)
dist.destroy_process_group()
