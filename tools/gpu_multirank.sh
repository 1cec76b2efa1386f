#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: 2 ranks over gloo sharing cuda:0
# (barriers, MAX-over-ranks timing, rank-0 output; RCCL itself needs distinct GPUs).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
WF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --cpu-baseline 0 --parity 0 > gpurun_out/mr_enc.json 2> gpurun_out/mr_enc.err || { tail -20 gpurun_out/mr_enc.err; exit 1; }
cut -c1-600 gpurun_out/mr_enc.json
WF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload sliding --steps 4 --warmup 1 > gpurun_out/mr_sw.json 2> gpurun_out/mr_sw.err || { tail -20 gpurun_out/mr_sw.err; exit 1; }
cut -c1-600 gpurun_out/mr_sw.json
