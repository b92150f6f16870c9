#!/bin/bash
# The bench's N > 1 path rehearsed on a one-GPU box: every rank on cuda:0 over gloo (ALVRL_BENCH_ONE_GPU=1)
set -o pipefail
mkdir -p gpurun_out
export ALVRL_BENCH_ONE_GPU=1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse_w2.json 2> gpurun_out/rehearse_w2.err &&
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse_w4.json 2> gpurun_out/rehearse_w4.err
