#!/bin/bash
# 2-rank rehearsal of bench.py's multi-GPU path on a 1-GPU box (gloo, both ranks on cuda:0)
set -o pipefail
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --backend gloo --splats ${1:-2000000} --steps 1 --warmup 1 \
    --no-cpu-baseline > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err || { tail -30 gpurun_out/rehearsal.err; exit 1; }
cat gpurun_out/rehearsal.json
