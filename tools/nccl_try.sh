#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 2 --backend nccl --splats 1000000 --steps 1 --warmup 1 \
    --no-cpu-baseline > gpurun_out/nccl_try.json 2> gpurun_out/nccl_try.err
echo "rc=$?"
tail -5 gpurun_out/nccl_try.err | cut -c1-400
cat gpurun_out/nccl_try.json | cut -c1-300
