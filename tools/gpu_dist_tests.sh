#!/bin/bash
# the sharded path's GPU tests (gloo ranks on one GPU + the RCCL leg), one line per test as it ends
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -v --timeout 300 --timeout-method thread 2>&1 | tee gpurun_out/distg.log
