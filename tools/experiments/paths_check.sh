#!/bin/bash
# parity tests of the config-3 path (transform / filter / Morton / chunk pack / PLY) + its stage bench and rocprof
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_ply_gpu.py -x -v --timeout 200 --timeout-method thread -k "transform or morton or compressed or filter or ply or decompress" > gpurun_out/paths_tests.log 2>&1 || { tail -40 gpurun_out/paths_tests.log; exit 1; }
tail -3 gpurun_out/paths_tests.log
bash tools/prof_paths.sh ${1:-paths}
