#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/bm_$tag.json 2> gpurun_out/bm_$tag.err || { echo "FAIL $tag"; tail -20 gpurun_out/bm_$tag.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/bm_$tag.json'));print('$tag', round(d['value'],3), round(d['ms_per_step'],1), d['verified'], d['config']['workload'], d['config']['parallelism'])"; }
run single --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-paths
run dist --dist --steps 2 --warmup 1 --no-cpu-baseline
run merge4 --merge 4 --steps 2 --warmup 1 --no-cpu-baseline
run total50 --total-splats 50000000 --steps 2 --warmup 1 --no-cpu-baseline
