#!/bin/bash
# HBM traffic of the HBM-bound kernels (config 3's transform / Morton / chunk pack, the 1-D
# k-means assign of the headline step): FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (kernel trace only, MI355X_MICROARCH.md HBM/rocprofv3 section); summarise with
# tools/pmc_paths.py <round>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmcp_paths_$c -o pmc --output-format csv -- \
      python3 tools/bench_paths.py 10000000 > gpurun_out/pmcp_paths_$c.log 2>&1 || { tail -20 gpurun_out/pmcp_paths_$c.log; exit 1; }
  echo "paths $c done"
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmcp_step_$c -o pmc --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-e2e --no-paths --no-cpu-baseline --no-verify > gpurun_out/pmcp_step_$c.log 2>&1 || { tail -20 gpurun_out/pmcp_step_$c.log; exit 1; }
  echo "step $c done"
done
echo done
