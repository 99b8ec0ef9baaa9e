#!/bin/bash
# one GPU call for a round's evidence: the full bench line + its rocprofv3 kernel summary
# (round_bench.sh), the sweep's HBM traffic passes (pmc_traffic.sh) and its utilisation
# passes (pmc.sh util); summarise afterwards with mk_profiles.py <tag> <round> and
# pmc_util.py util <round>
set -o pipefail
tag=${1:-r02}
bash tools/round_bench.sh "$tag" && bash tools/pmc_traffic.sh && bash tools/pmc.sh util --n 10000000 --iters 1
