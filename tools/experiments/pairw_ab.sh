#!/bin/bash
# k-means parity tests on the current library, then pair / ambiguous counts and k-means stage
# times of tools/var/base.so against tools/var/$1.so (experiment)
set -o pipefail
v=${1:-tight}
bash tools/kn_check.sh || exit 1
for lib in base $v base $v; do echo "== $lib"; ST_DEBUG=1 ST_LIB=tools/var/$lib.so timeout -k 10 300 python3 tools/kn_bench.py --n 10000000 --iters 2 2>&1 | grep -E "pairs=|kn\." ; done
