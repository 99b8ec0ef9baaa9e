#!/bin/bash
# sweep time vs point count around whole rounds of 512 resident workgroups (16 point tiles each):
# 38 rounds = 9,961,472 points, 39 rounds = 10,223,616; the bench's 10M is 38.15 rounds
set -o pipefail
for n in 9961472 10000000 10223616 9961472 10000000 10223616; do
  echo "== n=$n"
  timeout -k 10 200 python3 tools/kn_bench.py --n $n --iters 2 2>&1 | grep kn.sweep || exit 1
done
