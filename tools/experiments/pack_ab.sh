#!/bin/bash
# chunk pack: parity tests, then the config-3 stage table with the one-wave-per-chunk kernel and
# with the round-2 one-workgroup-per-chunk kernel (ST_PACK_WG=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_process_chain.py tests/test_typed_columns.py tests/test_ply_gpu.py tests/test_gpu_edges.py -q --timeout 200 --timeout-method thread -k "compressed or process or pack or chunk or ply or typed" > gpurun_out/pack_tests.log 2>&1 || { tail -40 gpurun_out/pack_tests.log; exit 1; }
tail -2 gpurun_out/pack_tests.log
for v in new old; do
  if [ $v = old ]; then export ST_PACK_WG=1; fi
  timeout -k 10 300 python tools/bench_paths.py > gpurun_out/pack_$v.json 2> gpurun_out/pack_$v.err || { tail -20 gpurun_out/pack_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pack_$v.json')); p=d.get('paths', d); print('$v', json.dumps({k: (v.get('ms'), round(v.get('frac_hbm', 0), 3)) for k, v in p.items() if isinstance(v, dict) and 'ms' in v}))"
done
