#!/bin/bash
# WebP / container parity tests, then the container sizes against libwebp at 10M SH-3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_webp_gpu.py tests/test_sog_container_cpu.py tests/test_js_host.py tests/test_multi_gpu.py -x -q --timeout 600 --timeout-method thread -k "webp or bundle or sog or container" > gpurun_out/webp_tests.log 2>&1 || { tail -40 gpurun_out/webp_tests.log; exit 1; }
tail -2 gpurun_out/webp_tests.log
timeout -k 10 600 python3 tools/bench_bundle.py 10000000 > gpurun_out/bundle.log 2>&1 || { tail -20 gpurun_out/bundle.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bundle.json'))
print(d['archive_bytes'], d.get('libwebp_total_bytes'), d['bundle_wall_ms'], d['device_kernel_ms'])
for k,v in d['libwebp_1thread'].items(): print(k, v['ours_bytes'], v['bytes'], round(v['ours_bytes']/v['bytes'],4))"
