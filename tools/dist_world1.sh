mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dist_gpu.py -v --timeout 400 --timeout-method thread > gpurun_out/distg.log 2>&1 && \
timeout -k 10 300 python bench.py --dist --backend nccl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bdist.json 2> gpurun_out/bdist.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/bplain.json 2> gpurun_out/bplain.err
echo rc=$?; tail -5 gpurun_out/distg.log; tail -3 gpurun_out/bdist.err
