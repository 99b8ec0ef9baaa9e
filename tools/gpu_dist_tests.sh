mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -v --timeout 500 --timeout-method thread > gpurun_out/distg.log 2>&1 && \
ST_REPLAY_CAP=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v --timeout 250 --timeout-method thread -k "cluster1d or kmeans1d or sog" > gpurun_out/cap0.log 2>&1
echo rc=$?; tail -9 gpurun_out/distg.log; tail -3 gpurun_out/cap0.log
