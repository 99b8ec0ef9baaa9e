set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all2.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_paths.py > gpurun_out/paths2.json 2> gpurun_out/paths2.err
rc=$?; tail -3 gpurun_out/gpu_all2.log; python3 -c "
import json; d=json.load(open('gpurun_out/paths2.json'))
for k in ('config3','config3_one_call','config3_host_one_call','config3_file'): print(k, {a:b for a,b in d.get(k,{}).items() if a!='what'})
for k,v in d['stages'].items(): print(k, round(v['ms'],3), round(v['frac_hbm'],3))
" ; exit $rc
