#!/bin/bash
# One GPU call's evidence, by named steps (replaces round 5's twenty one-off r05_*.sh wrappers;
# they are in the git history at 9528cc1).  Run from the repo root through gpurun:
#   bash tools/evidence.sh <tag> <step> [<step> ...]
# Outputs go under gpurun_out/<tag>_*; every GPU step runs under its own time limit and the first
# failure ends the call (the log's tail is printed).
#   suite    the whole GPU suite, then smoke() (the round-end driver's two steps)
#   bench    the driver's bench command (bench.py --gpus 1 --steps 20 --warmup 5), summary line
#   prof     the same command under rocprofv3 --kernel-trace --stats (no extra records, no CPU
#            baseline: their launches would mix into the sweep's average)
#   pmc      the sweep's HBM traffic passes + utilisation passes, the fix-up's counter passes
#   configs  BASELINE configs 3/4/5 at full size and the world-8 rehearsal (shared memory)
#   dist     st_dev_sog against the sharded path at world 1 (--dist), interleaved, at an 8-way
#            rank's 1.25M rows and at 10M (wall time per step)
#   dist1    the sharded path at world 1 (one-rank RCCL communicator, torch's process group on gloo)
#            at an 8-way rank's 1.25M rows, verified
#   stats    the N-D assign classification on Gaussian and heavy-tailed SH at 10M (kn_bench)
#   quick    a k-means test selection + kn_bench timings (a quick check of a kernel change)
#   ab       interleaved bench steps of tools/ab/base.so against tools/ab/new.so (ST_LIB; $AB_ARGS
#            extra bench.py arguments, e.g. --total-splats 1250000)
#   abenv    interleaved bench steps of this library with and without $AB_ENV (VAR=value) ($AB_ARGS)
#   node     the Node drop-in's PLY -> .sog job with phase stamps (tools/node_probe.py)
#   read     readPly's host form under its settings (tools/read_probe.py)
#   paths    the config-3 stage table and file paths (tools/bench_paths.py)
set -o pipefail
tag=${1:?usage: evidence.sh <tag> <step>...}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/$tag
fail() { echo "step $1 failed"; tail -40 "$2"; exit 1; }
for step in "$@"; do
  case $step in
  suite)
    timeout -k 10 880 python -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread > ${O}_suite.log 2>&1 \
      || fail suite ${O}_suite.log
    tail -3 ${O}_suite.log
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > ${O}_smoke.log 2>&1 \
      || fail smoke ${O}_smoke.log
    tail -2 ${O}_smoke.log ;;
  bench)
    timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > ${O}_bench.json 2> ${O}_bench.err \
      || fail bench ${O}_bench.err
    python3 -c "
import json; r = json.load(open('${O}_bench.json'))
print('bench', round(r['value'], 3), round(r['ms_per_step'], 2), r['verified'], round(r['roofline']['avg_launch_ms'], 3),
      round(r['roofline']['frac'], 4))
e = r['end_to_end_file'] or {}
nh = e.get('node_host') or {}
print('e2e', round(e.get('Msplats_per_s', 0), 2), 'node', round(nh.get('Msplats_per_s', 0), 2), nh.get('archive_equals_library'))
rr = (r['extra_records'] or {}).get('realistic_10M') or {}
print('realistic', rr.get('ms_per_step'), rr.get('vs_main_step'), rr.get('verified'))" ;;
  prof)
    rm -rf ${O}_prof
    timeout -k 10 700 rocprofv3 --kernel-trace --stats -d ${O}_prof -o bench --output-format csv -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > ${O}_prof.json 2> ${O}_prof.err \
      || fail prof ${O}_prof.err
    echo profiled ;;
  pmc)
    bash tools/pmc_traffic.sh && bash tools/pmc.sh util --n 10000000 --iters 1 > ${O}_util.log && bash tools/pmc_fix.sh \
      && python3 tools/pmc_fix.py gpurun_out gpurun_out/pmc_fixup.json > /dev/null || { echo "step pmc failed"; exit 1; }
    echo pmc done ;;
  configs)
    timeout -k 10 880 python -u -m pytest -x -v --timeout 840 --timeout-method thread tests/test_configs_full_gpu.py \
      tests/test_world8_gpu.py > ${O}_configs.log 2>&1 || fail configs ${O}_configs.log
    tail -3 ${O}_configs.log ;;
  dist)
    for n in 1250000 10000000; do
      for i in 1 2; do
        for m in single dist; do
          f=""; [ $m = dist ] && f="--dist"
          timeout -k 10 300 python3 bench.py $f --total-splats $n --steps 6 --warmup 1 --no-verify --no-cpu-baseline \
            --no-e2e --no-paths --no-extra > ${O}_dist_$m$n$i.json 2> ${O}_dist_$m$n$i.err || fail dist ${O}_dist_$m$n$i.err
          python3 -c "import json; r=json.load(open('${O}_dist_$m$n$i.json')); print('$m', $n, $i, round(r['ms_per_step'], 2))"
        done
      done
    done ;;
  dist1)
    timeout -k 10 300 python3 bench.py --dist --total-splats 1250000 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
      --no-paths --no-extra > ${O}_dist1.json 2> ${O}_dist1.err || fail dist1 ${O}_dist1.err
    python3 -c "
import json; r = json.load(open('${O}_dist1.json'))
print('dist1', round(r['ms_per_step'], 2), r['transport'], r['torch_backend'], r['rccl_version'], r['verified'])" ;;
  stats)
    for d in gauss t3; do
      timeout -k 10 300 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist $d > ${O}_stats_$d.txt 2>&1 \
        || fail stats ${O}_stats_$d.txt
      grep "kmeans total\|assign classification" ${O}_stats_$d.txt
    done ;;
  quick)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_sog65k.py tests/test_config2_gpu.py \
      tests/test_dist_gpu.py tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_quick.log 2>&1 \
      || fail quick ${O}_quick.log
    tail -2 ${O}_quick.log
    for rep in 1 2; do
      timeout -k 10 170 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist gauss > ${O}_q$rep.log 2>&1 \
        || fail quick ${O}_q$rep.log
      echo "$rep: $(grep -h 'kmeans total\|kn.fixrow\|kn.sweep' ${O}_q$rep.log | tr '\n' ' ')"
    done ;;
  ab)
    for i in 1 2 3 4; do
      for v in base new; do
        ST_LIB=tools/ab/$v.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
          --no-paths --no-extra --no-verify $AB_ARGS > ${O}_ab_$v$i.json 2> ${O}_ab_$v$i.err || fail ab ${O}_ab_$v$i.err
        python3 -c "import json; b=json.load(open('${O}_ab_$v$i.json')); k=b['kernels']; print('$v', $i, round(b['ms_per_step'], 2), b['textures_sha256'][:12], 'fixrow', round(k['kn.fixrow']['avg_ms'], 3), 'sweep', round(k['kn.sweep']['avg_ms'], 2))"
      done
    done ;;
  abenv)
    # the same library with and without $AB_ENV (e.g. ST_FIX_SERIAL=1), interleaved; $AB_ARGS as for ab
    for i in 1 2 3 4; do
      for v in base env; do
        e=""; [ $v = env ] && e="$AB_ENV"
        env $e timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
          --no-paths --no-extra --no-verify $AB_ARGS > ${O}_abe_$v$i.json 2> ${O}_abe_$v$i.err || fail abenv ${O}_abe_$v$i.err
        python3 -c "import json; b=json.load(open('${O}_abe_$v$i.json')); k=b['kernels']; print('$v', $i, round(b['ms_per_step'], 2), b['textures_sha256'][:12], 'fixrow', round(k['kn.fixrow']['avg_ms'], 3), 'sweep', round(k['kn.sweep']['avg_ms'], 2))"
      done
    done ;;
  node)
    timeout -k 10 500 python3 -u tools/node_probe.py > ${O}_node.log 2>&1 || fail node ${O}_node.log
    grep -v 'st xfer' ${O}_node.log | tail -30 ;;
  read)
    ST_DEBUG=1 timeout -k 10 500 python3 -u tools/read_probe.py > ${O}_read.log 2>&1 || fail read ${O}_read.log
    tail -3 ${O}_read.log ;;
  paths)
    timeout -k 10 500 python3 -u tools/bench_paths.py > ${O}_paths.log 2>&1 || fail paths ${O}_paths.log
    cp gpurun_out/paths.json ${O}_paths.json
    python3 -c "import json; d=json.load(open('${O}_paths.json')); print(json.dumps(d['config3_file']))" ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
