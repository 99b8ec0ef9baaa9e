set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in "8 8" "16 8" "8 4" "4 8" "12 12"; do
  set -- $cfg
  ST_XFER_THREADS=$1 ST_PLY_READERS=$2 timeout -k 10 200 python3 -u tools/read_probe.py > gpurun_out/rp_$1_$2.log 2>&1 || { tail -5 gpurun_out/rp_$1_$2.log; exit 1; }
  echo "xfer=$1 readers=$2 $(tail -1 gpurun_out/rp_$1_$2.log)"
done
