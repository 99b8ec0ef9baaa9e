#!/bin/bash
# round 5 (late): st_dev_sog_file against st_dev_sog (alternated) under a kernel trace, with the
# sog-file phase stamps (ST_DEBUG)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/psf
ST_DEBUG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/psf -o sf -- python3 $R/tools/experiments/sog_file_trace.py > $R/gpurun_out/psf.txt 2> $R/gpurun_out/psf.err || { tail -20 $R/gpurun_out/psf.err; exit 1; }
cat $R/gpurun_out/psf.txt; grep "st sog file" $R/gpurun_out/psf.err | tail -4; grep "hook\|splat_hip" $R/gpurun_out/psf.err | tail -6
