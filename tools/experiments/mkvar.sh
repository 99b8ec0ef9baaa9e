#!/bin/bash
# build a variant of libsplat_hip.so with one source file replaced:
#   tools/experiments/mkvar.sh NAME TARGET SRC.hip   (TARGET = basename of the replaced csrc file, e.g. st_kmeans_nd)
# (experiments only; load it with ST_LIB=tools/var/NAME.so)
set -e
name=$1; base=$2; src=$3
R=$(cd "$(dirname "$0")/../.." && pwd)
B=$R/splat-transform_amd/build
mkdir -p $R/tools/var
flags="-O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result"
[ "$base" = st_kmeans_nd ] && flags="$flags -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans -fno-slp-vectorize"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $flags $EXTRA -I$R/splat-transform_amd/csrc -I$R/include -c $src -o /tmp/var_$name.o
objs=$(ls $B/*.o | grep -v "/${base}.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -pthread -o $R/tools/var/$name.so $objs /tmp/var_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built tools/var/$name.so
