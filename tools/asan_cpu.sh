#!/bin/bash
# the CPU test suite (-m "not gpu") with the host code of the library and the oracle under
# AddressSanitizer + UndefinedBehaviorSanitizer (clang's shared runtime, preloaded into python)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -j8 -C "$R/splat-transform_amd" asan && make -s -C "$R/oracle" asan || exit 1
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export ST_LIB=$R/splat-transform_amd/lib/libsplat_hip_asan.so ST_ORACLE_LIB=$R/oracle/build/libst_oracle_asan.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:verify_asan_link_order=0 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
cd "$R" && LD_PRELOAD=$RT python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
