#!/bin/bash
# Kernel-trace profile of each locomouse_cpp_amd/exp/liblocomouse_hip_<v>.so (installed in turn as the
# product library), one stream, then the per-kernel union table; restores the original library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abp
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB gpurun_out/abp/orig.so
for f in locomouse_cpp_amd/exp/liblocomouse_hip_*.so; do
  v=$(basename $f .so | sed 's/liblocomouse_hip_//')
  cp $f $LIB
  rm -rf gpurun_out/abp/$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abp/$v -o run -- python3 bench.py ${PROF_ARGS:---streams 1 --steps 12 --warmup 3 --no-cpu} > gpurun_out/abp/$v.out 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abp/$v.out; cp gpurun_out/abp/orig.so $LIB; exit 1; }
  echo "== $v"; python3 scripts/prof_union.py gpurun_out/abp/$v/run_kernel_trace.csv 4 3 | head -16
done
cp gpurun_out/abp/orig.so $LIB
