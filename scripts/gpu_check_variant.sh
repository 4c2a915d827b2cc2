#!/bin/bash
# Parity of an experiment library: install locomouse_cpp_amd/exp/liblocomouse_hip_<v>.so
# as the product library, run the parity and edge tests, restore.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB gpurun_out/ab/orig_check.so
rc=0
for v in "$@"; do
  cp locomouse_cpp_amd/exp/liblocomouse_hip_$v.so $LIB
  timeout -k 10 400 python3 -m pytest -q -x -p no:cacheprovider --timeout 200 tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_pipeline.py > gpurun_out/ab/$v.check 2>&1
  r=$?; echo "$v check rc=$r: $(tail -1 gpurun_out/ab/$v.check)"; [ $r -eq 0 ] || rc=$r
  [ $r -eq 0 ] || break
done
cp gpurun_out/ab/orig_check.so $LIB
exit $rc
