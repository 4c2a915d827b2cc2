#!/bin/bash
# A/B of library builds on one box: for each locomouse_cpp_amd/exp/liblocomouse_hip_<v>.so
# (and the in-tree library as "base"), install it as the product library and run the bench
# (no CPU baseline) REPS times; optional quick parity check per variant; restores the original.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB gpurun_out/ab/orig.so
cp $LIB locomouse_cpp_amd/exp/liblocomouse_hip_base.so
for rep in $(seq 1 ${REPS:-2}); do
for f in locomouse_cpp_amd/exp/liblocomouse_hip_*.so; do
  v=$(basename $f .so | sed 's/liblocomouse_hip_//')
  cp $f $LIB
  if [ -n "$CHECK" ] && [ "$rep" = "1" ]; then
    timeout -k 10 300 python3 -m pytest -q -x -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_edges.py > gpurun_out/ab/$v.check 2>&1 || { echo "$v parity FAILED"; tail -5 gpurun_out/ab/$v.check; cp gpurun_out/ab/orig.so $LIB; exit 1; }
  fi
  timeout -k 10 180 python3 bench.py --no-cpu --no-check ${BENCH_ARGS:---steps 40 --warmup 5} > gpurun_out/ab/lib_$v.$rep.json 2> gpurun_out/ab/lib_$v.$rep.err || { echo "$v failed"; tail -5 gpurun_out/ab/lib_$v.$rep.err; cp gpurun_out/ab/orig.so $LIB; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/lib_$v.$rep.json')); print('$v', '$rep', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
done
cp gpurun_out/ab/orig.so $LIB
