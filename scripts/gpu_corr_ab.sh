#!/bin/bash
# Correlation A/B on one box: quick parity on the in-tree library, then for
# the in-tree library ("base") and each locomouse_cpp_amd/exp/liblocomouse_hip_<v>.so:
#   - bench (default 4 streams) and bench --streams 1 with per-width launches,
#   - a rocprofv3 kernel-stats pass of the 1-stream bench (per-width k_corr_rw times).
# The original library is restored at the end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
TAG=${TAG:-ab}
LIB=locomouse_cpp_amd/liblocomouse_hip.so
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py \
    > gpurun_out/ab/${TAG}_parity.log 2>&1
  rc=$?; tail -2 gpurun_out/ab/${TAG}_parity.log; [ $rc -eq 0 ] || exit $rc
fi
cp $LIB gpurun_out/ab/orig.so
cp $LIB locomouse_cpp_amd/exp/liblocomouse_hip_base.so
for f in locomouse_cpp_amd/exp/liblocomouse_hip_*.so; do
  v=$(basename $f .so | sed 's/liblocomouse_hip_//')
  cp $f $LIB
  for st in ${STREAMS:-4 1}; do
    timeout -k 10 180 python bench.py --no-cpu --streams $st --steps ${STEPS:-40} --warmup 5 > gpurun_out/ab/${TAG}_${v}_s$st.json 2> gpurun_out/ab/${TAG}_${v}_s$st.err \
      || { echo "$v bench failed"; tail -5 gpurun_out/ab/${TAG}_${v}_s$st.err; cp gpurun_out/ab/orig.so $LIB; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab/${TAG}_${v}_s$st.json')); print('$v', 's$st', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
  if [ -z "$NO_PROF" ]; then
    rm -rf gpurun_out/ab/prof_${TAG}_$v
    LM_CORR_PLAN=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab/prof_${TAG}_$v -o run -- python bench.py --no-cpu --streams 1 --steps 10 --warmup 2 > gpurun_out/ab/prof_${TAG}_$v.out 2>&1 \
      || { echo "$v rocprof failed"; tail -5 gpurun_out/ab/prof_${TAG}_$v.out; cp gpurun_out/ab/orig.so $LIB; exit 1; }
    python -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'corr' in r['Name']:
        print('$v', r['Name'].split('(')[0], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us')
" gpurun_out/ab/prof_${TAG}_$v/run_kernel_stats.csv
  fi
done
cp gpurun_out/ab/orig.so $LIB
