#!/bin/bash
# One GPU call: parity tests, bench (with CPU baseline), rocprofv3 kernel stats,
# then one PMC pass each for FETCH_SIZE and WRITE_SIZE (HBM traffic).
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$TAG.log
  tail -3 gpurun_out/gpu_tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 40 --warmup 5 --cpu-seconds 10} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
[ -n "$NO_PROF" ] && exit 0
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 20 --warmup 3 --no-cpu ${PROF_ARGS} > gpurun_out/prof_$TAG.out 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.out; exit 1; }
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \;
python scripts/prof_union.py gpurun_out/prof_$TAG/run_kernel_trace.csv 4 ${PROF_SKIP:-6} > gpurun_out/prof_union_$TAG.txt && cat gpurun_out/prof_union_$TAG.txt
[ -n "$NO_PMC" ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$TAG/$c
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -f csv -d gpurun_out/pmc_$TAG/$c -o run -- python bench.py --steps 4 --warmup 1 --no-cpu ${PROF_ARGS} > gpurun_out/pmc_${TAG}_$c.out 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_${TAG}_$c.out; exit 1; }
  echo "pmc $c ok"
done
