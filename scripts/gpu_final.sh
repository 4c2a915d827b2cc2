#!/bin/bash
# Round-end evidence in one GPU call: GPU tests, smoke, bench (with CPU
# baselines), rocprofv3 kernel trace/stats of the bench, and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE) that profiles/pmc_k_corr.json is built from.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-final}
timeout -k 10 420 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { cat gpurun_out/smoke_$TAG.txt; exit 1; }
cat gpurun_out/smoke_$TAG.txt
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --no-check > gpurun_out/prof_$TAG.out 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.out; exit 1; }
python scripts/prof_union.py gpurun_out/prof_$TAG/run_kernel_trace.csv 4 6 > gpurun_out/prof_union_$TAG.txt && cat gpurun_out/prof_union_$TAG.txt
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$TAG/$c
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -f csv -d gpurun_out/pmc_$TAG/$c -o run -- python bench.py --steps 4 --warmup 1 --no-cpu --no-check > gpurun_out/pmc_${TAG}_$c.out 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_${TAG}_$c.out; exit 1; }
  echo "pmc $c ok"
done
python scripts/pmc_traffic.py gpurun_out/pmc_$TAG 256 gpurun_out/pmc_k_corr_$TAG.json > /dev/null && echo "traffic ok"
