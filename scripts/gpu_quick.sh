#!/bin/bash
# One GPU call: GPU tests, then the default bench REPS times (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-q}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 240 python bench.py --no-cpu ${BENCH_ARGS:---steps 40 --warmup 5} > gpurun_out/bench_${TAG}_$r.json 2> gpurun_out/bench_${TAG}_$r.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], 'k_corr', d['roofline']['avg_launch_ms'], d['roofline']['frac'])" gpurun_out/bench_${TAG}_$r.json
done
