#!/bin/bash
# Round 3 check on the current tree: every GPU test, smoke, then the bench
# across context / lane splits (no CPU legs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-r3c}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { cat gpurun_out/smoke_$TAG.txt; exit 1; }
fi
for sl in ${SPLITS:-"4 1" "1 1" "1 2" "1 4" "2 2"}; do
  set -- $sl
  timeout -k 10 240 python bench.py --no-cpu --streams $1 --lanes $2 --steps 40 --warmup 5 > gpurun_out/bench_${TAG}_s$1_l$2.json 2> gpurun_out/bench_${TAG}_s$1_l$2.err \
    || { echo "bench s$1 l$2 failed"; tail -20 gpurun_out/bench_${TAG}_s$1_l$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench s$1 l$2', d['value'], 'k_corr', d['roofline']['avg_launch_ms'], d['roofline']['frac'])" gpurun_out/bench_${TAG}_s$1_l$2.json
done
