#!/bin/bash
# Round 3, first full check: every GPU test, then the bench across context /
# lane splits, then the correlation A/B (scripts/gpu_corr_ab.sh, no tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-r3a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for sl in "4 1" "1 4" "2 2" "1 6"; do
  set -- $sl
  timeout -k 10 240 python bench.py --no-cpu --streams $1 --lanes $2 --steps 40 --warmup 5 > gpurun_out/bench_${TAG}_s$1_l$2.json 2> gpurun_out/bench_${TAG}_s$1_l$2.err \
    || { echo "bench s$1 l$2 failed"; tail -20 gpurun_out/bench_${TAG}_s$1_l$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench s$1 l$2', d['value'], 'k_corr', d['roofline']['avg_launch_ms'], d['roofline']['frac'])" gpurun_out/bench_${TAG}_s$1_l$2.json
done
NO_TESTS=1 STREAMS="4" TAG=$TAG bash scripts/gpu_corr_ab.sh
