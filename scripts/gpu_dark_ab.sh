#!/bin/bash
# Dark-tile skipping: parity tests, then the bench with and without it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-dark}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_pipeline.py} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for dk in 1 0; do
for sl in ${SPLITS:-"4 1" "1 1" "1 4"}; do
  set -- $sl
  LM_CORR_DARK=$dk timeout -k 10 240 python bench.py --no-cpu --streams $1 --lanes $2 --steps 40 --warmup 5 > gpurun_out/bench_${TAG}_d${dk}_s$1_l$2.json 2> gpurun_out/bench_${TAG}_d${dk}_s$1_l$2.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_d${dk}_s$1_l$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('dark=$dk s$1 l$2', d['value'], 'k_corr', d['roofline']['avg_launch_ms'], d['roofline']['frac'])" gpurun_out/bench_${TAG}_d${dk}_s$1_l$2.json
done
done
