#!/bin/bash
# f16 + dark-tile tests, then C5 f16 / fp32 and C3 benches (each step time-limited).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-r3p}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f16.py tests/test_gpu_edges.py tests/test_gpu_parity.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/bench_${TAG}_$n.json 2> gpurun_out/bench_${TAG}_$n.err \
    || { echo "bench $n failed"; tail -20 gpurun_out/bench_${TAG}_$n.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench $n', d['value'], 'k_corr', r['avg_launch_ms'], r['frac'], r['algorithmic_frac'])" gpurun_out/bench_${TAG}_$n.json
}
run c5_f16 --config c5 --precision f16 --steps 10 --warmup 2
run c3_f16 --config c3 --precision f16 --steps 20 --warmup 2
run c3_s4 --streams 4 --steps 40 --warmup 5
run c3_s1l4 --streams 1 --lanes 4 --steps 40 --warmup 5
