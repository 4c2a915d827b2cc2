#!/bin/bash
# LM_CORR_F16: its GPU tests, then the C5 / C3 f16 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-f16}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f16.py > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for cfg in c5 c3; do
  timeout -k 10 300 python bench.py --no-cpu --config $cfg --precision f16 --steps ${STEPS:-10} --warmup 2 > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err \
    || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench $cfg f16', d['value'], 'k_corr', r['avg_launch_ms'], r['frac'], r['algorithmic_frac'])" gpurun_out/bench_${TAG}_$cfg.json
done
