#!/bin/bash
# One GPU call for the LM_CORR_F16 mode: its tests, then C5 fp32 vs f16 and C3 f16 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-f16}
timeout -k 10 300 python -u -m pytest tests/test_gpu_f16.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for run in "c5 fp32" "c5 f16" "c3 f16"; do
  set -- $run
  timeout -k 10 240 python bench.py --config $1 --precision $2 --steps ${STEPS:-20} --warmup 3 --no-cpu > gpurun_out/bench_${TAG}_$1_$2.json 2> gpurun_out/bench_${TAG}_$1_$2.err || { echo "bench $run failed"; tail -20 gpurun_out/bench_${TAG}_$1_$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'fps', d['roofline']['achieved'], 'TF', d['roofline']['frac'], d['kernel_busy_ms_per_batch'])" gpurun_out/bench_${TAG}_$1_$2.json "$run"
done
