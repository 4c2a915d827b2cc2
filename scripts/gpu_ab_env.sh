#!/bin/bash
# A/B of runtime switches on one box: for each VARIANTS entry "name:ENV=val,ENV2=val"
# run the bench (no CPU baseline) REPS times; optional GPU tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
for v in ${VARIANTS:-default:}; do
  name=${v%%:*}; envs=${v#*:}
  timeout -k 10 180 env ${envs//,/ } python3 bench.py --no-cpu --no-check ${BENCH_ARGS:---steps 40 --warmup 5} > gpurun_out/ab/${TAG}_$name.$rep.json 2> gpurun_out/ab/${TAG}_$name.$rep.err || { echo "$name failed"; tail -5 gpurun_out/ab/${TAG}_$name.$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${TAG}_$name.$rep.json')); print('$name', '$rep', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
done
