#!/bin/bash
# Round-6 step check: the GPU tests on the in-tree library (optional), then a
# throughput A/B against the experiment libraries in locomouse_cpp_amd/exp/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r6/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r6/gpu_tests.log | head -20; exit $rc; }
fi
REPS=${REPS:-3} bash scripts/gpu_ab_lib.sh
