#!/bin/bash
# Round-6: ring window rows as buffer loads (uniform base + scalar row offset
# + 32-bit lane offset) -- all GPU tests, then an A/B against the previous
# global-load source (prev), every line checked against the oracle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
CHECK=1 TAG=r6k REPS=4 VARIANTS="base:base: prev:prev:" bash scripts/gpu_ab_combo.sh
