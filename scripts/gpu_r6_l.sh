#!/bin/bash
# Round-6: ring stores and ds_read2 rows at precomputed LDS byte addresses
# plus one scalar slot offset (base) vs the stores only (la) vs neither (bl):
# correlation GPU tests, then an A/B with every line checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
CHECK=1 TAG=r6l REPS=3 VARIANTS="base:base: la:la: bl:bl:" bash scripts/gpu_ab_combo.sh
