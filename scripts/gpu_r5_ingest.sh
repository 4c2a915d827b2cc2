#!/bin/bash
# GPU tests of the tree, then per-kernel durations alone (one stream) and the
# correlation traffic of the experiment libraries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5i/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5i/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r5i/gpu_tests.log | head -20; exit $rc; }
KERNELS="k_ingest k_corr" bash scripts/gpu_kstats_ab.sh || exit 1
bash scripts/gpu_traffic_ab.sh || exit 1
