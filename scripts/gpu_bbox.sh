#!/bin/bash
# BB pass GPU parity tests.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bbox.py -x -v --timeout 120 --timeout-method thread > gpurun_out/bbox_tests.log 2>&1
rc=$?
tail -40 gpurun_out/bbox_tests.log
exit $rc
