#!/bin/bash
# Round-6: the dark-tile counters the bench's timing reads per batch are
# copied on the batch's stream at submit (no synchronous copy on the host's
# path): GPU tests, then the C4 video and the default stream line against
# the previous runtime (prevrt), every line checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_multictx.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
mv locomouse_cpp_amd/exp/liblocomouse_hip_r5.so /tmp/
CHECK=1 TAG=r6ov REPS=3 BENCH_ARGS="--video-frames 10000 --steps 3 --warmup 2" VARIANTS="base:base: prevrt:prevrt:" bash scripts/gpu_ab_combo.sh || exit 1
CHECK=1 TAG=r6o REPS=2 VARIANTS="base:base: prevrt:prevrt:" bash scripts/gpu_ab_combo.sh
