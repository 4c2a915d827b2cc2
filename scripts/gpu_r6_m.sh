#!/bin/bash
# Round-6: hardware queues per process (GPU_MAX_HW_QUEUES, 4 on the box) for
# the 8-context default line and the C4 shapes, every line checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
CHECK=1 TAG=r6m REPS=3 VARIANTS="q4:base: q8:base:GPU_MAX_HW_QUEUES=8 q16:base:GPU_MAX_HW_QUEUES=16" bash scripts/gpu_ab_combo.sh || exit 1
CHECK=1 TAG=r6mv REPS=2 BENCH_ARGS="--video-frames 10000 --steps 3 --warmup 2" VARIANTS="q4:base: q8:base:GPU_MAX_HW_QUEUES=8" bash scripts/gpu_ab_combo.sh || exit 1
CHECK=1 TAG=r6ms REPS=2 BENCH_ARGS="--video-frames 1250 --steps 10 --warmup 3" VARIANTS="q4:base: q8:base:GPU_MAX_HW_QUEUES=8" bash scripts/gpu_ab_combo.sh
CHECK=1 TAG=r6ms6 REPS=2 BENCH_ARGS="--video-frames 1250 --lanes 6 --steps 10 --warmup 3" VARIANTS="q8l6:base:GPU_MAX_HW_QUEUES=8" bash scripts/gpu_ab_combo.sh
