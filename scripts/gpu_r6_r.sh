#!/bin/bash
# Round-6: stream priorities in the C4 modes (whole video, shard), checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
CHECK=1 TAG=r6rv REPS=3 BENCH_ARGS="--video-frames 10000 --steps 3 --warmup 2" VARIANTS="prio:base: noprio:base:LM_STREAM_PRIO=0" bash scripts/gpu_ab_combo.sh || exit 1
CHECK=1 TAG=r6rs REPS=3 BENCH_ARGS="--video-frames 1250 --steps 10 --warmup 3" VARIANTS="prio:base: noprio:base:LM_STREAM_PRIO=0" bash scripts/gpu_ab_combo.sh
