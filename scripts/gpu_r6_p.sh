#!/bin/bash
# Round-6: stream priorities at the default 8 contexts (alternating high/low
# vs all equal, LM_STREAM_PRIO=0), every line checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mv locomouse_cpp_amd/exp/liblocomouse_hip_r5.so /tmp/ 2>/dev/null
CHECK=1 TAG=r6p REPS=3 VARIANTS="prio:base: noprio:base:LM_STREAM_PRIO=0" bash scripts/gpu_ab_combo.sh
