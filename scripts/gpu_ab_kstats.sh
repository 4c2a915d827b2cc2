#!/bin/bash
# Throughput A/B (with parity checks) of the experiment libraries, then their
# per-kernel durations alone (one stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
REPS=3 CHECK=1 bash scripts/gpu_ab_lib.sh || exit 1
KERNELS="k_ingest k_corr k_nms k_tail k_post k_minmax" bash scripts/gpu_kstats_ab.sh || exit 1
