#!/bin/bash
# Throughput A/B (with parity checks), then the correlation traffic, of the experiment libraries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
REPS=3 CHECK=1 bash scripts/gpu_ab_lib.sh || exit 1
bash scripts/gpu_traffic_ab.sh || exit 1
