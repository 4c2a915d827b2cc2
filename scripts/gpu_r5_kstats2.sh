#!/bin/bash
# Per-kernel durations alone of the experiment libraries (twice), then the
# k_nms / k_tail / k_post phase profile of the in-tree library (LM_KPROF=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
KERNELS="k_ingest k_nms k_tail k_corr" bash scripts/gpu_kstats_ab.sh || exit 1
KERNELS="k_ingest k_nms" bash scripts/gpu_kstats_ab.sh || exit 1
LM_KPROF=1 timeout -k 10 240 python bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-check > gpurun_out/kprof.json 2> gpurun_out/kprof.txt || { tail -5 gpurun_out/kprof.txt; exit 1; }
grep "kprof k_nms" gpurun_out/kprof.txt | tail -2
