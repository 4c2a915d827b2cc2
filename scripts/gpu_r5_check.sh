#!/bin/bash
# The GPU tests of the tree, then the kernel phase profiles (LM_KPROF=1, one
# stream) and the per-kernel durations alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/check/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/check/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/check/gpu_tests.log | head -20; exit $rc; }
LM_KPROF=1 timeout -k 10 240 python bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-check > gpurun_out/check/kprof.json 2> gpurun_out/check/kprof.txt || { tail -5 gpurun_out/check/kprof.txt; exit 1; }
grep -E "kprof k_ingest|kprof k_nms" gpurun_out/check/kprof.txt | tail -3
KERNELS="${KERNELS:-k_ingest k_nms k_corr}" bash scripts/gpu_kstats_ab.sh
