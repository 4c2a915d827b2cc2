#!/bin/bash
# GPU tests of the new edge cases, then the isolated correlation profile with
# the VALU / clock PMC passes (scripts/pmc_valu.txt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-r3b}
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_edges.py -k "occlusion or beyond_lds" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
PMC_FILE=scripts/pmc_valu.txt TAG=prof_$TAG PROF_ARGS="--streams 1 --steps 12 --warmup 3 --no-cpu" bash scripts/gpu_prof1.sh > gpurun_out/prof_$TAG.txt 2>&1
rc=$?; tail -5 gpurun_out/prof_$TAG.txt; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_clock.py gpurun_out/prof_$TAG corr
