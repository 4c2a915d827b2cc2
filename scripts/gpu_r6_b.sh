#!/bin/bash
# Round-6 check: full GPU tests, the MJPEG end-to-end run of the LocoMouse
# program, then throughput A/Bs (workgroup order variants at 8 contexts; the
# single-context plans).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 900 python -u scripts/cli_e2e_mjpeg.py --frames 10000 --reps 2 --out $O/e2e_mjpeg.json > $O/e2e.out 2> $O/e2e.err
rc=$?; tail -c 1500 $O/e2e.out; [ $rc -eq 0 ] || { tail -20 $O/e2e.err; exit $rc; }
TAG=r6b REPS=2 VARIANTS="base:base: r5:r5: c3:c3: i1:i1: i4:i4: pm5:pm5: w8:w8:" bash scripts/gpu_ab_combo.sh || exit 1
TAG=r6b1 REPS=2 BENCH_ARGS="--streams 1 --lanes 4 --steps 40 --warmup 5" VARIANTS="pw:base:LM_CORR_PLAN=0 mg:base:LM_CORR_PLAN=1" bash scripts/gpu_ab_combo.sh
TAG=r6bf REPS=2 BENCH_ARGS="--config c5 --precision f16 --streams 8 --steps 12 --warmup 2" VARIANTS="base:base: fu8:fu8: fu12:fu12:" bash scripts/gpu_ab_combo.sh
