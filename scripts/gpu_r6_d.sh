#!/bin/bash
# Round-6: the dense ring-wave packing restored -- GPU tests, an A/B against
# round 5's library and the 8-wave workgroup variant, then the C4 shard shapes
# (scripts/gpu_r6_c.sh) and the whole 10,000-frame video on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
TAG=r6d REPS=3 VARIANTS="base:base: r5:r5: w8:w8:" bash scripts/gpu_ab_combo.sh || exit 1
bash scripts/gpu_r6_c.sh || exit 1
timeout -k 10 300 python -u bench.py --video-frames 10000 --steps 5 --warmup 2 --no-cpu > $O/video10k.json 2> $O/video10k.err || { tail -5 $O/video10k.err; exit 1; }
tail -c 600 $O/video10k.json
