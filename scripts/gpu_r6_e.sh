#!/bin/bash
# Round-6: scalar row offsets in the ring kernels' row loads -- correlation
# GPU tests, an A/B against round 5's library and the 8-wave workgroup
# variant, then whole-video (C4) shapes on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
TAG=r6e REPS=3 VARIANTS="base:base: r5:r5: w8:w8:" bash scripts/gpu_ab_combo.sh || exit 1
for v in ${VIDEO_SHAPES:-8:1:448 8:1:320 4:1:448 6:1:448 4:2:256}; do
  IFS=: read ns nl nb <<< "$v"
  timeout -k 10 300 python -u bench.py --video-frames 10000 --streams $ns --lanes $nl --batch $nb --steps 5 --warmup 2 --no-cpu > $O/video_${ns}x${nl}x${nb}.json 2> $O/video_${ns}x${nl}x${nb}.err || { echo "video $v failed"; tail -5 $O/video_${ns}x${nl}x${nb}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/video_${ns}x${nl}x${nb}.json').read().strip().splitlines()[-1]); print('video $v', d['value'], d['ms_per_step'], d['config']['batches'], d.get('video_check',{}).get('bit_exact'))"
done
