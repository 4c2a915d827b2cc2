#!/bin/bash
# Round-6: the multi-rank GPU tests (C4's 8-rank shape at bench.py's new
# default), per-kernel durations alone (one stream) of this tree's library vs
# round 5's, and one C3 video at the default shape on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_multiproc.py -m gpu -x -v --timeout 650 --timeout-method thread > $O/gpu_multiproc.log 2>&1
rc=$?; tail -3 $O/gpu_multiproc.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_multiproc.log | head -20; exit $rc; }
KERNELS="k_corr k_nms k_ingest k_tail k_post" bash scripts/gpu_kstats_ab.sh > $O/kstats_streams1.txt 2>&1 || { tail -5 $O/kstats_streams1.txt; exit 1; }
grep -v "^\[" $O/kstats_streams1.txt | sort -k2,2 -k1,1
timeout -k 10 300 python -u bench.py --video-frames 10000 --steps 5 --warmup 2 --no-cpu > $O/video_default.json 2> $O/video_default.err || { tail -5 $O/video_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/video_default.json').read().strip().splitlines()[-1]); c=d['config']; print('video default', d['value'], d['ms_per_step'], c['contexts_per_gpu'], c['lanes_per_context'], c['batch_frames'], d['video_check']['bit_exact'])"
