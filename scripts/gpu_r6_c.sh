#!/bin/bash
# Round-6: the C4 shard (1,250 frames, one rank's share of the 10,000-frame
# video on 8 GPUs) in several context x lane x batch shapes, and the whole
# video on one GPU.  Each line checks every frame against the oracle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
for v in ${SHARD_SHAPES:-1:4:250 2:2:313 2:3:209 2:4:157 3:2:209 4:2:157}; do
  IFS=: read ns nl nb <<< "$v"
  timeout -k 10 300 python -u bench.py --video-frames 1250 --streams $ns --lanes $nl --batch $nb --steps 10 --warmup 3 --no-cpu > $O/shard_${ns}x${nl}x${nb}.json 2> $O/shard_${ns}x${nl}x${nb}.err || { echo "shard $v failed"; tail -5 $O/shard_${ns}x${nl}x${nb}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/shard_${ns}x${nl}x${nb}.json').read().strip().splitlines()[-1]); print('shard $v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('video_check',{}).get('bit_exact'))"
done
