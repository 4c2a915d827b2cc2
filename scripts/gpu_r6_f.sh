#!/bin/bash
# Round-6: per-kernel durations of this tree's library vs round 5's at the
# default bench shape, then C4 shapes: the whole 10,000-frame video on one
# GPU and the 1,250-frame shard, each line checked frame by frame.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
BENCH_ARGS="--steps 10 --warmup 3 --no-cpu --no-check" KERNELS="k_" bash scripts/gpu_kstats_ab.sh > $O/kstats.txt 2>&1 || { tail -5 $O/kstats.txt; exit 1; }
cat $O/kstats.txt
for v in ${VIDEO_SHAPES:-4:2:256 4:2:313 4:2:357 4:3:256 6:2:256 8:2:313 8:2:250 4:2:209}; do
  IFS=: read ns nl nb <<< "$v"
  timeout -k 10 300 python -u bench.py --video-frames 10000 --streams $ns --lanes $nl --batch $nb --steps 5 --warmup 2 --no-cpu > $O/video_${ns}x${nl}x${nb}.json 2> $O/video_${ns}x${nl}x${nb}.err || { echo "video $v failed"; tail -5 $O/video_${ns}x${nl}x${nb}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/video_${ns}x${nl}x${nb}.json').read().strip().splitlines()[-1]); print('video $v', d['value'], d['ms_per_step'], d['config']['batches'], d.get('video_check',{}).get('bit_exact'))"
done
for v in ${SHARD_SHAPES:-1:4:250 1:4:209 1:5:250 1:3:313 1:6:209 2:2:209}; do
  IFS=: read ns nl nb <<< "$v"
  timeout -k 10 300 python -u bench.py --video-frames 1250 --streams $ns --lanes $nl --batch $nb --steps 10 --warmup 3 --no-cpu > $O/shard_${ns}x${nl}x${nb}.json 2> $O/shard_${ns}x${nl}x${nb}.err || { echo "shard $v failed"; tail -5 $O/shard_${ns}x${nl}x${nb}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/shard_${ns}x${nl}x${nb}.json').read().strip().splitlines()[-1]); print('shard $v', d['value'], d['ms_per_step'], d['config']['batches'], d.get('video_check',{}).get('bit_exact'))"
done
