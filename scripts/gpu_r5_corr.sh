#!/bin/bash
# Round-5 k_corr_rw investigation in one call: (1) throughput A/B of the
# experiment libraries in locomouse_cpp_amd/exp/ against the in-tree one
# (gpu_ab_lib.sh), (2) per-width PMC passes of the in-tree library with one
# stream and per-width launches (LM_CORR_PLAN=0; scripts/pmc_r5.txt) plus the
# clock / VALU-busy summary, (3) optional 1,250-frame shard shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
S=",${STEPS:-ab,pmc,shard},"
on() { [[ $S == *",$1,"* ]]; }
if on ab; then
  REPS=${REPS:-3} CHECK=${CHECK:-1} bash scripts/gpu_ab_lib.sh || exit 1
fi
if on pmc; then
  LM_CORR_PLAN=0 TAG=${PMC_TAG:-r5pmc} PMC_FILE=scripts/pmc_r5.txt bash scripts/gpu_prof1.sh > gpurun_out/pmc_run.txt 2>&1 || { tail -20 gpurun_out/pmc_run.txt; exit 1; }
  python3 scripts/pmc_clock.py gpurun_out/${PMC_TAG:-r5pmc} k_corr > gpurun_out/${PMC_TAG:-r5pmc}/clock.txt && cat gpurun_out/${PMC_TAG:-r5pmc}/clock.txt
fi
if on shard; then
  mkdir -p gpurun_out/shard
  for v in ${SHARD_SHAPES:-1:4:320 1:5:256 1:4:208 1:8:160 1:6:216 2:2:320 2:4:320}; do
    IFS=: read ns nl nb <<< "$v"
    timeout -k 10 240 python3 -u bench.py --video-frames 1250 --streams $ns --lanes $nl --batch $nb --steps 10 --warmup 3 --no-cpu > gpurun_out/shard/s_${ns}x${nl}x${nb}.json 2> gpurun_out/shard/s_${ns}x${nl}x${nb}.err || { echo "shard $v failed"; tail -5 gpurun_out/shard/s_${ns}x${nl}x${nb}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['batches'], d['video_check']['bit_exact'])" gpurun_out/shard/s_${ns}x${nl}x${nb}.json
  done
fi
echo done
