#!/bin/bash
# Bench over contexts x lanes x batch size (no tests, no CPU legs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-bs}
for cfg in ${CFGS:-4x1x256 4x1x512 2x2x512 1x4x512 8x1x256 2x4x256}; do
  IFS=x read -r s l b <<< "$cfg"
  timeout -k 10 240 python bench.py --no-cpu --streams $s --lanes $l --batch $b --steps $((10240 / (s * b))) --warmup 3 > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err \
    || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench $cfg', d['value'], 'steps', d['steps'], 'k_corr', r['avg_launch_ms'], r['frac'])" gpurun_out/bench_${TAG}_$cfg.json
done
