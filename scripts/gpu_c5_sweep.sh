#!/bin/bash
# C5 f16 bench over contexts x lanes x batch size (no tests, no CPU legs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for cfg in ${CFGS:-4x1x256x10 4x1x128x20 2x2x256x20 1x4x256x40 4x1x384x7}; do
  IFS=x read -r s l b n <<< "$cfg"
  timeout -k 10 240 python bench.py --no-cpu --config c5 --precision f16 --streams $s --lanes $l --batch $b --steps $n --warmup 2 > gpurun_out/bench_c5s_$cfg.json 2> gpurun_out/bench_c5s_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_c5s_$cfg.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench $cfg', d['value'], 'k_corr', r['avg_launch_ms'], r['frac'])" gpurun_out/bench_c5s_$cfg.json
done
