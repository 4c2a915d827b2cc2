#!/bin/bash
# Throughput vs contexts per GPU (and k_corr serialisation across contexts).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for cfg in "1 1" "2 1" "2 0" "3 1" "4 1"; do
  set -- $cfg
  LM_CORR_SERIALIZE=$2 timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu --streams $1 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('streams $1 serialize $2:', d['value'], 'corr_ms', d['kernel_avg_ms']['k_corr'], 'TF', d['roofline']['achieved'], d['kernel_avg_ms'])" || exit 1
done
