#!/bin/bash
# A/B correlation variants in one box session (same device, interleaved rounds).
cd "${GRAFT_REPO_ROOT:-.}"
for round in 1 2; do
  for v in ${VARIANTS:-1 2 3}; do
    LM_CORR_VARIANT=$v timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu | python -c "import json,sys; d=json.load(sys.stdin); print('variant $v round $round', d['value'], 'corr_ms', d['kernel_avg_ms']['k_corr'], 'TF', d['roofline']['achieved'])" || exit 1
  done
done
