#!/bin/bash
# Throughput vs contexts (HIP streams + host threads) per GPU.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for ns in ${STREAMS:-1 2 3 4}; do
  timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu --streams $ns 2>gpurun_out/streams_$ns.err | python -c "import json,sys; d=json.load(sys.stdin); print('streams $ns:', d['value'], 'corr_ms', d['kernel_avg_ms']['k_corr'], 'TF', d['roofline']['achieved'], d['kernel_avg_ms'])" || exit 1
done
