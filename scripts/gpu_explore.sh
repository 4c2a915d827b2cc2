#!/bin/bash
# Exploration: throughput vs streams per GPU, correlation variants, and an
# N=2 rehearsal of the multi-process bench (both ranks on the one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
summ='import json,sys; d=json.load(sys.stdin); print(d["n_gpus"], d["config"]["streams_per_gpu"], d["value"], "corr_ms", d["kernel_avg_ms"]["k_corr"], "TF", d["roofline"]["achieved"], d["kernel_avg_ms"])'
for ns in ${STREAMS:-1 2 3}; do
  echo -n "streams $ns: "
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --streams $ns 2>gpurun_out/x_streams_$ns.err | python -c "$summ" || exit 1
done
for v in ${VARIANTS:-3 4 5}; do
  echo -n "variant $v: "
  LM_CORR_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu 2>gpurun_out/x_var_$v.err | python -c "$summ" || exit 1
done
if [ -z "$NO_N2" ]; then
  echo -n "N=2 rehearsal: "
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu 2>gpurun_out/x_n2.err | python -c "$summ" || { tail -20 gpurun_out/x_n2.err; exit 1; }
fi
