#!/bin/bash
# streams x batch sweep of bench.py (graphs + frame-batched ingest on)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/sweep2
for cfg in "3 256" "4 256" "2 512" "3 512" "4 192" "5 256"; do
  set -- $cfg
  timeout -k 10 150 python bench.py --streams $1 --batch $2 --steps 30 --warmup 4 --no-cpu > gpurun_out/sweep2/s$1_b$2.json 2>/dev/null || { echo "fail $cfg"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep2/s$1_b$2.json')); print('streams $1 batch $2', d['value'], d['roofline']['frac'])"
done
