#!/bin/bash
# Rehearsal of the driver's multi-GPU bench launch on one GPU (ranks
# oversubscribed: LOCAL_RANK % device count): torchrun with N ranks, every
# rank checks its gathered batches against the oracle (--check-all-ranks).
# Not a scaling measurement: all ranks share one device.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
for N in ${RANKS:-4 8}; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N --steps ${STEPS:-6} --warmup 2 --no-cpu --oversubscribe --check-all-ranks \
    > gpurun_out/multirank_n$N.json 2> gpurun_out/multirank_n$N.err || { echo "ranks $N failed"; tail -30 gpurun_out/multirank_n$N.err; exit 1; }
  python -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g=d['gathered']; p=d['parity_sample']
print('ranks', d['n_gpus'], 'frames/s', d['value'], 'gathered', g['frames'], 'whole_and_disjoint', g['whole_and_disjoint'], 'parity', p['bit_exact'], p['frames'], 'frames over', p['ranks'], 'ranks')
" gpurun_out/multirank_n$N.json
done
