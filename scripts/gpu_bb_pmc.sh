#!/bin/bash
# PMC counters of the BB pass kernels (one pass, SQ block only).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/bb_pmc
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -f csv -d gpurun_out/bb_pmc -o pmc -- python -u bench.py --workload bb --steps 2 --warmup 0 --no-cpu > gpurun_out/bb_pmc/run.log 2>&1 || { tail -5 gpurun_out/bb_pmc/run.log; exit 1; }
f=$(find gpurun_out/bb_pmc -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: int(v) for c, v in sorted(d.items())})
PY
