# Calibrate SQ counters: the pk_fma micro-benchmark vs k_corr (one stream).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cal; export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue; i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $line -f csv -d gpurun_out/cal/u$i -o run -- ./scripts/ubench/pkfma > gpurun_out/cal/u$i.log 2>&1 || { echo "ubench pass $i failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -f csv -d gpurun_out/cal/k$i -o run -- python bench.py --steps 4 --warmup 1 --no-cpu --streams 1 > gpurun_out/cal/k$i.log 2>&1 || { echo "kernel pass $i failed"; exit 1; }
  echo "pass $i ok"
done < scripts/pmc_cal.txt
