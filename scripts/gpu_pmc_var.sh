# SQ counters of the k_corr variants (one stream), two passes each.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pv; export TMPDIR=/tmp
for v in ${VARS:-3 6 7}; do
  i=0
  while read -r line; do
    [ -z "$line" ] && continue; i=$((i+1))
    LM_CORR_VARIANT=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -f csv -d gpurun_out/pv/v${v}_$i -o run -- python bench.py --steps 4 --warmup 1 --no-cpu --streams 1 > gpurun_out/pv/v${v}_$i.log 2>&1 || { echo "pass $v $i failed"; exit 1; }
  done < ${PMC_FILE:-scripts/pmc_var.txt}
  echo "variant $v ok"
done
