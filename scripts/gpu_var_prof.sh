# Per-dispatch durations of the correlation variants (rocprofv3 kernel stats, one stream).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARS:-3 6 7}; do
  rm -rf gpurun_out/vprof_$v
  LM_CORR_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/vprof_$v -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --streams 1 > gpurun_out/vprof_$v.out 2>&1 || { echo "prof $v failed"; tail -5 gpurun_out/vprof_$v.out; exit 1; }
  echo "== variant $v"; grep k_corr gpurun_out/vprof_$v/run_kernel_stats.csv | awk -F'",' '{print $1"\"", $4}' | sed 's/(LmConst[^"]*//' | cut -c1-60
done
