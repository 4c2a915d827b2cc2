cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for sk in ${SKIPS:-0 1}; do
rm -rf gpurun_out/skip_$sk
LM_CORR_SKIP=$sk timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/skip_$sk -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/skip_$sk.out 2>&1 || { echo fail; tail -3 gpurun_out/skip_$sk.out; exit 1; }
echo "skip=$sk"; python -c "
import csv
for r in csv.DictReader(open('gpurun_out/skip_$sk/run_kernel_stats.csv')):
    if 'k_corr' in r['Name']: print('   ', r['Name'].split('(')[0][:34], round(float(r['AverageNs'])/1e3,1), 'us')"
done
