set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in 1 2; do
for cfg in 4x1x256x40 4x1x512x20 1x4x256x160 1x4x384x106 1x4x512x80; do
  IFS=x read -r s l b n <<< "$cfg"
  timeout -k 10 240 python bench.py --no-cpu --streams $s --lanes $l --batch $b --steps $n --warmup 5 > gpurun_out/bench_bs4_${cfg}_$rep.json 2> gpurun_out/bench_bs4_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_bs4_$cfg.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench $cfg $rep', d['value'], d['parity_sample']['bit_exact'] if 'parity_sample' in d else '-', 'k_corr', r['avg_launch_ms'], r['frac'])" gpurun_out/bench_bs4_${cfg}_$rep.json
done; done
