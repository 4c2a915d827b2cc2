#!/bin/bash
# Round-6: GPU tests on this tree (2 x 2-wave f16 kernel, ring LDS sized by
# the correlation unit), then XCD run lengths 16 (base) / 64 / 128: frames/s
# with every line's batches checked, and the correlation traffic of 64 and 128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O /tmp/held
E=locomouse_cpp_amd/exp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
CHECK=1 TAG=r6i REPS=3 VARIANTS="base:base: x64:x64: x128:x128:" bash scripts/gpu_ab_combo.sh || exit 1
mv $E/liblocomouse_hip_r5.so /tmp/held/
bash scripts/gpu_traffic_ab.sh > $O/traffic_ab.txt 2>&1 || { tail -5 $O/traffic_ab.txt; mv /tmp/held/*.so $E/; exit 1; }
mv /tmp/held/*.so $E/; rm -f $E/liblocomouse_hip_base.so
grep -E "hit-rate|^[a-z0-9]+$" $O/traffic_ab.txt
for v in base x64 x128; do python3 -c "import json; d=json.load(open('gpurun_out/traffic/$v/pmc_k_corr.json')); print('$v', d['hbm_bytes_per_launch'], d['hbm_bytes_per_frame'])"; done
timeout -k 10 300 python -u bench.py --config c5 --precision f16 --streams 8 --steps 12 --warmup 2 --no-cpu > $O/bench_c5f16.json 2> $O/bench_c5f16.err || { tail -5 $O/bench_c5f16.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c5f16.json').read().strip().splitlines()[-1]); print('c5f16', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
