#!/bin/bash
# Round-4 GPU check in one call: GPU tests, smoke, bench lines with their
# oracle checks (C3 default, the drop-in 1 context x 4 lanes, C5 fp32), the
# C4 strong-scaling mode on one GPU and rehearsed with 4 oversubscribed
# ranks, and the launcher's refusal of --gpus 2 on a one-GPU box.
# STEPS=tests,smoke,bench,lanes,c5,video,refuse selects steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r4}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
S=",${STEPS:-tests,smoke,bench,lanes,c5,video,refuse},"
on() { [[ $S == *",$1,"* ]]; }
if on tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
fi
if on smoke; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
  tail -2 $O/smoke.txt
fi
bench() {  # name, args...
  local n=$1; shift
  timeout -k 10 420 python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail -20 $O/bench_$n.err; exit 1; }
  python - $O/bench_$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
p = d.get("parity_sample") or d.get("video_check") or {}
print(sys.argv[1].split("/")[-1], d["value"], d["unit"], "n_gpus", d["n_gpus"], "frac", r["frac"], "launch_ms", r["avg_launch_ms"],
      "exec_frac", r["executed_fraction"], "check", {k: p.get(k) for k in ("frames", "bit_exact", "seconds", "skipped")},
      "cpu", (d.get("cpu_baseline") or {}).get("value"), (d.get("cpu_baseline_threads") or {}).get("value"),
      (d.get("cpu_baseline_node") or {}).get("value"))
PY
}
on bench && bench c3 --steps 20 --warmup 5
on lanes && bench lanes4 --steps 40 --warmup 5 --streams 1 --lanes 4 --no-cpu
on c5 && bench c5 --config c5 --steps 10 --warmup 2 --no-cpu
on video && bench video1 --gpus 1 --video-frames 10000 --steps 3 --warmup 2 --no-cpu
on video && bench video4 --gpus 4 --oversubscribe --video-frames 10000 --steps 3 --warmup 2 --no-cpu
if on refuse; then
  timeout -k 10 240 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > $O/refuse.out 2> $O/refuse.err
  rc=$?
  echo "bench --gpus 2 on this box: rc=$rc (must be non-zero), stdout lines: $(wc -l < $O/refuse.out)"; tail -2 $O/refuse.err
  [ $rc -ne 0 ] || exit 1
fi
echo done
