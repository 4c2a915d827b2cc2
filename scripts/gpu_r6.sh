#!/bin/bash
# Round-6 GPU check in one call: GPU tests, smoke, bench lines with their
# oracle checks (the driver's C3 command and the bare default, the drop-in 1
# context x 4 lanes, C5 fp32), the C4 strong-scaling mode at bench.py's
# default shapes (the whole video on one GPU and over 4 oversubscribed ranks,
# one 1,250-frame shard), the host-frame (H2D) path, the launcher's refusal of
# --gpus 2 on a one-GPU box, the rocprof kernel trace and the PMC traffic
# passes of the default line.
# STEPS=tests,smoke,bench,default,lanes,c5,c5f16,video,shard,host,refuse,prof,traffic
# selects steps (default: all but kprof).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r6final}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
S=",${STEPS:-tests,smoke,bench,default,lanes,c5,c5f16,video,shard,host,refuse,prof,traffic},"
# kprof: phase cycles of k_nms / k_tail / k_post (LM_KPROF=1, one stream)
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
print(sys.argv[1].split("/")[-1], d["value"], d["unit"], "ms/step", d["ms_per_step"], "n_gpus", d["n_gpus"], "frac", r["frac"], "launch_ms", r["avg_launch_ms"],
      "exec_frac", r["executed_fraction"], "check", {k: p.get(k) for k in ("frames", "bit_exact", "seconds", "skipped")},
      "cpu", (d.get("cpu_baseline") or {}).get("value"), (d.get("cpu_baseline_threads") or {}).get("value"),
      (d.get("cpu_baseline_node") or {}).get("value"))
PY
}
on bench && bench c3 --gpus 1 --steps 20 --warmup 5
on default && bench default
on lanes && bench lanes4 --steps 40 --warmup 5 --streams 1 --lanes 4 --no-cpu
on c5 && bench c5 --config c5 --steps 10 --warmup 2 --no-cpu
# C5 in the non-parity f16 mode: 8 contexts (its longer correlation launches need more streams to fill each other's tails)
on c5f16 && bench c5f16 --config c5 --precision f16 --streams 8 --steps 12 --warmup 2 --no-cpu
on video && bench video1 --gpus 1 --video-frames 10000 --steps 3 --warmup 2 --no-cpu
on video && bench video4 --gpus 4 --oversubscribe --video-frames 10000 --steps 3 --warmup 2 --no-cpu
# one rank's C4 shard alone (1,250 frames) at the default shape (1 context x 4 lanes x 209)
on shard && bench shard --video-frames 1250 --steps 10 --warmup 3 --no-cpu
# frames in pinned host memory, H2D inside the timed loop
on host && bench host4 --host-frames --steps 20 --warmup 3 --no-cpu
on host && bench host_lanes --host-frames --streams 2 --lanes 4 --steps 20 --warmup 3 --no-cpu
if on refuse; then
  timeout -k 10 240 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > $O/refuse.out 2> $O/refuse.err
  rc=$?
  echo "bench --gpus 2 on this box: rc=$rc (must be non-zero), stdout lines: $(wc -l < $O/refuse.out)"; tail -2 $O/refuse.err
  [ $rc -ne 0 ] || exit 1
fi
if on kprof; then
  LM_KPROF=1 timeout -k 10 240 python bench.py --streams 1 --steps 3 --warmup 1 --no-cpu --no-check > $O/kprof.json 2> $O/kprof.txt || { tail -5 $O/kprof.txt; exit 1; }
  grep "kprof k_nms" $O/kprof.txt | tail -2
fi
# prof: rocprofv3 kernel trace + stats of the driver's bench command (no CPU
# legs), and the union of the correlation dispatches' spans
if on prof; then
  rm -rf $O/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-check > $O/prof.out 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.out; exit 1; }
  python3 scripts/prof_union.py $O/prof/run_kernel_trace.csv 4 40 > $O/prof_union.txt && tail -4 $O/prof_union.txt
fi
# traffic: FETCH_SIZE and WRITE_SIZE of the correlation, one --pmc pass each
# -> $O/pmc_k_corr.json (copied to profiles/r06/ for bench.py's traffic)
if on traffic; then
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmc/$c
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -f csv -d $O/pmc/$c -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-check > $O/pmc_$c.out 2>&1 || { echo "pmc $c failed"; tail -5 $O/pmc_$c.out; exit 1; }
  done
  python3 scripts/pmc_traffic.py $O/pmc 448 $O/pmc_k_corr.json > $O/pmc_traffic.txt && tail -3 $O/pmc_traffic.txt
fi
echo done
