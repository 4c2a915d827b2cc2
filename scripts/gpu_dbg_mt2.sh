cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { # tag ns dbg
  timeout -k 10 200 python -u scripts/debug_mt.py $2 23 $3 > gpurun_out/mt_$1.log 2>&1; rc=$?
  echo "$1: $(tail -1 gpurun_out/mt_$1.log)"; [ $rc -le 1 ] || exit $rc
}
for i in 1 2 3; do run q4_ns2_$i 2 0; done
for i in 1 2 3; do run q4_ns3_$i 3 0; done
export GPU_MAX_HW_QUEUES=8
for i in 1 2 3; do run q8_ns3_$i 3 0; done
for i in 1 2; do run q8_ns4_$i 4 0; done
