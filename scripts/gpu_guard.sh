cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
LM_CORR_VARIANT=8 timeout -k 10 300 python -u scripts/debug_mt.py 2 23 0 > gpurun_out/g1.log 2>&1; echo "v8 ns2 plain: rc=$? $(tail -1 gpurun_out/g1.log)"; grep -m3 "stream" gpurun_out/g1.log | cut -c1-300
LM_GUARD=1 LM_CORR_VARIANT=8 timeout -k 10 300 python -u scripts/debug_mt.py 2 23 0 > gpurun_out/g2.log 2>&1; echo "v8 ns2 guard: rc=$? $(tail -1 gpurun_out/g2.log)"; grep -m3 "stream" gpurun_out/g2.log | cut -c1-300
LM_GUARD=1 LM_ALLOW_QUEUE_SHARING=1 LM_CORR_VARIANT=3 timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/g3.log 2>&1; echo "v3 ns3 guard: rc=$? $(tail -1 gpurun_out/g3.log)"; grep -m3 "stream" gpurun_out/g3.log | cut -c1-300
LM_CORR_VARIANT=8 timeout -k 10 300 python -u scripts/debug_stream.py 6400 23 256 --check > gpurun_out/g4.log 2>&1; echo "v8 single ctx vs oracle: rc=$? $(tail -1 gpurun_out/g4.log)"
