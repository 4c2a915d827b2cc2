# Multi-context stress: 3-4 contexts in threads on one GPU, every batch
# compared with single-context runs (the configuration that exposed the
# k_nms tie-path race).  Failing slots are dumped.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/flat
export LM_DUMP_DIR=gpurun_out/flat
for i in 1 2 3 4; do
timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/flat/mt4_$i.log 2>&1; echo "ns4 concurrent: rc=$? $(tail -1 gpurun_out/flat/mt4_$i.log)"
done
for i in 1 2; do
timeout -k 10 300 python -u scripts/debug_mt.py 3 23 0 > gpurun_out/flat/ns3_$i.log 2>&1; echo "ns3 concurrent: rc=$? $(tail -1 gpurun_out/flat/ns3_$i.log)"
done
