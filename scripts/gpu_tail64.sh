cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/t64
for i in 1 2 3 4; do
timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/t64/n_$i.log 2>&1; echo "ns4 tail<64KB: rc=$? $(tail -1 gpurun_out/t64/n_$i.log)"; grep -m1 "mt:" gpurun_out/t64/n_$i.log | cut -c1-200
done
