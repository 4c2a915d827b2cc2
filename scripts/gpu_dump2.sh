cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dump2
export LM_CONCURRENT=1 LM_DUMP_DIR=gpurun_out/dump2
for i in 1 2 3; do
timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/dump2/mt_$i.log 2>&1; echo "run $i: $(tail -1 gpurun_out/dump2/mt_$i.log)"; grep -m2 "checkVel" gpurun_out/dump2/mt_$i.log | cut -c1-250
n=$(ls gpurun_out/dump2/*.bin 2>/dev/null | wc -l); [ $n -ge 2 ] && break
done
ls -la gpurun_out/dump2
