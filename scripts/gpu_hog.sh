cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/hog
for i in 1 2 3; do
LM_LDS_HOG=1 timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/hog/h_$i.log 2>&1; echo "ns4 lds hog: rc=$? $(tail -1 gpurun_out/hog/h_$i.log)"
timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/hog/n_$i.log 2>&1; echo "ns4 default: rc=$? $(tail -1 gpurun_out/hog/n_$i.log)"
done
