cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/hog2
for k in k_tail k_nms k_post k_corr; do
for i in 1 2 3; do
LM_LDS_HOG=$k timeout -k 10 300 python -u scripts/debug_mt.py 4 20 0 > gpurun_out/hog2/${k}_$i.log 2>&1; echo "ns4 hog $k: rc=$? $(tail -1 gpurun_out/hog2/${k}_$i.log)"
done; done
