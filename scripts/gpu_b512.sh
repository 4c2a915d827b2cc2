cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/b512
for i in 1 2; do
timeout -k 10 400 python -u tests/tools/debug_stream.py 0 12 512 --check > gpurun_out/b512/r$i.log 2>&1; echo "b512 run $i: rc=$? $(tail -1 gpurun_out/b512/r$i.log)"; grep -v amdgpu gpurun_out/b512/r$i.log | grep -m4 "error\|differs\|fails\|oracle" | cut -c1-300
done
timeout -k 10 400 python -u tests/tools/debug_stream.py 4608 2 256 --check > gpurun_out/b512/r256.log 2>&1; echo "b256 same frames: rc=$? $(tail -1 gpurun_out/b512/r256.log)"; grep -v amdgpu gpurun_out/b512/r256.log | grep -m4 "error\|differs\|fails" | cut -c1-300
