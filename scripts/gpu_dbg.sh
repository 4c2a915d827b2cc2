set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dbg
LIB=locomouse_cpp_amd/liblocomouse_hip.so
cp $LIB gpurun_out/dbg/orig.so
for v in base cap1024 cap2048; do
  [ $v = base ] || cp locomouse_cpp_amd/exp/liblocomouse_hip_$v.so $LIB
  timeout -k 10 300 python -m pytest -q -x -p no:cacheprovider tests/test_gpu_parity.py::test_long_stream_device_frames tests/test_gpu_multictx.py > gpurun_out/dbg/$v.txt 2>&1
  echo "$v rc=$?"; tail -2 gpurun_out/dbg/$v.txt
  cp gpurun_out/dbg/orig.so $LIB
done
