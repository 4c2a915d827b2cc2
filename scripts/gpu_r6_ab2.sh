set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_kernel_resources.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/gpu_tests_s2.log 2>&1
rc=$?; tail -3 gpurun_out/r6/gpu_tests_s2.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r6/gpu_tests_s2.log | head -20; exit $rc; }
TAG=s2 REPS=2 VARIANTS="base:base: r5:r5: m4p1:m4:LM_CORR_PLAN=1 basep1:base:LM_CORR_PLAN=1 x32:x32: x64:x64:" bash scripts/gpu_ab_combo.sh
