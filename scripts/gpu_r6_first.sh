set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=r6a STEPS=tests,smoke,bench bash scripts/gpu_r5.sh || exit 1
REPS=2 bash scripts/gpu_ab_lib.sh
