# GPU test suite only (run on the GPU box); log under gpurun_out/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
