# the whole GPU suite (run on the GPU box), log under gpurun_out/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ "$@" > gpurun_out/gpu_full.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_full.log
exit $rc
