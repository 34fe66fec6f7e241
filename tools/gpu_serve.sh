# The resident begin/commit server on the GPU box: its parity tests, then the
# drop-in latency from C with the server and with kernels launched per call.
# usage: tools/gpu_serve.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_gpu_serve.py > gpurun_out/${TAG}_serve_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_serve_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_serve_tests.log
: > gpurun_out/${TAG}_dropin.jsonl
for wf in 0 1; do
  timeout -k 10 120 tools/bin/dropin_latency 5000 4000 200 $wf >> gpurun_out/${TAG}_dropin.jsonl || exit 1
  KSG_SERVE=0 timeout -k 10 120 tools/bin/dropin_latency 5000 4000 200 $wf >> gpurun_out/${TAG}_dropin.jsonl || exit 1
done
timeout -k 10 120 tools/bin/dropin_latency 15000 2000 200 1 >> gpurun_out/${TAG}_dropin.jsonl || exit 1
timeout -k 10 120 tools/bin/dropin_latency 500 4000 200 1 >> gpurun_out/${TAG}_dropin.jsonl || exit 1
cat gpurun_out/${TAG}_dropin.jsonl
