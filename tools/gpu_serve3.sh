# server tests, then drop-in latency: grid server vs one-workgroup server
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
KSG_SERVE_DEBUG=1 timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_gpu_serve.py > gpurun_out/${TAG}_serve_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_serve_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/${TAG}_serve_tests.log
: > gpurun_out/${TAG}_dropin.jsonl
for n in 2000 5000 15000; do
  for g in 1 0; do
    KSG_SERVE_GRID=$g timeout -k 10 120 tools/bin/dropin_latency $n 3000 200 0 >> gpurun_out/${TAG}_dropin.jsonl || exit 1
  done
done
KSG_SERVE_GRID=1 timeout -k 10 120 tools/bin/dropin_latency 5000 3000 200 1 >> gpurun_out/${TAG}_dropin.jsonl || exit 1
KSG_SERVE_GRID=1 timeout -k 10 120 tools/bin/dropin_latency 50000 2000 200 0 >> gpurun_out/${TAG}_dropin.jsonl || exit 1
python - "$TAG" <<'PY'
import json, sys
for l in open(f"gpurun_out/{sys.argv[1]}_dropin.jsonl"):
    d = json.loads(l); print(d["nodes"], d["served"], d["want_fail"], d["us_p50"], d["us_p99"], d["begin_us_p50"], d["commit_us_p50"], round(d["pods_per_s"]))
PY
