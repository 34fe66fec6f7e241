# server parity tests, then per-stage stamps and latency at 500 / 5000 / 15000 nodes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_serve.py > gpurun_out/${TAG}_serve_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_serve_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_serve_tests.log
: > gpurun_out/${TAG}_stamps.txt
for n in 500 5000 15000; do
  for wf in 0 1; do
    KSG_SERVE_STAMPS=1 timeout -k 10 120 tools/bin/dropin_latency $n 2000 200 $wf >> gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
  done
done
python - "$TAG" <<'PY'
import json, sys
for l in open(f"gpurun_out/{sys.argv[1]}_stamps.txt"):
    if l.startswith("{"):
        d = json.loads(l); print(d["nodes"], d["want_fail"], d["us_p50"], d["begin_us_p50"], d["commit_us_p50"], round(d["pods_per_s"]))
    else:
        print(l.strip()[:200])
PY
