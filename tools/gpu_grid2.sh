# Grid drop-in server at 1 and 4 nodes per thread: serve tests, then per-pod latency from C.
# usage: tools/gpu_grid2.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
KSG_SERVE_DEBUG=1 timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_serve.py > gpurun_out/${TAG}_serve_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_serve_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/${TAG}_serve_tests.log
OUT=gpurun_out/${TAG}_dropin.jsonl
: > $OUT
for cfg in "5000 0" "5000 1" "15000 0" "15000 1" "30000 0" "50000 0" "100000 0"; do
  set -- $cfg
  if [ "$2" = 1 ]; then export KSG_SERVE_GRID_NPT4_MIN=0; else unset KSG_SERVE_GRID_NPT4_MIN; fi
  timeout -k 10 120 tools/bin/dropin_latency $1 1500 150 0 >> $OUT || exit 1
done
unset KSG_SERVE_GRID_NPT4_MIN
python - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["nodes"], d["served"], d["us_p50"], d["us_p99"], d["begin_us_p50"], d["commit_us_p50"], round(d["pods_per_s"]))
PY
