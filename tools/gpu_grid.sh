# Grid drop-in server: polling options and per-stage stamps (KSG_SERVE_STAMPS=1) from C.
# usage: tools/gpu_grid.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
KSG_SERVE_DEBUG=1 timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_serve.py > gpurun_out/${TAG}_serve_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_serve_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/${TAG}_serve_tests.log
OUT=gpurun_out/${TAG}_grid.txt
: > $OUT
for n in 2000 5000 15000 50000; do
  echo "nodes $n" >> $OUT
  KSG_SERVE_STAMPS=1 timeout -k 10 120 tools/bin/dropin_latency $n 2000 200 0 >> $OUT 2>&1 || exit 1
done
echo "nodes 5000 with fail codes" >> $OUT
KSG_SERVE_STAMPS=1 timeout -k 10 120 tools/bin/dropin_latency 5000 2000 200 1 >> $OUT 2>&1 || exit 1
echo "single 5000" >> $OUT
KSG_SERVE_STAMPS=1 KSG_SERVE_GRID=0 timeout -k 10 120 tools/bin/dropin_latency 5000 2000 200 0 >> $OUT 2>&1 || exit 1
python - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l); print(" ", d["nodes"], d["us_p50"], d["us_p99"], d["begin_us_p50"], d["commit_us_p50"], round(d["pods_per_s"]))
    else:
        print(l)
PY
