# Round-4 final build: drop-in per-pod latency from C (ksg_schedule_begin + ksg_schedule_commit)
# at 5k / 15k / 100k nodes (config 2's shape), config 4's policy at 900 and 5,000 nodes, and
# the extensions shape; one JSON line each into profiles/<tag>_dropin.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4}
OUT=gpurun_out/${TAG}_dropin.jsonl
: > $OUT
for n in 5000 15000 100000; do
  timeout -k 10 180 tools/bin/dropin_latency $n 4000 200 >> $OUT || exit 1
done
timeout -k 10 120 tools/bin/dropin_latency 900 4000 200 0 0 1 >> $OUT || exit 1
timeout -k 10 120 tools/bin/dropin_latency 5000 4000 200 0 0 1 >> $OUT || exit 1
timeout -k 10 120 tools/bin/dropin_latency 5000 4000 200 0 2 0 >> $OUT || exit 1
python - "$OUT" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["nodes"], d.get("policy",0), d.get("ext",0), d["us_p50"], d["us_p99"], round(d["pods_per_s"]), d.get("served"))
PY
