# Drop-in per-pod latency from C (ksg_schedule_begin + ksg_schedule_commit) for the given
# tools/bin/dropin_latency argument sets ("nodes pods warmup want_fail ext policy"), one JSON line
# each into gpurun_out/<tag>_dropin.jsonl. usage: tools/gpu_dropin.sh <tag> "<args>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/${TAG}_dropin.jsonl
: > $OUT
for args in "$@"; do
  timeout -k 10 180 tools/bin/dropin_latency $args >> $OUT || exit 1
done
python - "$OUT" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["nodes"], "policy", d.get("policy",0), "ext", d.get("ext",0), "p50", d["us_p50"], "p99", d["us_p99"], round(d["pods_per_s"]), (d.get("served") or {}).get("eligible"))
PY
