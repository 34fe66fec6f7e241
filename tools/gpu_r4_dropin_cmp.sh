# Round-4: drop-in latency of the previous round's library (tools/bin/lib_f29f29f) against this
# build's at 15k and 100k nodes, back to back on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for n in 15000 100000; do
  timeout -k 10 180 tools/bin/lib_f29f29f/dropin_latency $n 3000 200 >> gpurun_out/r4_dropin_cmp_old.jsonl || exit 1
  timeout -k 10 180 tools/bin/dropin_latency $n 3000 200 >> gpurun_out/r4_dropin_cmp_new.jsonl || exit 1
done
python - <<'PY'
import json
for k in ("old","new"):
    for l in open(f"gpurun_out/r4_dropin_cmp_{k}.jsonl"):
        d=json.loads(l); print(k, d["nodes"], d["us_p50"], d["us_p99"], round(d["pods_per_s"]), d["begin_us_p50"], d.get("commit_us_p50"))
PY
