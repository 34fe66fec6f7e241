# Round-4: extension scores (histogram normalisation), bench lines, and the drop-in per-pod
# latency of the final build against the round-3 15:00 build (tools/bin/lib_f29f29f,
# f29f29f), alternating, plus 15k / 100k nodes and config 4's shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_extensions.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_ext_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_ext_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_ext_tests.log
timeout -k 10 300 python bench.py --extensions --no-stages > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_c2_ext.json').read().strip().splitlines()[-1]); print('c2_ext', round(d['value']), round(d['latency']['resolver_cycles_per_pod']), d['config']['snapshots_in_timed'], d['cpu_baseline']['incremental_nproc']['whole_run_checked'])"
for r in 1 2; do
  timeout -k 10 120 tools/bin/lib_f29f29f/dropin_latency 5000 2000 200 >> gpurun_out/${TAG}_dropin_old.jsonl || exit 1
  timeout -k 10 120 tools/bin/dropin_latency 5000 2000 200 >> gpurun_out/${TAG}_dropin_new.jsonl || exit 1
done
for n in 15000 100000; do
  timeout -k 10 120 tools/bin/lib_f29f29f/dropin_latency $n 2000 200 >> gpurun_out/${TAG}_dropin_old.jsonl || exit 1
  timeout -k 10 120 tools/bin/dropin_latency $n 2000 200 >> gpurun_out/${TAG}_dropin_new.jsonl || exit 1
done
timeout -k 10 120 tools/bin/dropin_latency 5000 2000 200 0 0 1 >> gpurun_out/${TAG}_dropin_new.jsonl || exit 1
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for k in ("old","new"):
    for l in open(f"gpurun_out/{t}_dropin_{k}.jsonl"):
        d=json.loads(l); print(k, d["nodes"], d.get("policy",0), d["us_p50"], d["us_p99"], round(d["pods_per_s"]), d["begin_us_p50"], d["commit_us_p50"], d["served"])
PY
