# Round-4: extension scores with prefetched inputs; drop-in at 5k / 15k nodes after the applied revert.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_extensions.py tests/test_gpu_serve.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --extensions --no-stages > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_c2_ext.json').read().strip().splitlines()[-1]); print('c2_ext', round(d['value']), round(d['latency']['resolver_cycles_per_pod']), d['config']['snapshots_in_timed'], d['cpu_baseline']['incremental_nproc']['whole_run_checked'])"
for n in 5000 15000; do
  timeout -k 10 120 tools/bin/lib_f29f29f/dropin_latency $n 2000 200 >> gpurun_out/${TAG}_dropin_old.jsonl || exit 1
  timeout -k 10 120 tools/bin/dropin_latency $n 2000 200 >> gpurun_out/${TAG}_dropin_new.jsonl || exit 1
done
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for k in ("old","new"):
    for l in open(f"gpurun_out/{t}_dropin_{k}.jsonl"):
        d=json.loads(l); print(k, d["nodes"], d.get("policy",0), d["us_p50"], d["us_p99"], round(d["pods_per_s"]), d["begin_us_p50"], d["commit_us_p50"])
PY
