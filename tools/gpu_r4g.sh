# Round-4: flagger wave + pre-verdicts (parity, fuzz interleavings, extensions, servers), bench
# lines (config 2 with the stage breakdown, extensions, configs 3/5), drop-in 5k / 15k old vs new.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4g}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_extensions.py tests/test_gpu_serve.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --extensions --no-stages > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
for w in config3 config5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --workload $w > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail gpurun_out/${TAG}_bench_$w.err; exit 1; }
done
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","c2_ext","config3","config5"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    mt = (cb.get("incremental_nproc") or {})
    print(w, round(d["value"]), round((d.get("latency") or {}).get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"],3), d["config"]["snapshots_in_timed"], mt.get("whole_run_checked"))
d=json.loads(open(f"gpurun_out/{t}_bench_default.json").read().strip().splitlines()[-1])
print(json.dumps(d["latency"].get("stages")))
PY
for n in 5000 15000; do
  timeout -k 10 120 tools/bin/lib_f29f29f/dropin_latency $n 2000 200 >> gpurun_out/${TAG}_dropin_old.jsonl || exit 1
  timeout -k 10 120 tools/bin/dropin_latency $n 2000 200 >> gpurun_out/${TAG}_dropin_new.jsonl || exit 1
done
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for k in ("old","new"):
    for l in open(f"gpurun_out/{t}_dropin_{k}.jsonl"):
        d=json.loads(l); print(k, d["nodes"], d["us_p50"], d["us_p99"], round(d["pods_per_s"]), d["begin_us_p50"])
PY
