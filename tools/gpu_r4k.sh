# Round-4: checker slot rows in registers (stride-36 table): parity + fuzz, then config 2 (stages),
# configs 3/4/5 and extensions bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4k}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
for w in config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --workload $w > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail gpurun_out/${TAG}_bench_$w.err; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline --extensions > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","config3","config4","config5","c2_ext"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    print(w, round(d["value"]), round((d.get("latency") or {}).get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"],3), d["config"]["snapshots_in_timed"])
for w in ("default","c2_ext"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    print(w, json.dumps(d["latency"].get("stages")))
PY
