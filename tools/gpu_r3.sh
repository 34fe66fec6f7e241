# Round-3 GPU pass: the -m gpu suite, smoke(), the default bench line, then bench lines for the
# other configs (no CPU baseline). Logs and JSON lines under gpurun_out/r3_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
for w in config1 config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --workload $w > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail gpurun_out/${TAG}_bench_$w.err; exit 1; }
done
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","config1","config3","config4","config5"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    print(w, round(d["value"]), d["latency"].get("resolver_cycles_per_pod"), d["ms_per_step"], d.get("device_ms_per_step"), d["roofline"]["frac"])
PY
