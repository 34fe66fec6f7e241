# Round-4: phase A int32 scores / zero-count divide skip: full GPU suite, bench lines (config 2
# with stages, config 5, extensions with stages), then the resolver's instruction-cache counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4m}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --workload config5 > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err || { tail gpurun_out/${TAG}_bench_config5.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --extensions > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","config5","c2_ext"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    fs=d.get("filter_score") or {}
    print(w, round(d["value"]), round((d.get("latency") or {}).get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"],3), d["config"]["snapshots_in_timed"], "phaseA_us", round(fs.get("ms_avg",0)*1e3,2))
    st=(d.get("latency") or {}).get("stages")
    if st: print(json.dumps(st))
PY
bash tools/gpu_r4_icache.sh || exit 1
