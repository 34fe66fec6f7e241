# Round-4 record run (on the GPU box): the -m gpu suite, smoke(), the default bench line (config 2
# with its CPU baseline and stage breakdown), configs 1 / 3 / 4 / 5 and config 2 + extensions.
# usage: tools/gpu_r4.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
for w in config1 config3 config4 config5; do
  timeout -k 10 300 python bench.py --workload $w --no-stages > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail gpurun_out/${TAG}_bench_$w.err; exit 1; }
done
timeout -k 10 300 python bench.py --extensions > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","config1","config3","config4","config5","c2_ext"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    fs=d.get("filter_score") or {}
    cb=d.get("cpu_baseline") or {}
    print(w, round(d["value"]), round((d.get("latency") or {}).get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"],3),
          d["config"]["snapshots_in_timed"], "phaseA_us", round(fs.get("ms_avg",0)*1e3,2), "cpu", cb.get("value"))
    st=(d.get("latency") or {}).get("stages")
    if st and w in ("default","c2_ext"): print(json.dumps(st))
PY
