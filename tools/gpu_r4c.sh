# Round-4 pass: the whole -m gpu suite, smoke(), the default bench line and the config-5
# extension line, config 4 / 5 lines, then the resolver timing experiments at config 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --workload config5 --extensions --ext-filters-only --no-stages > gpurun_out/${TAG}_bench_c5_extf.json 2> gpurun_out/${TAG}_bench_c5_extf.err || { tail gpurun_out/${TAG}_bench_c5_extf.err; exit 1; }
for w in config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --workload $w > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail gpurun_out/${TAG}_bench_$w.err; exit 1; }
done
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","c5_extf","config3","config4","config5"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    mt = (cb.get("incremental_nproc") or {})
    print(w, round(d["value"]), (d.get("latency") or {}).get("resolver_cycles_per_pod"), round(d["ms_per_step"],3), round(d["roofline"]["frac"],4), mt.get("whole_run_checked"), mt.get("decisions_identical"))
PY
bash tools/gpu_r4_exp.sh ${TAG}x config2
