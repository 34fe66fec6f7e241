# Round-4 pass: the resident-server and extension GPU tests (ADVICE r3 fixes, config 5 with
# extended resources at full size), then the default bench line and the config-5 extension line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_serve.py tests/test_gpu_extensions.py tests/test_gpu_scheduler_api.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --workload config5 --extensions --ext-filters-only --no-stages > gpurun_out/${TAG}_bench_c5_extf.json 2> gpurun_out/${TAG}_bench_c5_extf.err || { tail gpurun_out/${TAG}_bench_c5_extf.err; exit 1; }
for w in config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --workload $w > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail gpurun_out/${TAG}_bench_$w.err; exit 1; }
done
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","c5_extf","config4","config5"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    mt = (cb.get("incremental_nproc") or {})
    print(w, round(d["value"]), (d.get("latency") or {}).get("resolver_cycles_per_pod"), d["ms_per_step"], d["roofline"]["frac"], mt.get("whole_run_checked"), mt.get("decisions_identical"))
PY
