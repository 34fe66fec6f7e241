# Round-4: extension scores on the window path (GPU parity), the plain resolver after the
# pre-verdict revert, bench lines (default, extensions with scores, config 5).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_extensions.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_ext_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_ext_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_ext_tests.log
timeout -k 10 300 python bench.py --no-stages > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --extensions --no-stages > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --workload config5 --no-stages > gpurun_out/${TAG}_bench_config5.json 2> gpurun_out/${TAG}_bench_config5.err || { tail gpurun_out/${TAG}_bench_config5.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","c2_ext","config5"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    mt = (cb.get("incremental_nproc") or {})
    print(w, round(d["value"]), (d.get("latency") or {}).get("resolver_cycles_per_pod"), round(d["ms_per_step"],3), d["config"]["snapshots_in_timed"], mt.get("whole_run_checked"), mt.get("decisions_identical"))
PY
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
