# extensions on the window path: parity (extensions, plain-resolver families), then bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_extensions.py tests/test_gpu_parity.py -k "not full_size and not config5_full and not faithful" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --extensions --ext-filters-only > gpurun_out/${TAG}_bench_c2_extf.json 2> gpurun_out/${TAG}_bench_c2_extf.err || { tail gpurun_out/${TAG}_bench_c2_extf.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-stages --extensions --ext-filters-only --workload config5 > gpurun_out/${TAG}_bench_c5_extf.json 2> gpurun_out/${TAG}_bench_c5_extf.err || { tail gpurun_out/${TAG}_bench_c5_extf.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("c2_extf","c5_extf"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    print(w, round(d["value"]), d["ms_per_step"], d["config"]["snapshots_in_timed"], d["config"]["placed_in_timed"], d["config"]["fit_errors_in_timed"])
PY
