# Round-4: validate the extension re-score changes (full -m gpu suite), bench lines (config 2 and
# config 2 + extensions, with stages), the final drop-in records, config-2 profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4o}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail gpurun_out/${TAG}_bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --extensions > gpurun_out/${TAG}_bench_c2_ext.json 2> gpurun_out/${TAG}_bench_c2_ext.err || { tail gpurun_out/${TAG}_bench_c2_ext.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
for w in ("default","c2_ext"):
    d=json.loads(open(f"gpurun_out/{t}_bench_{w}.json").read().strip().splitlines()[-1])
    print(w, round(d["value"]), round((d.get("latency") or {}).get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"],3), d["config"]["snapshots_in_timed"])
    print(json.dumps((d.get("latency") or {}).get("stages")))
PY
bash tools/gpu_r4_dropin.sh r4 || exit 1
bash tools/gpu_r4_pmc.sh r4_c2 --workload config2 --steps 4 --warmup 1 || exit 1
