# Round-5: one bench line (args in $BENCH_ARGS, default config 2 with stages, no CPU baseline)
# and its stage breakdown. usage: tools/gpu_r5_bench.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r5x}
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
d=json.loads(open(f"gpurun_out/{t}_bench.json").read().strip().splitlines()[-1])
lat=d.get("latency") or {}
print(d["config"]["workload"], round(d["value"]), round(lat.get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"],3))
st=lat.get("stages")
if st:
    for k,v in st.items(): print(k, json.dumps(v))
PY
