# Round-5 quick check on the GPU box: selected -m gpu tests (pytest -k expression in $K),
# then the default bench line (config 2, stages) unless NOBENCH is set.
# usage: K='expr' tools/gpu_r5_quick.sh <tag> [test files...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r5q}; shift
FILES=${@:-tests}
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
python - "$TAG" <<'PY'
import json,sys
t=sys.argv[1]
d=json.loads(open(f"gpurun_out/{t}_bench.json").read().strip().splitlines()[-1])
lat=d.get("latency") or {}
print(d["config"]["workload"], round(d["value"]), round(lat.get("resolver_cycles_per_pod") or 0), round(d["ms_per_step"],3))
st=lat.get("stages")
if st: print(json.dumps(st))
PY
