# Round-5 A/B: the default bench (config 2, no CPU baseline) under each ENV=value setting given,
# printing value, resolver cycles/pod and the stage breakdown of each.
# usage: tools/gpu_r5_ab.sh <tag> name:VAR=val[,VAR=val] ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for spec in "$@"; do
  n=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do export "$kv"; done
    timeout -k 10 240 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err ) || { tail gpurun_out/${TAG}_$n.err; exit 1; }
  python - "$TAG" "$n" <<'PY'
import json,sys
t,n=sys.argv[1],sys.argv[2]
d=json.loads(open(f"gpurun_out/{t}_{n}.json").read().strip().splitlines()[-1])
lat=d.get("latency") or {}
print("==", n, round(d["value"]), round(lat.get("resolver_cycles_per_pod") or 0))
st=lat.get("stages") or {}
for k,v in st.items():
    if isinstance(v, dict): print("  ", k, json.dumps(v))
PY
done
