# Quick check on the GPU box: selected -m gpu tests (pytest -k expression in $K, files
# in $FILES), then the default bench (config 2 unless BENCH_ARGS) under each ENV spec given.
# usage: K='expr' FILES='tests/x.py ...' tools/gpu_quick.sh <tag> [name:VAR=val[,VAR=val] ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6q}; shift
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${FILES:-tests} -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
for spec in "$@"; do
  n=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
    timeout -k 10 240 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err ) || { tail gpurun_out/${TAG}_$n.err; exit 1; }
  python - "$TAG" "$n" <<'PY'
import json,sys
t,n=sys.argv[1],sys.argv[2]
d=json.loads(open(f"gpurun_out/{t}_{n}.json").read().strip().splitlines()[-1])
lat=d.get("latency") or {}
rf=d.get("roofline") or {}
print("==", n, d["config"]["workload"], round(d["value"]), "ms/step", round(d["ms_per_step"],3), "dev", round(d.get("device_ms_per_step") or 0,3),
      "res_cyc", round(lat.get("resolver_cycles_per_pod") or 0), "kms", round((rf.get("kernel_ms_avg") or 0)*1e3,1),
      "eval", round((rf.get("win_eval_ms_avg") or 0)*1e3,1), "t0", round((rf.get("win_t0_ms_avg") or 0)*1e3,1),
      "launches", rf.get("launches"), "snap", json.dumps(d["config"].get("snapshots_in_timed")))
st=lat.get("stages") or {}
for k,v in st.items():
    if isinstance(v, dict): print("  ", k, json.dumps(v))
PY
done
