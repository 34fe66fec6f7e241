# Round-5 phase-A A/B: bench.py (no CPU baseline, no stages) per library variant on one
# workload, printing pods/s, phase A's mean launch time and the resolver's cycles per pod.
# usage: tools/gpu_r5_pa.sh <tag> <workload> name:KSG_LIB_value ...   ("main" = the in-tree build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; WL=$2; shift 2
for spec in "$@"; do
  n=${spec%%:*}; lib=${spec#*:}
  ( [ "$lib" != "main" ] && export KSG_LIB=$lib
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-stages --workload $WL ${BENCH_ARGS} \
      > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err ) || { tail gpurun_out/${TAG}_$n.err; exit 1; }
  python - "$TAG" "$n" <<'PY'
import json,sys
t,n=sys.argv[1],sys.argv[2]
d=json.loads(open(f"gpurun_out/{t}_{n}.json").read().strip().splitlines()[-1])
fs=d.get("filter_score") or {}
lat=d.get("latency") or {}
print("==", n, d["config"]["workload"], round(d["value"]), "phaseA_us", round(1e3*(fs.get("ms_avg") or 0), 2),
      "res_cyc", round(lat.get("resolver_cycles_per_pod") or 0), "ms/step", round(d["ms_per_step"], 3))
PY
done
