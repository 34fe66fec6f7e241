# A/B experiment: bench lines for the given workloads with and without extra env (run on the GPU box)
# usage: tools/gpu_exp.sh <tag> "<ENV=..>" workload...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
ENVS=$1; shift
for w in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --workload $w > gpurun_out/${TAG}_${w}_a.json 2> gpurun_out/${TAG}_${w}_a.err || exit 1
  env $ENVS timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --workload $w > gpurun_out/${TAG}_${w}_b.json 2> gpurun_out/${TAG}_${w}_b.err || exit 1
  python - "$TAG" "$w" <<'PY'
import json,sys
t,w=sys.argv[1:]
for s in "ab":
    d=json.loads(open(f"gpurun_out/{t}_{w}_{s}.json").read().strip().splitlines()[-1])
    print(w, s, round(d["value"]), d["latency"]["resolver_cycles_per_pod"], d["ms_per_step"])
PY
done
