# Timing experiments on the plain resolver (KSG_DEBUG bits 24..27 make decisions WRONG; timing
# only): which role bounds the per-pod chain at a workload. One bench line per switch set.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4x}
WL=${2:-config2}
for x in ${XS:-0 1 2 3 4 7 8 15}; do
  KSG_DEBUG=$((x << 24)) timeout -k 10 120 python bench.py --workload $WL --no-cpu-baseline --no-stages > gpurun_out/${TAG}_${WL}_x$x.json 2> gpurun_out/${TAG}_${WL}_x$x.err || { tail gpurun_out/${TAG}_${WL}_x$x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_${WL}_x$x.json').read().strip().splitlines()[-1]); print('x=$x', round(d['value']), round(d['latency']['resolver_cycles_per_pod']), d['config']['snapshots_in_timed'])"
done
