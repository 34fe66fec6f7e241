# Stage breakdowns (KSG_DEBUG=8 second run) of config 2 under KSG_DEBUG values given as
# name=value pairs (timing switches 24..27 make decisions WRONG: timing only).
# usage: tools/gpu_r4_stages.sh <tag> name=dbg ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
for nv in "$@"; do
  n=${nv%%=*}; v=${nv#*=}
  KSG_DEBUG=$v timeout -k 10 200 python bench.py --no-cpu-baseline --workload ${WL:-config2} > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { tail gpurun_out/${TAG}_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_$n.json').read().strip().splitlines()[-1]); st=d['latency'].get('stages') or {}; print('$n', round(d['value']), round(d['latency']['resolver_cycles_per_pod']), d['config']['snapshots_in_timed']); print(json.dumps(st))"
done
