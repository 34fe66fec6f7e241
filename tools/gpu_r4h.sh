# Round-4: pre-verdicts on / off (KSG_DEBUG bit 28) under the flagger wave, with the stage
# breakdown, and the timing switches (bits 24..27, decisions WRONG: timing only) on both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4h}
run() {  # name, KSG_DEBUG, extra bench args
  KSG_DEBUG=$2 timeout -k 10 200 python bench.py --no-cpu-baseline ${@:3} > gpurun_out/${TAG}_$1.json 2> gpurun_out/${TAG}_$1.err || { tail gpurun_out/${TAG}_$1.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_$1.json').read().strip().splitlines()[-1]); st=d['latency'].get('stages') or {}; print('$1', round(d['value']), round(d['latency']['resolver_cycles_per_pod']), d['config']['snapshots_in_timed'], json.dumps({k: st.get(k) for k in ('committer','handoff','xchecker')}))"
}
P=$((1 << 28))
run pre 0 && run nopre $P || exit 1
for x in 1 4 8; do run pre_x$x $((x << 24)) --no-stages && run nopre_x$x $((P | (x << 24))) --no-stages || exit 1; done
run ext_pre 0 --extensions --no-stages && run ext_nopre $P --extensions --no-stages
