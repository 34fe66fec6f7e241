# Same-box A/B of whole trees (tools/build_tree.sh): the current tree against _ab/<name> trees,
# interleaved (rep x workload x tree), each bench line without CPU baseline or stage rerun.
# usage: REPS=2 WLS="config5 config3" tools/gpu_ab_trees.sh <tag> <name>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=$PWD/gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for wl in ${WLS:-config5 config3}; do
    for t in cur "$@"; do
      d=$PWD; [ "$t" != cur ] && d=$PWD/_ab/$t
      ( cd "$d" && timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-stages ${BENCH_ARGS} \
          > $OUT/${TAG}_${t}_${wl}_$rep.json 2> $OUT/${TAG}_${t}_${wl}_$rep.err ) || { tail $OUT/${TAG}_${t}_${wl}_$rep.err; exit 1; }
      python - "$OUT/${TAG}_${t}_${wl}_$rep.json" "$t" "$wl" "$rep" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lat=d.get("latency") or {}
rf=d.get("roofline") or {}
print("==", sys.argv[2], sys.argv[3], "rep", sys.argv[4], round(d["value"]), "ms/step", round(d["ms_per_step"], 3),
      "res_cyc", round(lat.get("resolver_cycles_per_pod") or 0), "kms", round((rf.get("kernel_ms_avg") or 0) * 1e3, 1),
      "launches", rf.get("launches"), flush=True)
PY
    done
  done
done
