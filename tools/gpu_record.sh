# Record run on the GPU box, in steps (each GPU step under its own time limit; the
# first failure ends the script). usage: KSG_ROUND=r6 tools/gpu_record.sh <tag> <step> [args]
#   tests                 pytest -m gpu (every GPU test) and __graft_entry__.smoke()
#   bench <wl> [args]     one bench.py line (default shape, CPU baseline included) -> <tag>_bench_<wl>.json
#   prof <wl> [args]      rocprofv3 kernel-trace stats, then one PMC pass each for FETCH_SIZE and
#                         WRITE_SIZE, folded into profiles/traffic.json (KSG_ROUND, default r6; the sources' sha)
#   sq <wl>               one PMC pass of 8 SQ counters (busy / issue / wait fractions)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; STEP=$2; shift 2
case "$STEP" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
      || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
    tail -2 gpurun_out/${TAG}_tests.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
      || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
    tail -3 gpurun_out/${TAG}_smoke.log ;;
  bench)
    WL=$1; shift
    timeout -k 10 400 python bench.py --workload $WL "$@" > gpurun_out/${TAG}_bench_$WL.json 2> gpurun_out/${TAG}_bench_$WL.err \
      || { tail gpurun_out/${TAG}_bench_$WL.err; exit 1; }
    python - gpurun_out/${TAG}_bench_$WL.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lat=d.get("latency") or {}; r=d["roofline"]; fs=d.get("filter_score") or {}
print(d["config"]["workload"], round(d["value"]), "cyc", round(lat.get("resolver_cycles_per_pod") or 0),
      "ms/step", round(d["ms_per_step"], 3), "frac", round(r["frac"], 4), "traffic", r.get("traffic"),
      "fs_frac", round(fs.get("frac") or 0, 4), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
    ;;
  prof)
    WL=$1; shift
    OUT=gpurun_out/prof_${TAG}_$WL
    mkdir -p $OUT
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
      python3 bench.py --no-cpu-baseline --no-stages --workload $WL "$@" > $OUT/bench_kt.json 2> $OUT/bench_kt.err \
      || { tail $OUT/bench_kt.err; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
      python3 bench.py --no-cpu-baseline --no-stages --workload $WL "$@" > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err \
      || { tail $OUT/bench_fetch.err; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
      python3 bench.py --no-cpu-baseline --no-stages --workload $WL "$@" > $OUT/bench_write.json 2> $OUT/bench_write.err \
      || { tail $OUT/bench_write.err; exit 1; }
    NN=$(python3 -c "import json,sys; print(json.loads(open('$OUT/bench_kt.json').read().strip().splitlines()[-1])['config']['nodes'])")
    mv $OUT/fetch/*/run_counter_collection.csv $OUT/fetch/ 2>/dev/null; mv $OUT/write/*/run_counter_collection.csv $OUT/write/ 2>/dev/null
    KSG_ROUND=${KSG_ROUND:-r6} python3 tools/traffic_from_pmc.py $OUT $WL $NN profiles/traffic.json && cp profiles/traffic.json gpurun_out/${TAG}_traffic.json
    python3 - $OUT <<'PY'
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True))
for r in csv.DictReader(open(f[0])):
    if "ksg_" in r["Name"]:
        print(r["Name"].split("(")[0][5:70], r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2))
PY
    ;;
  sq)
    WL=$1; shift
    OUT=gpurun_out/sq_${TAG}_$WL
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      --output-format csv -d $OUT -o run -- python3 bench.py --no-cpu-baseline --no-stages --workload $WL --steps 3 --warmup 1 "$@" \
      > $OUT.json 2> $OUT.err || { tail $OUT.err; exit 1; }
    ls $OUT ;;
  *) echo "unknown step $STEP"; exit 2 ;;
esac
