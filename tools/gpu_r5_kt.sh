# Round-5: rocprofv3 kernel-trace stats of bench.py for each (workload, library) pair given,
# printing each window-path kernel's mean duration; the stats CSVs stay under gpurun_out/kt_<tag>_*.
# usage: tools/gpu_r5_kt.sh <tag> <workload>:<name>:<KSG_LIB|main> ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
for spec in "$@"; do
  IFS=: read -r wl n lib <<< "$spec"
  OUT=gpurun_out/kt_${TAG}_${wl}_$n
  ( [ "$lib" != "main" ] && export KSG_LIB=$lib
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
      python3 bench.py --no-cpu-baseline --no-stages --workload $wl ${BENCH_ARGS} > "$OUT.log" 2>&1 ) || { tail "$OUT.log"; exit 1; }
  python3 - "$OUT" "$wl" "$n" <<'PY'
import csv, glob, sys
out, wl, n = sys.argv[1:]
f = sorted(glob.glob(out + "/**/*kernel_stats.csv", recursive=True))
for r in csv.DictReader(open(f[0])):
    if "ksg_win" in r["Name"]:
        print(wl, n, r["Name"].split("(")[0][5:60], r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2))
PY
done
