# Round-4 profiles of one bench workload (run on the GPU box): kernel-trace stats, then one PMC
# pass each for FETCH_SIZE, WRITE_SIZE, L2 hit / miss, and last the TA stall counters
# (MI355X_MICROARCH.md: one pass per counter group; a pass that hangs is killed, nothing after it).
# usage: tools/gpu_r4_pmc.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
  python3 bench.py --no-cpu-baseline --no-stages "$@" > "$OUT/bench_kt.log" 2>&1 || exit 1
for pass in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  name=$(echo $pass | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$OUT/$name" -o run -- \
    python3 bench.py --no-cpu-baseline --no-stages "$@" > "$OUT/bench_$name.log" 2>&1 || exit 1
done
find "$OUT" -name '*.csv' | sort
