#!/bin/bash
# Kernel-trace stats + HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE in separate
# runs, MI355X_MICROARCH.md "rocprofv3 PMC slots") of one bench.py workload.
# usage: tools/profile_gpu.sh <tag> [bench args...]   (run on the GPU box)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_kt.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_write.log" 2>&1
find "$OUT" -name '*.csv' | sort
