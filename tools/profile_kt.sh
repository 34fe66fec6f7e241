# rocprofv3 kernel-trace stats of one bench.py workload (run on the GPU box).
# usage: tools/profile_kt.sh <tag> [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_kt.log" 2>&1
