# Round-4: instruction-cache counters of the resolver at config 2 (one PMC pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq_r4
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQC_TC_INST_REQ SQC_TC_STALL SQ_INSTS_VALU \
  --output-format csv -d "$OUT/config2_ic" -o run -- \
  python3 bench.py --no-cpu-baseline --no-stages --workload config2 --steps 3 --warmup 1 > "$OUT/config2_ic.log" 2>&1 || exit 1
