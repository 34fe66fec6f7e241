# Round-4: SQ counters of the resolver (config 2) and of phase A (config 5), one PMC pass per
# group of <= 8 SQ counters (MI355X_MICROARCH.md rocprofv3 limits); a killed pass ends the script.
# usage: tools/gpu_r4_sq.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_LDS SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE"
for wl in config2 config5; do
  n=1
  for pass in "$P1" "$P2" "$P3"; do
    timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$OUT/${wl}_p$n" -o run -- \
      python3 bench.py --no-cpu-baseline --no-stages --workload $wl --steps 3 --warmup 1 > "$OUT/${wl}_p$n.log" 2>&1 || exit 1
    n=$((n + 1))
  done
done
find "$OUT" -name '*counter_collection.csv' | sort
