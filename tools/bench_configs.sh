# Bench lines (with the CPU baseline) for BASELINE configs 1, 4, 5 on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for w in config1 config4 config5; do
  timeout -k 10 200 python bench.py --workload $w --cpu-seconds 10 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit 1
done
