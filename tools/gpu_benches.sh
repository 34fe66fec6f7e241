# One default-shaped bench line per BASELINE config on one GPU (with the CPU
# baselines and the resolver's stage breakdown), run on the GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for wl in "$@"; do
  timeout -k 10 400 python bench.py --workload "$wl" > "gpurun_out/r2_bench_$wl.json" 2> "gpurun_out/r2_bench_$wl.err" || exit 1
done
