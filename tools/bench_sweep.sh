set -o pipefail
cd "$GRAFT_REPO_ROOT"
for w in config2 config3 config2 config3 config4 config5; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --workload $w >> gpurun_out/b3.log 2>&1 || exit 1
done
