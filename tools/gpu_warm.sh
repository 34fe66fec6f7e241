set -o pipefail
cd "$GRAFT_REPO_ROOT"
for k in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --warmup 10 > gpurun_out/w_c2_$k.json 2> gpurun_out/w_c2_$k.err || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --warmup 10 --steps 20 > gpurun_out/w_c2_3.json 2> gpurun_out/w_c2_3.err
