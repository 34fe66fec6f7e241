# three back-to-back default benches (config 2) and one config 3 (run on the GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages > gpurun_out/p3_c2_$k.json 2> gpurun_out/p3_c2_$k.err || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --workload config3 > gpurun_out/p3_c3.json 2> gpurun_out/p3_c3.err
