# GPU suite, then v15 profiles (kernel trace + FETCH/WRITE passes) and bench lines
# for configs 2 and 3 (run on the GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
bash tools/profile_gpu.sh v15c2 --workload config2 && \
bash tools/profile_gpu.sh v15c3 --workload config3 && \
timeout -k 10 200 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
timeout -k 10 200 python bench.py --workload config3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
