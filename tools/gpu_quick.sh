# quick GPU loop: focused parity tests, then the default bench and debug stamps (run on the GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_affinity_trap.py "$@" > gpurun_out/gpu_quick.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
KSG_DEBUG=8 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/dbg_c2.json 2> gpurun_out/dbg_c2.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --workload config3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
