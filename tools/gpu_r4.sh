# resolver experiments (run on the GPU box): parity of the alternatives, then benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "alternative" > gpurun_out/r4_tests.log 2>&1 && \
KSG_DEBUG=1024 timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages > gpurun_out/r4_c2.json 2> gpurun_out/r4_c2.err && \
KSG_DEBUG=1032 timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --steps 4 > gpurun_out/r4_dbg_c2.json 2> gpurun_out/r4_dbg_c2.err && \
KSG_DEBUG=1024 timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --workload config3 > gpurun_out/r4_c3.json 2> gpurun_out/r4_c3.err
