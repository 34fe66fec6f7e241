#!/bin/bash
# diagnostics read once around the timed loop (ksg_batch_totals): parity tests, configs 2/3/2/1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t_tests.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/t_c2a.json 2> gpurun_out/t_c2a.err &&
timeout -k 10 200 $B --workload config3 > gpurun_out/t_c3a.json 2> gpurun_out/t_c3a.err &&
timeout -k 10 200 $B > gpurun_out/t_c2b.json 2> gpurun_out/t_c2b.err &&
timeout -k 10 200 $B --workload config1 > gpurun_out/t_c1a.json 2> gpurun_out/t_c1a.err
