#!/bin/bash
# host-overlap check: the uid/duplicate tests, then configs 2 and 3 (twice each)
set -o pipefail
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_threads.py > gpurun_out/h_tests.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/h_c2a.json 2> gpurun_out/h_c2a.err &&
timeout -k 10 200 $B --workload config3 > gpurun_out/h_c3a.json 2> gpurun_out/h_c3a.err &&
timeout -k 10 200 $B > gpurun_out/h_c2b.json 2> gpurun_out/h_c2b.err &&
timeout -k 10 200 $B --workload config3 > gpurun_out/h_c3b.json 2> gpurun_out/h_c3b.err
