#!/bin/bash
# rotating kernel-event sample: the sampling tests, configs 2/3/4, kernel traces of configs 3 and 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "sampling or totals or duplicate or config2" > gpurun_out/r_tests.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/r_c2.json 2> gpurun_out/r_c2.err &&
timeout -k 10 200 $B --workload config3 > gpurun_out/r_c3.json 2> gpurun_out/r_c3.err &&
timeout -k 10 200 $B --workload config4 > gpurun_out/r_c4.json 2> gpurun_out/r_c4.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r_c3/kt -o run -- python3 bench.py --no-cpu-baseline --no-stages --workload config3 > gpurun_out/r_kt3.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r_c2/kt -o run -- python3 bench.py --no-cpu-baseline --no-stages > gpurun_out/r_kt2.log 2>&1
