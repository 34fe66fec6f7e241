#!/bin/bash
# kernel-event sampling: the parity tests, then configs 2 and 3 with events
# around every 4th window launch (default) and around every launch, back to back,
# and a kernel trace of config 2 at the default stride
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/e_tests.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/e_c2a.json 2> gpurun_out/e_c2a.err &&
KSG_KERNEL_EVENTS=1 timeout -k 10 200 $B > gpurun_out/e_c2b.json 2> gpurun_out/e_c2b.err &&
timeout -k 10 200 $B --workload config3 > gpurun_out/e_c3a.json 2> gpurun_out/e_c3a.err &&
KSG_KERNEL_EVENTS=1 timeout -k 10 200 $B --workload config3 > gpurun_out/e_c3b.json 2> gpurun_out/e_c3b.err &&
timeout -k 10 200 $B > gpurun_out/e_c2c.json 2> gpurun_out/e_c2c.err &&
KSG_KERNEL_EVENTS=1 timeout -k 10 200 $B > gpurun_out/e_c2d.json 2> gpurun_out/e_c2d.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e_c2/kt -o run -- python3 bench.py --no-cpu-baseline --no-stages > gpurun_out/e_kt.log 2>&1
