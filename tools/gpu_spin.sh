#!/bin/bash
# the -m gpu suite and smoke, then configs 2 and 3 with the spinning batch wait
# (default) and with hipStreamSynchronize (KSG_SPIN_WAIT=0), back to back
set -o pipefail
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/s_c2a.json 2> gpurun_out/s_c2a.err &&
KSG_SPIN_WAIT=0 timeout -k 10 200 $B > gpurun_out/s_c2b.json 2> gpurun_out/s_c2b.err &&
timeout -k 10 200 $B --workload config3 > gpurun_out/s_c3a.json 2> gpurun_out/s_c3a.err &&
KSG_SPIN_WAIT=0 timeout -k 10 200 $B --workload config3 > gpurun_out/s_c3b.json 2> gpurun_out/s_c3b.err &&
timeout -k 10 200 $B > gpurun_out/s_c2c.json 2> gpurun_out/s_c2c.err &&
KSG_SPIN_WAIT=0 timeout -k 10 200 $B > gpurun_out/s_c2d.json 2> gpurun_out/s_c2d.err
