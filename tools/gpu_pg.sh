#!/bin/bash
# phase A pods per wave A/B (built with the KSG_PG under test): parity tests, configs 2/3/5/1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-stages"
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py > gpurun_out/pg_tests.log 2>&1 &&
for wl in config2 config3 config5 config1 config4; do
  timeout -k 10 200 $B --workload $wl > gpurun_out/pg_$wl.json 2>/dev/null || exit 1
done
