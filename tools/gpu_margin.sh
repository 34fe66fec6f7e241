#!/bin/bash
# round sizing A/B: windows per round = margin x pods left / pods per window + 1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-stages"
for wl in config2 config3 config4 config1; do
  i=0
  for m in 1.1 1.0 1.1 1.0; do
    i=$((i + 1))
    KSG_ROUND_MARGIN=$m timeout -k 10 200 $B --workload $wl > gpurun_out/m_${wl}_${m}_$i.json 2>/dev/null || exit 1
  done
done
