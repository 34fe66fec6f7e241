set -o pipefail
cd "$GRAFT_REPO_ROOT"
for w in config2 config3 config4; do
  KSG_DEBUG=8 timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 4 > gpurun_out/dbg_$w.json 2> gpurun_out/dbg_$w.err || exit 1
done
