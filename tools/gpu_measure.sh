# Round measurement pass (run on the GPU box): default bench (with the latency
# breakdown), the drop-in per-call latency harness, and kernel-trace + PMC
# passes of configs 1-5 (tools/profile_gpu.sh). Outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py > gpurun_out/m_bench_c2.json 2> gpurun_out/m_bench_c2.err && \
timeout -k 10 120 ./tools/bin/dropin_latency 5000 4000 200 > gpurun_out/m_dropin_latency.json 2> gpurun_out/m_dropin.err && \
for wl in "$@"; do
  timeout -k 10 600 bash tools/profile_gpu.sh "$wl" --workload "$wl" --no-stages || exit 1
done
