# Round measurement pass (run on the GPU box): bench lines for configs 1-5 with
# the CPU baselines and stage breakdowns, then kernel-trace + FETCH/WRITE PMC
# passes for configs 2, 3 and 4 (tools/profile_gpu.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_benches.sh config1 config2 config3 config4 config5 && \
timeout -k 10 400 bash tools/profile_gpu.sh r2f_config2 --workload config2 --no-stages && \
timeout -k 10 400 bash tools/profile_gpu.sh r2f_config3 --workload config3 --no-stages && \
timeout -k 10 400 bash tools/profile_gpu.sh r2f_config4 --workload config4 --no-stages
