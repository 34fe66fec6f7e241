# Round-4: finer resolver stamps at config 2 (committer head / verdict reads, checker 0 loads /
# resources + LR), then config-5 profiles (kernel-trace stats and PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r4_stages.sh r4l x0=0 || exit 1
bash tools/gpu_r4_pmc.sh r4_c5 --workload config5 --steps 4 --warmup 1 || exit 1
