# A/B bench lines (run on the GPU box): each argument is "tag|ENV=..|bench args"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages $args > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || exit 1
done
