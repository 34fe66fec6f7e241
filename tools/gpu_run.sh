# GPU call in steps (each its own time limit; the first failure ends the call):
#   tests <k-expr> <files...>  : selected -m gpu tests
#   kt <tag> [bench args]      : rocprofv3 kernel + memory-copy trace of one bench run (no PMC)
#   ab <tag> <trees...>        : same-box tree A/B (tools/gpu_ab_trees.sh; REPS / WLS env)
#   bench <tag> [bench args]   : one bench line (with CPU baselines and stages)
# usage: tools/gpu_run.sh "<step>" "<step>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  set -- $step
  kind=$1; shift
  case $kind in
    tests)
      k=$1; shift
      timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -q --timeout 600 --timeout-method thread -k "$k" \
        > gpurun_out/tests_$k.log 2>&1 || { tail -40 gpurun_out/tests_$k.log; exit 1; }
      tail -2 gpurun_out/tests_$k.log ;;
    kt)
      tag=$1; shift
      mkdir -p gpurun_out/kt_$tag
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/kt_$tag -o run -- \
        python3 bench.py --no-cpu-baseline --no-stages "$@" > gpurun_out/kt_$tag/bench.json 2> gpurun_out/kt_$tag/bench.err \
        || { tail gpurun_out/kt_$tag/bench.err; exit 1; }
      echo "kt $tag done" ;;
    ab)
      tag=$1; shift
      bash tools/gpu_ab_trees.sh $tag "$@" || exit 1 ;;
    bench)
      tag=$1; shift
      timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
        || { tail gpurun_out/bench_$tag.err; exit 1; }
      tail -c 600 gpurun_out/bench_$tag.json ;;
  esac
done
