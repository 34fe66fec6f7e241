# Config 4 loop (run on the GPU box): anti-affinity parity tests, bench line,
# kernel-trace stats.  usage: tools/gpu_c4.sh <tag> [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_affinity_trap.py -k "anti or config4 or fuzz or trap" \
  > gpurun_out/c4_tests_$TAG.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --workload config4 "$@" > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err && \
timeout -k 10 300 bash tools/profile_kt.sh c4_$TAG --workload config4 --no-stages "$@"
