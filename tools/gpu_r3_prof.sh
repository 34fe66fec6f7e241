# Round-3 measurements on the GPU box: host<->kernel mailbox round trips (tools/mailbox_rtt.hip),
# the drop-in per-pod latency from C, then kernel-trace stats + FETCH/WRITE passes for the given
# workloads (tools/profile_gpu.sh).  usage: tools/gpu_r3_prof.sh <tag> [workload...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
: > gpurun_out/${TAG}_rtt.jsonl
for m in "0 64" "1 64" "1 256" "2 64" "2 256"; do
  timeout -k 10 60 tools/bin/mailbox_rtt $m 20000 >> gpurun_out/${TAG}_rtt.jsonl || exit 1
done
cat gpurun_out/${TAG}_rtt.jsonl
timeout -k 10 120 tools/bin/dropin_latency 5000 4000 200 > gpurun_out/${TAG}_dropin.json || exit 1
cat gpurun_out/${TAG}_dropin.json
for w in "$@"; do
  bash tools/profile_gpu.sh ${TAG}_$w --workload $w --no-stages > gpurun_out/${TAG}_prof_$w.log 2>&1 || { tail gpurun_out/${TAG}_prof_$w.log; exit 1; }
done
