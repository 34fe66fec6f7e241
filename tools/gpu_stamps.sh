# drop-in latency with the server's per-stage stamps (KSG_SERVE_STAMPS=1), stderr holds the stage line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
: > gpurun_out/${TAG}_stamps.txt
for n in 500 5000 15000; do
  KSG_SERVE_STAMPS=1 timeout -k 10 120 tools/bin/dropin_latency $n 2000 200 1 >> gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
done
cut -c1-400 gpurun_out/${TAG}_stamps.txt
