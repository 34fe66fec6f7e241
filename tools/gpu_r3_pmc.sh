# FETCH_SIZE calibration (tools/fetch_calib.hip), then kernel-trace stats + FETCH / WRITE passes
# of the given bench workloads (tools/profile_gpu.sh), final round-3 build.
# usage: tools/gpu_r3_pmc.sh <tag> [workload...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/${TAG}_calib
timeout -k 10 60 tools/bin/fetch_calib > gpurun_out/${TAG}_calib/bytes.json || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_calib/fetch -o run -- \
  tools/bin/fetch_calib > gpurun_out/${TAG}_calib/run.log 2>&1 || { tail gpurun_out/${TAG}_calib/run.log; exit 1; }
for w in "$@"; do
  bash tools/profile_gpu.sh ${TAG}_$w --workload $w > gpurun_out/${TAG}_prof_$w.log 2>&1 || { tail gpurun_out/${TAG}_prof_$w.log; exit 1; }
done
find gpurun_out -path "*${TAG}*" -name '*.csv' | sort
