tools/gpu_dropin.sh for the in-tree library and for KSG_LIB=$ALT (same box).
# usage: ALT=_alt/<name>/libkschedgpu.so tools/gpu_dropin_ab.sh <tag> "<args>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
echo "== in-tree"; bash tools/gpu_dropin.sh ${TAG}_new "$@" || exit 1
echo "== $ALT"; KSG_LIB=$ALT bash tools/gpu_dropin.sh ${TAG}_alt "$@" || exit 1
