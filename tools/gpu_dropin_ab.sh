# tools/gpu_dropin.sh for the in-tree library and for an _ab/<name> tree (same box): the tree's own
# tools/bin/dropin_latency, linked to its library (build it with tools/build_tree.sh, then
# `gcc -O2 _ab/<name>/tools/dropin_latency.c -I_ab/<name>/include -L_ab/<name>/kubernetes_amd -lkschedgpu
#  -Wl,-rpath,'$ORIGIN/../../kubernetes_amd' -o _ab/<name>/tools/bin/dropin_latency`).
# usage: ALT=<name> tools/gpu_dropin_ab.sh <tag> "<args>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
echo "== in-tree"; bash tools/gpu_dropin.sh ${TAG}_new "$@" || exit 1
echo "== $ALT"
OUT=gpurun_out/${TAG}_alt_dropin.jsonl
: > $OUT
for args in "$@"; do
  timeout -k 10 180 _ab/$ALT/tools/bin/dropin_latency $args >> $OUT || exit 1
done
cat $OUT | cut -c1-300
