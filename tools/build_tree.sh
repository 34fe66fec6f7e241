# Same-box A/B of whole trees: export git revision REV into _ab/<name>/ (git archive) and
# build its libkschedgpu.so there (no UBSan twin, no oracle: its bench runs with
# --no-cpu-baseline), so `cd _ab/<name> && python bench.py ...` runs that round's library
# with that round's bench.py on the box next to the current tree's.
# usage: tools/build_tree.sh <name> <REV>
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=$2
D=_ab/$NAME
rm -rf "$D"; mkdir -p "$D"
git archive "$REV" | tar -x -C "$D"
C=$D/kubernetes_amd/csrc
mkdir -p "$C/_obj"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-strict-aliasing -Wall -Wno-unused-function"
pids=""
for s in kernels window plain admit serve; do
  hipcc $F -c "$C/ksg_$s.hip" -o "$C/_obj/ksg_$s.o" & pids="$pids $!"
done
hipcc $F -c "$C/ksg_runtime.cpp" -o "$C/_obj/ksg_runtime.o" & pids="$pids $!"
L=""
if [ -f "$C/ksg_plain_large.hip" ]; then  # (round 6: the large-shard resolvers under the max-ILP scheduler)
  hipcc $F -mllvm -amdgpu-sched-strategy=max-ilp -c "$C/ksg_plain_large.hip" -o "$C/_obj/ksg_plain_large.o" & pids="$pids $!"
  L="$C/_obj/ksg_plain_large.o"
fi
for p in $pids; do wait $p; done
hipcc --offload-arch=gfx950 -shared -fPIC $C/_obj/ksg_{kernels,window,plain,admit,serve}.o $L $C/_obj/ksg_runtime.o \
  -o "$D/kubernetes_amd/libkschedgpu.so" -lrccl
rm -rf "$C/_obj"
# (its tests and docs are not needed on the box)
rm -rf "$D/tests" "$D/profiles" "$D"/*.md "$D"/*_r0*.json
echo "built $D/kubernetes_amd/libkschedgpu.so from $(git rev-parse --short "$REV")"
