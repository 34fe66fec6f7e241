# A/B helper: build kubernetes_amd/_alt/<name>/libkschedgpu.so with one kernel source compiled
# under extra defines, or from another git revision, the other objects from the main build
# (run the main build first); load it with KSG_LIB=_alt/<name>/libkschedgpu.so (abi.py).
# usage: tools/build_alt.sh <name> <plain|window> [REV|-] [hipcc defines...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; REV=$3; shift 3
O=kubernetes_amd/csrc/_obj
D=kubernetes_amd/_alt/$NAME
mkdir -p "$D"
F=kubernetes_amd/csrc/ksg_$SRC.hip
if [ "$REV" != "-" ]; then
  git show "$REV:$F" > "$D/ksg_$SRC.hip"
  F="$D/ksg_$SRC.hip"
fi
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-strict-aliasing -Wall -Wno-unused-function \
  -I kubernetes_amd/csrc -I include "$@" -c "$F" -o "$D/ksg_$SRC.o"
objs=""
for k in kernels window plain admit serve; do
  if [ "$k" = "$SRC" ]; then objs="$objs $D/ksg_$k.o"; else objs="$objs $O/ksg_$k.o"; fi
done
hipcc --offload-arch=gfx950 -shared -fPIC $objs $O/ksg_runtime.o -o "$D/libkschedgpu.so" -lrccl
rm -f "$D/ksg_$SRC.o" "$D/ksg_$SRC.hip"
