# A/B helper: build kubernetes_amd/_alt/libkschedgpu.so with ksg_plain.hip compiled under extra
# defines (e.g. tools/build_alt.sh -DKSG_POST_RELEASE), the other objects from the main build;
# load it with KSG_LIB=kubernetes_amd/_alt/libkschedgpu.so (abi.py).
set -e
cd "$(dirname "$0")/.."
O=kubernetes_amd/csrc/_obj
mkdir -p kubernetes_amd/_alt
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-strict-aliasing -Wall -Wno-unused-function \
  "$@" -c kubernetes_amd/csrc/ksg_plain.hip -o $O/ksg_plain_alt.o
hipcc --offload-arch=gfx950 -shared -fPIC $O/ksg_kernels.o $O/ksg_window.o $O/ksg_plain_alt.o $O/ksg_admit.o \
  $O/ksg_serve.o $O/ksg_runtime.o -o kubernetes_amd/_alt/libkschedgpu.so -lrccl
