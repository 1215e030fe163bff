#!/bin/bash
# Dev build: libnps_<name>.so = libnps_hip.so with one source (env SRC, default conv2d_x3) compiled under extra
# -D flags.  usage: [SRC=spectral] tools/build_variant.sh <name> -DFOO=1 ...   (run on the CPU host after `make`)
set -e
NAME=$1; shift
SRC=${SRC:-conv2d_x3}
cd "$(dirname "$0")/../neural-pde-surrogates_amd/csrc"
mkdir -p build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics "$@" -c $SRC.hip -o build_var/${SRC}_$NAME.o
OBJS=""
for o in conv2d conv2d_x3 conv1x1_res wgrad_x3 spectral spectral3d spectral_abi data pointwise backward bf16 conv3d; do
  if [ "$o" = "$SRC" ]; then OBJS="$OBJS build_var/${SRC}_$NAME.o"; else OBJS="$OBJS build/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o ../nps_hip/libnps_$NAME.so
