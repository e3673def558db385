#!/bin/bash
# A/B build of one translation unit with extra defines, linked with the regular objects:
#   bash tools/build_variant.sh NAME csrc/FILE.hip "-DFOO=1 -DBAR=0"
#   -> vit.rs_amd/build_NAME/libvit_hip.so  (select with VIT_LIB=vit.rs_amd/build_NAME/libvit_hip.so)
# Run after make (the other objects come from vit.rs_amd/build/).
set -eu
cd "$(dirname "$0")/../vit.rs_amd"
name=$1; src=$2; defs=${3:-}
obj=$(basename "$src" .hip).o
mkdir -p "build_$name"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I/opt/rocm/include \
    $defs -c "$src" -o "build_$name/$obj"
objs=$(ls build/*.o | grep -v "/$obj\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "build_$name/libvit_hip.so" $objs "build_$name/$obj" \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built vit.rs_amd/build_$name/libvit_hip.so"
