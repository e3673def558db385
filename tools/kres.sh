#!/bin/bash
# usage: tools/kres.sh file.hip [name-filter]  -> kernel  VGPRs  scratch  (gfx950 resource usage)
f=$1; flt=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I/opt/rocm/include -I$(dirname $f) -c $f -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
awk '/Function Name:/{n=$5} /VGPRs:/{v=$4} /ScratchSize/{s=$5; print n, "vgpr=" v, "scratch=" s}' | grep -E "$flt"
