#!/bin/bash
# Diagnostic builds of the one-wave-per-SIMD GEMM engine (gemm_w4.hip, VIT_W4_DIAG = 1 no LDS-DMA in
# the K-loop, 2 no fragment reads, 3 neither; timing only, results wrong) linked with the regular
# objects -> vit.rs_amd/build_w4d<N>/libvit_hip.so (select with VIT_LIB=...).  Run after make.
set -eu
cd "$(dirname "$0")/../vit.rs_amd"
for d in "$@"; do
  mkdir -p build_w4d$d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I/opt/rocm/include \
      -DVIT_W4_DIAG=$d -c csrc/gemm_w4.hip -o build_w4d$d/gemm_w4.o
  objs=$(ls build/*.o | grep -v gemm_w4.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_w4d$d/libvit_hip.so $objs build_w4d$d/gemm_w4.o \
      -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
