#!/bin/bash
# Timing-only variants of the library (tools/variants/, never loaded by the product path) with the
# 16-byte slab stores through a buffer store of cache policy G2048_SLAB_AUX: 16 = sc1, 2 = nt
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -fvisibility=hidden -mllvm -amdgpu-kernarg-preload-count=16"
C=reinforcement-learning-2048_amd/csrc
SRCS="$C/g2048.hip $C/g2048_qnet.hip $C/g2048_qtrain.hip $C/g2048_adam.hip $C/g2048_mlp.hip $C/g2048_learn64.hip $C/g2048_conv64.hip $C/g2048_astar.hip $C/g2048_dense.hip"
for A in 16 2; do
  /opt/rocm/bin/hipcc $F -DG2048_SLAB_AUX=$A -o tools/variants/libg2048_slab$A.so $SRCS &
done
wait
