#!/bin/bash
# Timing-only variants of the library (tools/variants/, never loaded by the product path) built
# with another machine scheduler (AMDGPU --amdgpu-sched-strategy) for every source:
#   tools/sched_variants.sh [strategy ...]   (default: max-ilp max-memory-clause)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -fvisibility=hidden -mllvm -amdgpu-kernarg-preload-count=16"
C=reinforcement-learning-2048_amd/csrc
SRCS="$C/g2048.hip $C/g2048_qnet.hip $C/g2048_qtrain.hip $C/g2048_adam.hip $C/g2048_mlp.hip $C/g2048_learn64.hip $C/g2048_conv64.hip $C/g2048_astar.hip $C/g2048_dense.hip"
for S in ${@:-max-ilp max-memory-clause}; do
  /opt/rocm/bin/hipcc $F -mllvm --amdgpu-sched-strategy=$S -o tools/variants/libg2048_$S.so $SRCS &
done
wait
