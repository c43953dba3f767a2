#!/bin/bash
# Timing-only variants of the library (tools/variants/, never loaded by the product path): the
# float64 conv update's k_conv64_wgrad without its GEMM MFMAs (G2048_TIMING_WG_NOGEMM: operand
# fetch, conv1 and LDS staging only) and without its per-stage staging (G2048_TIMING_WG_NOPUT:
# the GEMM over stale LDS) -- where the kernel's time goes.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -fvisibility=hidden -mllvm -amdgpu-kernarg-preload-count=16"
C=reinforcement-learning-2048_amd/csrc
SRCS="$C/g2048.hip $C/g2048_qnet.hip $C/g2048_qtrain.hip $C/g2048_adam.hip $C/g2048_mlp.hip $C/g2048_learn64.hip $C/g2048_conv64.hip $C/g2048_astar.hip $C/g2048_dense.hip"
/opt/rocm/bin/hipcc $F -DG2048_TIMING_WG_NOGEMM -o tools/variants/libg2048_wg_nogemm.so $SRCS &
/opt/rocm/bin/hipcc $F -DG2048_TIMING_WG_NOPUT -o tools/variants/libg2048_wg_noput.so $SRCS &
wait
