#!/bin/bash
# Timing-only variant of the library (tools/variants/, never loaded by the product path): the
# float64 conv update without its conv2 / fc1 weight-gradient MFMAs and slab traffic
# (G2048_TIMING_NO_WGRAD) -- the bound on what moving those gradients to K = B GEMMs over stored
# activations could save.  Timed by tools/learner_ab.py against the library.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -fvisibility=hidden -mllvm -amdgpu-kernarg-preload-count=16"
C=reinforcement-learning-2048_amd/csrc
SRCS="$C/g2048.hip $C/g2048_qnet.hip $C/g2048_qtrain.hip $C/g2048_adam.hip $C/g2048_mlp.hip $C/g2048_learn64.hip $C/g2048_conv64.hip $C/g2048_astar.hip $C/g2048_dense.hip"
/opt/rocm/bin/hipcc $F -DG2048_TIMING_NO_WGRAD -o tools/variants/libg2048_nowgrad.so $SRCS
