#!/bin/bash
# GPU box: iterative machine-scheduler strategies against the in-tree build, learners + env step
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
for L in "" tools/variants/libg2048_iterative-ilp.so tools/variants/libg2048_iterative-maxocc.so tools/variants/libg2048_iterative-minreg.so; do
  timeout -k 10 240 python -u tools/learner_ab.py "$L" conv,dense || exit 1
  timeout -k 10 120 python -u tools/blockbench.py $L || exit 1
done
