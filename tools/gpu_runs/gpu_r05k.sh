#!/bin/bash
# GPU box: slab-store cache policy A/B (in-tree plain stores vs sc1 vs nt), conv learners
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
for r in 1 2; do
  for L in "" tools/variants/libg2048_slab16.so tools/variants/libg2048_slab2.so; do
    timeout -k 10 180 python -u tools/learner_ab.py "$L" conv || exit 1
  done
done
