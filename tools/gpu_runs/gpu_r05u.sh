#!/bin/bash
# GPU box: machine-scheduler strategy A/B (in-tree default vs max-ilp vs max-memory-clause)
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
for L in "" tools/variants/libg2048_max-ilp.so tools/variants/libg2048_max-memory-clause.so; do
  timeout -k 10 240 python -u tools/learner_ab.py "$L" conv,dense || exit 1
  timeout -k 10 120 python -u tools/blockbench.py $L || exit 1
done
