#!/bin/bash
# GPU box: conv learner sources built with other -mllvm scheduling knobs, one at a time (tools/sched_file_variants.py opt:...)
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/learner_ab.py "" conv || exit 1
for L in tools/variants/libg2048_g2048_qnet_*.so tools/variants/libg2048_g2048_qtrain_*.so tools/variants/libg2048_g2048_conv64_*.so; do
  timeout -k 10 240 python -u tools/learner_ab.py "$L" conv || exit 1
done
timeout -k 10 240 python -u tools/learner_ab.py "" conv || exit 1
