#!/bin/bash
# round 6 (u): train B's dW2 loop read half a step ahead (variant build -DG2048_DW2_PIPE) against
# the library: conv learner update time, alternating, and the kernel averages
set -o pipefail
export PYTHONUNBUFFERED=1
for r in 1 2; do
  timeout -k 10 200 python tools/learner_ab.py "" conv || exit 1
  timeout -k 10 200 python tools/learner_ab.py tools/variants/libg2048_dw2pipe.so conv || exit 1
done
