#!/bin/bash
# round 6 (q): run-to-run determinism of the conv64 gradients with a slab learner in between
# (the train-B conv1 staging race), then the learner timing of both forms
set -o pipefail
export PYTHONUNBUFFERED=1
for b in 700 33 4096 8192; do timeout -k 10 120 python tools/conv64_wgrad_det.py $b slab || exit 1; done
timeout -k 10 300 python tools/learner_ab.py "" conv
