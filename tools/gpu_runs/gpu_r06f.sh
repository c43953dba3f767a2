#!/bin/bash
# round 6 (f): the bound on the K = B weight-gradient restructure -- the float64 conv update with
# and without its conv2 / fc1 weight-gradient MFMAs and slab traffic (timing-only variant)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06f
timeout -k 10 300 python tools/learner_ab.py "" conv > gpurun_out/r06f/lib.txt 2>&1 && \
timeout -k 10 300 python tools/learner_ab.py tools/variants/libg2048_nowgrad.so conv > gpurun_out/r06f/nowgrad.txt 2>&1 && \
timeout -k 10 300 python tools/learner_ab.py "" conv > gpurun_out/r06f/lib2.txt 2>&1
rc=$?
grep -h "us/update" gpurun_out/r06f/*.txt; exit $rc
