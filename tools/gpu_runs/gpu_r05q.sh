#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/soak_rollout.py
