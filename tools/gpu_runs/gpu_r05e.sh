#!/bin/bash
# GPU box: eight-wave train A (bitwise vs four-wave, f64 parity, A/B timing) + the HIP graph knob
# bisect of the stale torch reduction
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_runs/gpu_r05d.sh || exit 1
bash tools/gpu_runs/gpu_r05c.sh
