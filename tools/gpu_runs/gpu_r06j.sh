#!/bin/bash
# round 6 (j): the GEMM-form weight gradients -- parity subset, then the kernel-trace A/B (r06i)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_learner_gpu.py -k "wgrad or fused_f64 or conv64" > gpurun_out/r06j/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r06j/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_runs/gpu_r06i.sh
