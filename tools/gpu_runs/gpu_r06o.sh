#!/bin/bash
# round 6 (o): learner GPU tests (both weight-gradient forms), the kernel-trace A/B of the two
# forms (r06i) and the wgrad probes (r06l)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06o
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_learner_gpu.py > gpurun_out/r06o/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r06o/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_runs/gpu_r06i.sh && bash tools/gpu_runs/gpu_r06l.sh
