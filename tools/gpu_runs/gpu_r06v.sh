#!/bin/bash
# round 6 (v): the whole GPU suite once more on another box (flake check), then the f64 conv
# determinism script with both weight-gradient forms interleaved at four batches
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06v
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06v/gpu_tests.log 2>&1
rc=$?
tail -n 2 gpurun_out/r06v/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for b in 1 700 5000 8192; do
  for m in slab gemm; do timeout -k 10 120 python tools/conv64_wgrad_det.py $b $m | grep -c "diff elements 0" || exit 1; done
done
