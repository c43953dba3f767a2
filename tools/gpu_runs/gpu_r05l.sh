#!/bin/bash
# GPU box: fp32 conv slab with 16-byte fc1 stores -- conv learner tests, then update timing
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_learner_gpu.py tests/test_qnet_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/l_tests.log; grep -E "^E " gpurun_out/l_tests.log | head -20
[ $rc -eq 0 ] || exit 1
for r in 1 2; do timeout -k 10 180 python -u tools/learner_ab.py "" conv || exit 1; done
