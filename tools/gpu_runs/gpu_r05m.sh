#!/bin/bash
# GPU box: tiny-batch parity cases (B = 1, 17, 33) of the fused learners
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_qnet_gpu.py tests/test_learner_gpu.py tests/test_dense_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -k "matches_autograd or equals_torch_path or equals_autograd" > gpurun_out/m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/m_tests.log; grep -E "FAILED|ERROR" gpurun_out/m_tests.log | cut -c1-200 | head; grep -E "^E " gpurun_out/m_tests.log | head -30
exit $rc
