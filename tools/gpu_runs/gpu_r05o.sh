#!/bin/bash
# GPU box: env edge cases (clock past 2^32, steps across clock moves)
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -x -v -m gpu --timeout 240 --timeout-method thread -k "clock" > gpurun_out/o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED" gpurun_out/o_tests.log | cut -c1-120; grep -E "^E " gpurun_out/o_tests.log | head -20
exit $rc
