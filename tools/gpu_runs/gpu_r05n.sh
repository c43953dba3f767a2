#!/bin/bash
# GPU box: the maximum-size env test alone
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -x -v -m gpu --timeout 240 --timeout-method thread -k max_boards > gpurun_out/n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/n_tests.log; grep -E "^E " gpurun_out/n_tests.log | head -20
exit $rc
