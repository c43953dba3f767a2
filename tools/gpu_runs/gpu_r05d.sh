#!/bin/bash
# GPU box: eight-wave train A -- bitwise test against the four-wave kernel, the f64 learner
# parity tests, A/B timing, rocprof of both
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_learner_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread -k "train_a8 or fused_f64 or conv" > gpurun_out/a8_tests.log 2>&1 || { tail -30 gpurun_out/a8_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/a8_tests.log; tail -2 gpurun_out/a8_tests.log
timeout -k 10 300 python -u tools/conv64_ab.py > gpurun_out/a8_ab.txt 2>&1 || { tail -20 gpurun_out/a8_ab.txt; exit 1; }
cat gpurun_out/a8_ab.txt
rm -rf /tmp/pa8 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pa8 -o a8 -- python tools/conv64_ab.py 8192 50 1 > gpurun_out/a8_prof.log 2>&1 && cp $(find /tmp/pa8 -name '*kernel_stats.csv') gpurun_out/a8_kernel_stats.csv && cut -d, -f1-4 gpurun_out/a8_kernel_stats.csv | grep -i conv64
