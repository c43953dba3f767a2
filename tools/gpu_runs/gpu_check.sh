#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprofv3 kernel trace (run via gpurun).
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf /tmp/prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python bench.py --steps 1000 --no-cpu-baseline --train '' --rollout-k-extra '' > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp $(find /tmp/prof -name "*kernel_stats.csv") gpurun_out/bench_kernel_stats.csv
if [ -n "$G2048_SWEEP" ]; then timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err || { tail -20 gpurun_out/sweep.err; exit 1; }; cat gpurun_out/sweep.jsonl; fi
if [ -x tools/prof_conv64 ]; then timeout -k 10 120 tools/prof_conv64 > gpurun_out/prof_conv64.txt 2>&1 || { tail -20 gpurun_out/prof_conv64.txt; exit 1; }; fi
rm -rf /tmp/prl && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prl -o p -- python bench.py --steps 5 --warmup 2 --step-steps 0 --train conv --train-dtypes fp32,fp64 --no-cpu-baseline > gpurun_out/plearn.log 2>&1 && cp $(find /tmp/prl -name '*kernel_stats.csv') gpurun_out/learner_conv_kernel_stats.csv
