#!/bin/bash
# GPU box: rocprofv3 kernel-trace summaries of the bench's env legs and learner legs, PMC passes
mkdir -p gpurun_out/prof
set -o pipefail
export TMPDIR=/tmp
rm -rf /tmp/prof_bench /tmp/prof_learn
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o bench \
    -- python bench.py --no-cpu-baseline --train "" --rollout-k-extra "" > gpurun_out/prof/bench_rocprof.json 2> gpurun_out/prof/bench_rocprof.err \
    || { tail -20 gpurun_out/prof/bench_rocprof.err; exit 1; }
cp "$(find /tmp/prof_bench -name '*kernel_stats.csv' | head -1)" gpurun_out/prof/bench_kernel_stats.csv
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_learn -o learn \
    -- python bench.py --no-cpu-baseline --step-steps 0 --steps 5 --rollout-k-extra "" --large-n "" --hbm-ring-launches 0 > gpurun_out/prof/learner_rocprof.json 2> gpurun_out/prof/learner_rocprof.err \
    || { tail -20 gpurun_out/prof/learner_rocprof.err; exit 1; }
cp "$(find /tmp/prof_learn -name '*kernel_stats.csv' | head -1)" gpurun_out/prof/learner_kernel_stats.csv
bash tools/gpu_pmc.sh > gpurun_out/prof/pmc.log 2>&1 && cp gpurun_out/pmc.json gpurun_out/prof/pmc.json
head -12 gpurun_out/prof/bench_kernel_stats.csv | cut -d, -f1-4
