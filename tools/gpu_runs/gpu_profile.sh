#!/bin/bash
# GPU box: the round's committed evidence under gpurun_out/prof/ -- the default bench line, the
# rocprofv3 kernel-trace --stats summary of the same bench command, and the PMC passes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 420 python bench.py > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err \
    || { tail -20 gpurun_out/prof/bench.err; exit 1; }
# the headline legs alone (rollout at the headline K + one-launch-per-step kernel): the k_rollout average here is
# the bench's launches only (the learner legs' K = 16 prefill launches are profiled separately)
rm -rf /tmp/prof_bench /tmp/prof_learn
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o bench \
    -- python bench.py --no-cpu-baseline --train "" --rollout-k-extra "" > gpurun_out/prof/bench_rocprof.json 2> gpurun_out/prof/bench_rocprof.err \
    || { tail -20 gpurun_out/prof/bench_rocprof.err; exit 1; }
cp "$(find /tmp/prof_bench -name '*kernel_stats.csv' | head -1)" gpurun_out/prof/bench_kernel_stats.csv
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_learn -o learn \
    -- python bench.py --no-cpu-baseline --step-steps 0 --steps 5 --rollout-k-extra "" > gpurun_out/prof/learner_rocprof.json 2> gpurun_out/prof/learner_rocprof.err \
    || { tail -20 gpurun_out/prof/learner_rocprof.err; exit 1; }
cp "$(find /tmp/prof_learn -name '*kernel_stats.csv' | head -1)" gpurun_out/prof/learner_kernel_stats.csv
bash tools/gpu_pmc.sh && cp gpurun_out/pmc.json gpurun_out/prof/pmc.json
