#!/bin/bash
# GPU box: N-sweep + rocprof kernel stats of the sweep
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err || { tail -20 gpurun_out/sweep.err; exit 1; }
cat gpurun_out/sweep.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sweep -o sweep --output-format csv -- python tools/sweep.py > gpurun_out/prof_sweep.log 2>&1 || { tail -20 gpurun_out/prof_sweep.log; exit 1; }
