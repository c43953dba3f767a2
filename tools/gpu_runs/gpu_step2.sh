#!/bin/bash
# GPU box: the env parity tests and the one-launch-per-step kernel's time (bench step leg, twice)
mkdir -p gpurun_out/step
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_fullsize_gpu.py tests/test_boundary_gpu.py tests/test_abi_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/step/t.log 2>&1 || { tail -30 gpurun_out/step/t.log; exit 1; }
tail -2 gpurun_out/step/t.log
for k in 1 2; do
  timeout -k 10 200 python bench.py --train '' --no-cpu-baseline --rollout-k-extra '' --steps 50 > gpurun_out/step/b$k.json 2> gpurun_out/step/b$k.err || { tail -20 gpurun_out/step/b$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/step/b$k.json'));print(d['step_kernel'])"
done
if [ -x tools/prof_step ]; then timeout -k 10 60 tools/prof_step > gpurun_out/step/prof_step.txt 2>&1; cat gpurun_out/step/prof_step.txt; fi
