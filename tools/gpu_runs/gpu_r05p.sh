#!/bin/bash
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/clock_probe.py || exit 1
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/p_tests.log; grep -E "^E " gpurun_out/p_tests.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --train "" --rollout-k-extra "" --large-n "" --hbm-ring-launches 0 --step-steps 0 > gpurun_out/p_bench.json 2> gpurun_out/p_bench.err || { tail -5 gpurun_out/p_bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/p_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], d['roofline']['launch_us'])"
