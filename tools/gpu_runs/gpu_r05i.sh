#!/bin/bash
# GPU box: k_step quad cache -- env / full-size / boundary tests, smoke, the step leg of the bench
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_fullsize_gpu.py tests/test_abi_gpu.py tests/test_boundary_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/i_tests.log; grep -E "FAILED|ERROR" gpurun_out/i_tests.log | cut -c1-200 | head
grep -E "^E " gpurun_out/i_tests.log | head -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 120 python -u tools/blockbench.py || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --train "" --rollout-k-extra "" --large-n "" --hbm-ring-launches 0 > gpurun_out/i_bench.json 2> gpurun_out/i_bench.err || { tail -20 gpurun_out/i_bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/i_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac']); print('step', d['step_kernel'])"
