#!/bin/bash
# GPU box: reductions with more CUs (fp32 conv pre-reduce, fp64 conv reduce) -- learner / qnet /
# graph-hazard tests, then the conv learner legs of the bench
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_learner_gpu.py tests/test_qnet_gpu.py tests/test_graph_hazards_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/h_tests.log; grep -E "FAILED|ERROR" gpurun_out/h_tests.log | cut -c1-200 | head
grep -E "^E " gpurun_out/h_tests.log | head -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --step-steps 0 --rollout-k-extra "" --large-n "" --hbm-ring-launches 0 --train conv --no-cpu-baseline > gpurun_out/h_bench.json 2> gpurun_out/h_bench.err || { tail -20 gpurun_out/h_bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/h_bench.json').read().strip().splitlines()[-1])
for k,v in d['learner'].items(): print(k, round(v['update_ms'],4), 'ms', round(v['flop_frac'],4), v['path'], 'loop', round(v['loop_iter_ms'],3), round(v['loop_late_iter_ms'],3))"
rm -rf /tmp/ph && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ph -o h -- python bench.py --steps 5 --warmup 2 --step-steps 0 --rollout-k-extra "" --large-n "" --hbm-ring-launches 0 --train conv --no-cpu-baseline > gpurun_out/h_prof.log 2>&1 && cp $(find /tmp/ph -name '*kernel_stats.csv') gpurun_out/h_kernel_stats.csv && grep -E "reduce|train|targets" gpurun_out/h_kernel_stats.csv | cut -d, -f1-4
