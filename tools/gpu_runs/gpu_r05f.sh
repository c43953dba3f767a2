#!/bin/bash
# GPU box: fused dense-ref update -- parity tests, then the learner legs of the bench for dense
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dense_gpu.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/dense_tests.log 2>&1
echo "dense tests rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/dense_tests.log | cut -c1-150 | tail -40
grep -E "^E " gpurun_out/dense_tests.log | head -30
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --step-steps 0 --rollout-k-extra "" --large-n "" --hbm-ring-launches 0 --train dense,dense@5000 --no-cpu-baseline > gpurun_out/dense_bench.json 2> gpurun_out/dense_bench.err || { tail -20 gpurun_out/dense_bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/dense_bench.json').read().strip().splitlines()[-1])
for k,v in d['learner'].items(): print(k, round(v['update_ms'],3), 'ms', round(v['flop_frac'],3), v['path'], 'loop', round(v['loop_iter_ms'],3), round(v['loop_late_iter_ms'],3))"
rm -rf /tmp/pd && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pd -o d -- python bench.py --steps 5 --warmup 2 --step-steps 0 --rollout-k-extra "" --large-n "" --hbm-ring-launches 0 --train dense --no-cpu-baseline > gpurun_out/dense_prof.log 2>&1 && cp $(find /tmp/pd -name '*kernel_stats.csv') gpurun_out/dense_kernel_stats.csv && cut -d, -f1-4 gpurun_out/dense_kernel_stats.csv | head -20
