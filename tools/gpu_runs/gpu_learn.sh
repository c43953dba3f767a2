#!/bin/bash
# GPU box: the conv learners' parity tests (fp32 + fp64), their bench legs and a rocprofv3 kernel
# trace of them (the per-kernel times of one update).
mkdir -p gpurun_out/learn
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_qnet_gpu.py tests/test_learner_gpu.py tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/learn/t.log 2>&1 || { tail -40 gpurun_out/learn/t.log; exit 1; }
tail -3 gpurun_out/learn/t.log
for t in prof_conv64_old prof_conv64; do
  if [ -x tools/$t ]; then timeout -k 10 120 tools/$t > gpurun_out/learn/$t.txt 2>&1 || { tail -20 gpurun_out/learn/$t.txt; exit 1; }; fi
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --step-steps 0 --train conv --train-dtypes fp32,fp64 --no-cpu-baseline > gpurun_out/learn/b.json 2>gpurun_out/learn/b.err || { tail -20 gpurun_out/learn/b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/learn/b.json'));[print(k, {x: v[x] for x in ('updates_per_s','update_ms','flop_frac','loop_iter_ms','loop_late_iter_ms')}) for k,v in d['learner'].items()]"
rm -rf /tmp/prl && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prl -o p -- python bench.py --steps 5 --warmup 2 --step-steps 0 --train conv --train-dtypes fp32,fp64 --no-cpu-baseline > gpurun_out/learn/p.log 2>&1 && cp $(find /tmp/prl -name '*kernel_stats.csv') gpurun_out/learn/kernel_stats.csv && cut -d, -f1-8 gpurun_out/learn/kernel_stats.csv | head -16
