set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --rollout-k 0 > gpurun_out/bench_step.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_step.json'))
print('value', d['value'])
for k,v in d['learner'].items(): print(k, round(v['update_ms']*1e3,2), 'us/update', round(v['loop_iter_ms']*1e3,1), round(v['loop_late_iter_ms']*1e3,1))"
