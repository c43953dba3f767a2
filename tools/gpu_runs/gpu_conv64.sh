# GPU box: the fp64 learner's parity tests, its bench leg and a rocprofv3 kernel trace of it
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_qnet_gpu.py tests/test_learner_gpu.py tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread -k "f64 or fused or fp64" > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -4 gpurun_out/t2.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --step-steps 0 --train conv,dense64 --train-dtypes fp64 --no-cpu-baseline > gpurun_out/b64.json 2>gpurun_out/b64.err || { tail -20 gpurun_out/b64.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b64.json'));[print(k, {x: v[x] for x in ('updates_per_s','update_ms','flop_frac','loop_iter_ms','loop_late_iter_ms')}) for k,v in d['learner'].items()]"
rm -rf /tmp/pr64 && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pr64 -o p -- python bench.py --steps 5 --warmup 2 --step-steps 0 --train conv --train-dtypes fp64 --no-cpu-baseline > gpurun_out/p64.log 2>&1 && cp $(find /tmp/pr64 -name '*kernel_stats.csv') gpurun_out/conv64_kernel_stats.csv && cut -d, -f1-8 gpurun_out/conv64_kernel_stats.csv | head -12
