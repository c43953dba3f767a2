set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_qnet_gpu.py tests/test_env_gpu.py tests/test_train_gpu.py -x -v --timeout 120 --timeout-method thread -k "greedy or dense64" > gpurun_out/new_tests.log 2>&1 || { tail -60 gpurun_out/new_tests.log; exit 1; }
tail -3 gpurun_out/new_tests.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --rollout-k 0 > gpurun_out/bench_greedy.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench_greedy.json
