mkdir -p gpurun_out/r04i
for b in launch_floor launch_floor_pre launch_floor launch_floor_pre; do echo $b; timeout -k 5 30 tools/bin/$b || exit 1; done
timeout -k 10 400 python -u -m pytest tests/test_dense_gpu.py tests/test_env_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04i/t.log 2>&1; tail -3 gpurun_out/r04i/t.log
timeout -k 10 100 python tools/dense_fwd_bench.py > gpurun_out/r04i/dfwd.txt 2>&1; cat gpurun_out/r04i/dfwd.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --train "" --rollout-k-extra "" > gpurun_out/r04i/b.json 2> gpurun_out/r04i/b.err || { tail gpurun_out/r04i/b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04i/b.json')); print(d['value'], d['step_kernel'])"
