mkdir -p gpurun_out/r04j
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04j/t.log 2>&1; tail -3 gpurun_out/r04j/t.log
timeout -k 10 100 python tools/dense_fwd_bench.py > gpurun_out/r04j/dfwd.txt 2>&1; cat gpurun_out/r04j/dfwd.txt
