set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/prof_train > gpurun_out/prof_train.txt 2>&1 || { cat gpurun_out/prof_train.txt; exit 1; }
cat gpurun_out/prof_train.txt
timeout -k 10 300 python -u -m pytest tests/test_qnet_gpu.py tests/test_learner_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qnet_tests.log 2>&1 || { tail -60 gpurun_out/qnet_tests.log; exit 1; }
tail -2 gpurun_out/qnet_tests.log
