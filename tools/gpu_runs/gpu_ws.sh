mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_fullsize_gpu.py tests/test_env_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -3 gpurun_out/t5.log
for n in 262144 524288; do timeout -k 10 150 tools/rollexp $n 64 > gpurun_out/ws_$n.txt 2>&1 || exit 1; done
grep -E "lean  |k_rollout_lean|ws2|5 waves" gpurun_out/ws_262144.txt gpurun_out/ws_524288.txt | head -30
