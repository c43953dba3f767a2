# GPU box: the rollout leg of bench.py under a few launch configurations, beside tools/rollexp
set -o pipefail
mkdir -p gpurun_out/kt
B="python bench.py --no-cpu-baseline --train '' --rollout-k-extra '' --step-steps 0"
timeout -k 10 120 tools/rollexp 65536 64 > gpurun_out/kt/rollexp_a.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --train "" --rollout-k-extra "" --step-steps 0 > gpurun_out/kt/b_default.json 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --train "" --rollout-k-extra "" --step-steps 0 --graph-steps 20 > gpurun_out/kt/b_g20.json 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --train "" --rollout-k-extra "" --step-steps 0 --seed 7 > gpurun_out/kt/b_seed7.json 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --train "" --rollout-k-extra "" --step-steps 0 --steps 1000 --warmup 200 > gpurun_out/kt/b_long.json 2>&1 &&
timeout -k 10 120 tools/rollexp 65536 64 > gpurun_out/kt/rollexp_b.txt 2>&1
