#!/bin/bash
mkdir -p gpurun_out
set -o pipefail
for n in 65536 131072 262144; do
  timeout -k 10 200 python bench.py --boards $n --steps 50 --warmup 5 --train '' --large-n '' --hbm-ring-launches 0 --rollout-k-extra '' --no-cpu-baseline > gpurun_out/stepn_$n.json 2> gpurun_out/stepn_$n.err || exit 1
done
