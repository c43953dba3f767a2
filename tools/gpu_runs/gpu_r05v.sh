#!/bin/bash
# GPU box: the bench's env legs with the default scheduler and with max-ilp, twice each
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
A="--no-cpu-baseline --train '' --rollout-k-extra ''"
for r in 1 2; do
  for L in reinforcement-learning-2048_amd/g2048/libg2048.so tools/variants/libg2048_max-ilp.so; do
    timeout -k 10 300 python -u tools/bench_with_lib.py $L --no-cpu-baseline --train "" --rollout-k-extra "" > gpurun_out/v.json 2> gpurun_out/v.err || { tail -5 gpurun_out/v.err; exit 1; }
    python -c "
import json,sys;d=json.loads(open('gpurun_out/v.json').read().strip().splitlines()[-1])
print('$L'.split('/')[-1], 'headline', round(d['value']/1e9,1), 'launch', round(d['roofline']['launch_us'],2), 'hbm64k', round(d['rollout_64k_hbm']['roofline']['frac'],3), 'large', round(d['rollout_large_n']['frac'],3), 'step', round(d['step_kernel']['launch_us_graph'],3))"
  done
done
