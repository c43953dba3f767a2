#!/bin/bash
# round 6 (t): the soaks on the ABI-v5 tree (one-launch steps + training loop, rollouts at 4M and
# 64k, seeded learners) -> gpurun_out/r06t/
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06t
timeout -k 10 500 python tools/soak_step.py > gpurun_out/r06t/soak_step.txt 2>&1 && \
timeout -k 10 500 python tools/soak_rollout.py > gpurun_out/r06t/soak_rollout.txt 2>&1 && \
timeout -k 10 500 python tools/soak_learner.py > gpurun_out/r06t/soak_learner.txt 2>&1
rc=$?
for f in gpurun_out/r06t/*.txt; do tail -n 5 "$f"; done
exit $rc
