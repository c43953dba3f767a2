#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC passes (tools/gpu_pmc.sh): the bench's headline launch
(k_rollout, 65 536 boards x K = 64 steps, replay ring of N*K rows), the one-launch-per-step
kernel at 64k boards, and both at 4M boards (past the 256 MiB Infinity Cache, where the
memory-side counters see the HBM stream: rollout K = 16).  With argument "r8": only the 64k x 64
launch into a ring of 8 launches' rows (bench.py's rollout_64k_hbm leg; 1.27 GB, streamed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402

# boards -> rollout K (tools/pmc_summary.py keys the results by this table)
SHAPES = {65536: 64, 1 << 22: 16}

RING = 8 if sys.argv[1:] == ["r8"] else 1
for n, k in ({65536: 64} if RING > 1 else SHAPES).items():
    env = g2048.VecEnv2048(n, seed=3, device="cuda:0")
    rb = g2048.ReplayBuffer(n * k * RING, device="cuda:0")
    for _ in range(8):
        env.rollout(k, replay=rb)
    torch.cuda.synchronize()
    if RING > 1:
        continue
    r = torch.empty(n, dtype=torch.int32, device="cuda:0")
    d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    lg = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    for _ in range(20):
        env.step(None, reward=r, done=d, legal=lg)
    torch.cuda.synchronize()
    del env, rb
    torch.cuda.empty_cache()
print("pmc workload done")
