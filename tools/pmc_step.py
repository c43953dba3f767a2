#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC passes (tools/gpu_pmc.sh): the bench's headline launch
(k_rollout, 65 536 boards x K = 64 steps, replay ring of N*K rows), the one-launch-per-step
kernel at 64k boards, and both at 4M boards (past the 256 MiB Infinity Cache, where the
memory-side counters see the HBM stream: rollout K = 16)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402

# boards -> rollout K (tools/pmc_summary.py keys the results by this table)
SHAPES = {65536: 64, 1 << 22: 16}

for n, k in SHAPES.items():
    env = g2048.VecEnv2048(n, seed=3, device="cuda:0")
    rb = g2048.ReplayBuffer(n * k, device="cuda:0")
    for _ in range(8):
        env.rollout(k, replay=rb)
    torch.cuda.synchronize()
    r = torch.empty(n, dtype=torch.int32, device="cuda:0")
    d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    lg = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    for _ in range(20):
        env.step(None, reward=r, done=d, legal=lg)
    torch.cuda.synchronize()
    del env, rb
    torch.cuda.empty_cache()
print("pmc workload done")
