#!/usr/bin/env python3
"""Workload for the PMC passes (FETCH_SIZE / WRITE_SIZE): eager g2048_env_step launches at
64k boards (the bench config) and at 4M boards (past the 256 MiB Infinity Cache, where the
counters see the real HBM stream), plus a k_rollout launch with replay append."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402

for n in (65536, 1 << 22):
    env = g2048.VecEnv2048(n, seed=3, device="cuda:0")
    r = torch.empty(n, dtype=torch.int32, device="cuda:0")
    d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    lg = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    for _ in range(50):
        env.step(None, reward=r, done=d, legal=lg)
    torch.cuda.synchronize()
    rb = g2048.ReplayBuffer(n * 8, device="cuda:0")
    for _ in range(3):
        env.rollout(8, replay=rb)
    torch.cuda.synchronize()
    del env, rb
    torch.cuda.empty_cache()
print("pmc workload done")
