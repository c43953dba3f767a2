#!/usr/bin/env python3
"""Workload for `rocprofv3 --kernel-trace --stats`: N learner updates of one net / dtype at
B = 8192 on a 1M-row ring (bench.py's bench_train setup, updates only).
Usage: prof_learner.py <net> <fp32|fp64> [updates] [batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from g2048.learner import DQNLearner  # noqa: E402

net, dt = sys.argv[1], sys.argv[2]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 20
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 8192
dev = torch.device("cuda", 0)
n = 65536
env = g2048.VecEnv2048(n, seed=9, device=dev)
rb = g2048.ReplayBuffer(16 * n, device=dev)
env.rollout(16, replay=rb)
L = DQNLearner(rb, net=net, dtype=torch.float32 if dt == "fp32" else torch.float64,
               batch_size=batch, target_sync_every=100)
for _ in range(3):
    L.update()
torch.cuda.synchronize()
for _ in range(k):
    L.update()
torch.cuda.synchronize()
print("done", float(L.last_loss))
