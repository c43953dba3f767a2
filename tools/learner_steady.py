#!/usr/bin/env python3
"""Steady-state time of one learner update (graph-replayed, after a clock-settling warm-up) at
BASELINE's shapes: 64k boards, 1M-row ring, B = 8192.  Run under `rocprofv3 --kernel-trace
--stats` for the per-kernel split.  Usage: python tools/learner_steady.py [net] [fp32|fp64] [n]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from g2048.learner import DQNLearner, flops_per_update  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "conv"
dt = torch.float64 if (sys.argv[2] if len(sys.argv) > 2 else "fp64") == "fp64" else torch.float32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
n = 65536
env = g2048.VecEnv2048(n, device="cuda:0", seed=3)
rb = g2048.ReplayBuffer(16 * n, device="cuda:0")
env.rollout(16, replay=rb)
L = DQNLearner(rb, net=net, dtype=dt, batch_size=8192, target_sync_every=100)
L.update()
torch.cuda.synchronize()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.1:
    L.update()
    torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    L.update()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
peak = 78.6 if dt == torch.float64 else 157.3
tf = flops_per_update(net, 8192) / us / 1e6
print(f"{net} {dt}: {us:.1f} us per update, {1e6 / us:.0f} updates/s, {tf:.1f} TF = {tf / peak:.3f} "
      f"of {peak} TF", flush=True)
