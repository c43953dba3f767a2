#!/usr/bin/env python3
"""Soak: two identically seeded fused learners of each net / dtype, 1 000 graph-replayed updates
each, interleaved (another learner's graph replays between every pair of replays): their online
and target weights and Adam moments must stay bitwise equal and finite; prints the loss trend."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from g2048.learner import DQNLearner  # noqa: E402

dev = torch.device("cuda", 0)
n = 65536
env = g2048.VecEnv2048(n, seed=21, device=dev)
rb = g2048.ReplayBuffer(16 * n, device=dev)
env.rollout(16, replay=rb)
bad = 0
for net in ("conv", "dense", "dense64"):
    for dt in (torch.float32, torch.float64):
        a, b = (DQNLearner(rb, net=net, dtype=dt, batch_size=8192, target_sync_every=100, seed=4)
                for _ in range(2))
        b.model.load_state_dict(a.model.state_dict())
        b.target.load_state_dict(a.target.state_dict())
        losses = []
        for k in range(1000):
            a.update()
            b.update()
            if k % 250 == 0:
                losses.append(float(a.last_loss))
        torch.cuda.synchronize()
        ps = lambda L: list(L.model.parameters()) + list(L.target.parameters())
        same = all(torch.equal(p, q) for p, q in zip(ps(a), ps(b)))
        same = same and torch.equal(a.grad_flat, b.grad_flat)
        if a._adam is not None:
            same = same and torch.equal(a._adam.exp_avg, b._adam.exp_avg)
            same = same and torch.equal(a._adam.exp_avg_sq, b._adam.exp_avg_sq)
        finite = all(bool(torch.isfinite(p).all()) for p in ps(a))
        ok = same and finite and int(a.step_dev) == 1000
        bad += 0 if ok else 1
        print(f"{net} {str(dt)[-7:]}: bitwise {same}, finite {finite}, step {int(a.step_dev)}, "
              f"loss {[round(x, 1) for x in losses]} -> {float(a.last_loss):.1f}", flush=True)
        del a, b
        torch.cuda.empty_cache()
sys.exit(1 if bad else 0)
