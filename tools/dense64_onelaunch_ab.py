#!/usr/bin/env python3
"""Timing of the dense-64 update forms: two launches (the default) and the one-launch kernel
(G2048_DENSE64_ONE_LAUNCH=1), fp32 and fp64.  Each form: a fresh learner (its own captured graph),
300 graph-replayed updates after 100 untimed, HIP events.  (The round-6 experiment modes -- reducers
not waiting, no reduce, an atomic-RMW poll, the tile phase alone -- were a build-time switch since
removed; their numbers are in profiles/r06/dense64_onelaunch_ab.txt.)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from g2048.learner import DQNLearner  # noqa: E402

dev = torch.device("cuda", 0)
n = 65536
env = g2048.VecEnv2048(n, seed=9, device=dev)
rb = g2048.ReplayBuffer(16 * n, device=dev)
env.rollout(16, replay=rb)
modes = sys.argv[1:] or ["two", "one"]
for dt in (torch.float32, torch.float64):
    for mode in modes:
        os.environ.pop("G2048_DENSE64_ONE_LAUNCH", None)
        if mode == "one":
            os.environ["G2048_DENSE64_ONE_LAUNCH"] = "1"
        L = DQNLearner(rb, net="dense64", dtype=dt, batch_size=8192, target_sync_every=100)
        for _ in range(100):
            L.update()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(300):
            L.update()
        e1.record()
        torch.cuda.synchronize()
        print(f"{str(dt)[6:]} mode {mode}: {e0.elapsed_time(e1) / 300 * 1e3:.2f} us per update",
              flush=True)
