#!/usr/bin/env python3
"""Learner update timing with a given library build (tools/variants/*.so; no argument = the
in-tree library): conv fp32 / fp64 (and optionally other nets) at B = 8192, each learner captured,
clock-settled, then HIP events over `reps` graph-replayed updates, three rounds."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

from g2048 import _native as N  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else None
nets = sys.argv[2].split(",") if len(sys.argv) > 2 else ["conv"]
if lib:
    N.LIB_PATH = os.path.abspath(lib)
import g2048  # noqa: E402
from g2048.learner import DQNLearner  # noqa: E402

dev = torch.device("cuda", 0)
n = 65536
env = g2048.VecEnv2048(n, seed=7, device=dev)
rb = g2048.ReplayBuffer(16 * n, device=dev)
env.rollout(16, replay=rb)
tag = os.path.basename(N.LIB_PATH)
for net in nets:
    for dt in (torch.float32, torch.float64):
        L = DQNLearner(rb, net=net, dtype=dt, batch_size=8192, seed=3)
        L.update()
        torch.cuda.synchronize()
        reps = 200 if dt == torch.float32 else 100
        out = []
        for _ in range(3):
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.05:
                L.update()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                L.update()
            e1.record()
            e1.synchronize()
            out.append(round(e0.elapsed_time(e1) / reps * 1e3, 1))
        print(tag, net, str(dt).split(".")[-1], "us/update", out, "loss", float(L.last_loss), flush=True)
        del L
        torch.cuda.empty_cache()
