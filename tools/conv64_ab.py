#!/usr/bin/env python3
"""A/B timing of the float64 conv update with the four-wave train A (default) against the
eight-wave one (G2048_CONV64_TRAIN_A=8): two learners on the same ring, each captured with its
variant, replayed alternately after a clock settle; prints us per update (HIP events)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from g2048.learner import DQNLearner  # noqa: E402


def main(batch=8192, reps=200, rounds=3):
    dev = torch.device("cuda", 0)
    n = 65536
    env = g2048.VecEnv2048(n, seed=7, device=dev)
    rb = g2048.ReplayBuffer(16 * n, device=dev)
    env.rollout(16, replay=rb)
    Ls = {}
    for name, eight in (("4 waves", False), ("8 waves", True)):
        if eight:
            os.environ["G2048_CONV64_TRAIN_A"] = "8"
        Ls[name] = DQNLearner(rb, net="conv", dtype=torch.float64, batch_size=batch, seed=3)
        Ls[name].update()  # captured here, with this variant
        os.environ.pop("G2048_CONV64_TRAIN_A", None)
    torch.cuda.synchronize()
    for r in range(rounds):
        for name, L in Ls.items():
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.05:
                L.update()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                L.update()
            e1.record()
            torch.cuda.synchronize()
            print(f"round {r} {name}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us per update", flush=True)


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
