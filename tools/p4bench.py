#!/usr/bin/env python3
"""Rollout rate at p(4) = 0.5 vs 0.1 (64k boards x 64 steps, graph-replayed after the clock
settles, as in bench.py): the p(4) = 0.1 instances draw two more Philox blocks per quad."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from sweep import graph_of, timed, ROLLOUT_BYTES  # noqa: E402


def main():
    n, kk, gl = 65536, 64, 16
    for p4 in (0.5, 0.1):
        env = g2048.VecEnv2048(n, seed=1, device="cuda:0", p4=p4)
        rb = g2048.ReplayBuffer(n * kk, device="cuda:0")
        gr = graph_of(lambda: env.rollout(kk, replay=rb), gl)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.06:
            gr.replay()
            torch.cuda.synchronize()
        tr = timed(gr.replay, 8) / gl
        print(json.dumps({"p4": p4, "boards": n, "k": kk, "launch_us": tr * 1e6,
                          "steps_per_s": n * kk / tr,
                          "GBs": ROLLOUT_BYTES * n * kk / tr / 1e9}), flush=True)
        del env, rb, gr


if __name__ == "__main__":
    main()
