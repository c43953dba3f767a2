#!/usr/bin/env python3
"""Env-step throughput at 64k boards with the boards split into K shards, each stepped by its own
captured graph on its own HIP stream (K independent hardware queues), vs one stream.  The shards
are board_offset slices of one env, so the boards after any number of steps are bitwise those of
the single 64k-board env (checked here)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402

DEV = torch.device("cuda", 0)
N, G, REPS, SEED = 65536, 100, 20, 0x2048


def run(k):
    n = N // k
    envs = [g2048.VecEnv2048(n, seed=SEED, device=DEV, board_offset=i * n) for i in range(k)]
    streams = [torch.cuda.Stream(DEV) for _ in range(k)]
    outs = [(torch.empty(n, dtype=torch.int32, device=DEV), torch.empty(n, dtype=torch.uint8, device=DEV),
             torch.empty(n, dtype=torch.uint8, device=DEV)) for _ in range(k)]
    graphs = []
    torch.cuda.synchronize()
    for e, s, o in zip(envs, streams, outs):
        s.wait_stream(torch.cuda.current_stream(DEV))
        with torch.cuda.stream(s):
            e.step(None, reward=o[0], done=o[1], legal=o[2])  # warm
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(G):
                    e.step(None, reward=o[0], done=o[1], legal=o[2])
        graphs.append(g)
    torch.cuda.synchronize()
    for g, s in zip(graphs, streams):  # warm replays
        with torch.cuda.stream(s):
            g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        for g, s in zip(graphs, streams):
            with torch.cuda.stream(s):
                g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = G * REPS + G + 1  # graph replays + warm-up (per board)
    boards = torch.cat([e.board for e in envs])
    return dict(k=k, us_per_step=dt / (G * REPS) * 1e6, env_steps_per_s=N * G * REPS / dt,
                steps=steps), boards


if __name__ == "__main__":
    res, ref = [], None
    for k in (1, 2, 4, 8):
        r, b = run(k)
        if ref is None:
            ref = b
        r["boards_equal_k1"] = bool(torch.equal(b, ref))
        res.append(r)
        print(json.dumps(r), flush=True)
