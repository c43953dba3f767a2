#!/usr/bin/env python3
"""g2048_env_step at 64k boards under different output sets and graph-capture styles (events over
20 replays of a 100-step graph, every repetition printed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import g2048  # noqa: E402
from g2048 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
n = 65536
env = g2048.VecEnv2048(n, seed=0x2048, device=dev)
r = torch.empty(n, dtype=torch.int32, device=dev)
d = torch.empty(n, dtype=torch.uint8, device=dev)
lg = torch.empty(n, dtype=torch.uint8, device=dev)
lib = N.load()


def mk(rp, dp, lp):
    def f():
        N.check(lib.g2048_env_step(env._h, None, rp, dp, lp, None, N.stream_of(dev)), "step")
    return f


def side_stream_graph(f):
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(100):
                f()
    torch.cuda.synchronize()
    return g


def timed(g, label):
    g.replay()
    torch.cuda.synchronize()
    out = []
    for _ in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            g.replay()
        b.record()
        b.synchronize()
        out.append(round(a.elapsed_time(b) * 1e3 / 2000, 3))
    print(label, out, "us/step", flush=True)


variants = {"all": mk(N.ptr(r), N.ptr(d), N.ptr(lg)), "none": mk(None, None, None),
            "reward": mk(N.ptr(r), None, None), "done+legal": mk(None, N.ptr(d), N.ptr(lg)),
            "legal": mk(None, None, N.ptr(lg)), "reward+done": mk(N.ptr(r), N.ptr(d), None)}
for name, f in variants.items():
    timed(side_stream_graph(f), name)
timed(bench.capture(lambda: env.step(None, reward=r, done=d, legal=lg), 100), "bench.capture")

