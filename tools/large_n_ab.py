#!/usr/bin/env python3
"""A/B of the large-N rollout leg (k_rollout_ws, 4M boards x K = 16, 2.55 GB of ring per launch)
by WHERE its buffers come from (bench.py times it ~10 % slower than
tools/rollexp.hip does).  Every variant runs the same g2048_env_rollout call, timed the way
bench.py times it (hipGraphs of 100 launches, each replayed once, 60 ms settle, HIP events around
`--launches` launches on the launch stream) and the way rollexp does (a 20-launch graph, 10 timed
replays), in one process, interleaved over `--rounds` rounds:

  torch/torch   env tensors and ring from torch's caching allocator (bench.py)
  torch/lib     torch env, ring from g2048_replay_create (library hipMalloc, as rollexp)
  lib/lib       env from g2048_env_create too (rollexp)
  torch/torch+  as torch/torch with the ring allocation offset to a 2 MiB boundary + 1 MiB
  torch/fresh   as torch/torch after torch.cuda.empty_cache() (ring on freshly mapped memory)

Usage: python tools/large_n_ab.py [--boards 4194304] [--k 16] [--rounds 3]"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from g2048 import _native as N  # noqa: E402


class LibEnv:
    def __init__(self, n, seed, dev):
        self.n, self._h = n, C.c_void_p()
        N.check(N.load().g2048_env_create(C.byref(self._h), n, seed, 0, dev.index, 0,
                                          N.stream_of(dev)), "g2048_env_create")
        self.dev = dev

    def rollout(self, k, replay):
        N.check(N.load().g2048_env_rollout(self._h, k, replay.handle, None, N.stream_of(self.dev)),
                "g2048_env_rollout")

    def check_errors(self):
        c = C.c_int64()
        N.check(N.load().g2048_env_error_count(self._h, C.byref(c), N.stream_of(self.dev)), "err")
        assert c.value == 0

    def __del__(self):
        N.load().g2048_env_destroy(self._h)


class LibReplay:
    def __init__(self, capacity, dev):
        self.handle = C.c_void_p()
        N.check(N.load().g2048_replay_create(C.byref(self.handle), capacity, dev.index,
                                             N.stream_of(dev)), "g2048_replay_create")

    def __del__(self):
        N.load().g2048_replay_destroy(self.handle)


def offset_replay(capacity, dev, offset, pad=0):
    """ReplayBuffer sections carved from one torch allocation starting `offset` bytes past a
    2 MiB boundary (the default layout otherwise); `pad` extra bytes after each section (breaks
    the power-of-two distances between the sections at power-of-two capacities)."""
    c = capacity
    up = lambda x: (x + 255) // 256 * 256 + pad  # noqa: E731
    o_s2 = up(16 * c)
    o_r = o_s2 + up(16 * c)
    o_a = o_r + up(4 * c)
    o_d = o_a + up(c)
    o_c = o_d + up(c)
    raw = torch.zeros(o_c + 256 + (4 << 20), dtype=torch.uint8, device=dev)
    base = (-raw.data_ptr()) % (2 << 20) + offset
    m = raw[base:]
    rb = g2048.ReplayBuffer(c, device=dev, sections=(
        m[0:16 * c].view(c, 16), m[o_s2:o_s2 + 16 * c].view(c, 16), m[o_a:o_a + c],
        m[o_r:o_r + 4 * c].view(torch.int32), m[o_d:o_d + c], m[o_c:o_c + 8].view(torch.int64)))
    rb._raw = raw
    return rb


def capture(fn, n):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    return g


def time_graph(g, reps, settle_ms):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < settle_ms:
        g.replay()
        torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        g.replay()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--boards", type=int, default=1 << 22)
    p.add_argument("--k", type=int, default=16)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=200)
    p.add_argument("--variants", default="torch/torch,torch/lib,lib/lib,torch/torch+,torch/fresh")
    p.add_argument("--rings", type=int, default=0,
                   help="mode 2: this many rings allocated up front (default layout, then padded "
                        "layouts), one env, each ring timed once per round: is the time a property "
                        "of the allocation?")
    p.add_argument("--ring-mult", type=int, default=1, help="mode 2: ring of this many launches' rows")
    p.add_argument("--pads", default="", help="mode 2 with these section pads (comma list)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    n, k = a.boards, a.k
    algo = 38.0 * n * k
    if a.rings or a.pads:
        env = g2048.VecEnv2048(n, seed=0x2048, device=dev)
        pads = ([int(x) for x in a.pads.split(",")] if a.pads else
                [0] * (a.rings // 2) + [4096 * (j + 1) + 256 * j for j in range(a.rings - a.rings // 2)])
        rings = [offset_replay(n * k * a.ring_mult, dev, 0, pad) for pad in pads]
        for rnd in range(a.rounds):
            for j, rb in enumerate(rings):
                fn = lambda: env.rollout(k, replay=rb)  # noqa: E731
                g = capture(fn, 20)
                g.replay()
                t = time_graph(g, 10, 20.0) / 200
                env.check_errors()
                print(f"round {rnd} ring {j} pad {pads[j]:6d} base {rb.s.data_ptr():#x} "
                      f"{t * 1e6:8.1f} us ({algo / t / 8e12:.3f})", flush=True)
                del g
        return
    for rnd in range(a.rounds):
        for v in a.variants.split(","):
            ev, rv = v.split("/")
            if rv == "fresh":
                torch.cuda.empty_cache()
            env = LibEnv(n, 0x2048, dev) if ev == "lib" else g2048.VecEnv2048(n, seed=0x2048, device=dev)
            rb = (LibReplay(n * k, dev) if rv == "lib" else
                  offset_replay(n * k, dev, 1 << 20) if rv == "torch+" else
                  g2048.ReplayBuffer(n * k, device=dev))
            fn = lambda: env.rollout(k, replay=rb)  # noqa: E731
            gb = capture(fn, 100)
            gb.replay()
            for _ in range(5):
                fn()
            tb = time_graph(gb, a.launches // 100, 60.0) / (a.launches // 100 * 100)
            gr = capture(fn, 20)
            gr.replay()
            tr = time_graph(gr, 10, 0.0) / 200
            env.check_errors()
            print(f"round {rnd} {v:13s} bench-style {tb * 1e6:8.1f} us ({algo / tb / 8e12:.3f})   "
                  f"rollexp-style {tr * 1e6:8.1f} us ({algo / tr / 8e12:.3f})", flush=True)
            del gb, gr, env, rb
            torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
