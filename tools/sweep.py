#!/usr/bin/env python3
"""N-sweep of the env-step kernel (hard part ii): per-step time of one
g2048_env_step launch (hipGraph-replayed) vs boards per launch, and the rollout kernel.
At small N the launch floor dominates; at large N the step is bandwidth/VALU bound."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402

# algorithmic bytes per env step: one launch per step in random mode 37 B (54 B with
# the meta / legal bookkeeping the kernel also moves); the rollout's replay append 38 B
STEP_BYTES, STEP_BYTES_BOOK, ROLLOUT_BYTES = 37, 54, 38


def graph_of(fn, k):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(k):
            fn()
    return g


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def main():
    out = []
    for n in [1024, 4096, 16384, 65536, 262144, 1 << 20, 1 << 22, 1 << 24, 1 << 26]:
        env = g2048.VecEnv2048(n, seed=1, device="cuda:0")
        r = torch.empty(n, dtype=torch.int32, device="cuda:0")
        d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        lg = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        K = 50 if n <= (1 << 22) else 10
        g = graph_of(lambda: env.step(None, reward=r, done=d, legal=lg), K)
        t = timed(g.replay, 4) / K
        row = {"boards": n, "step_us": t * 1e6, "steps_per_s": n / t,
               "step_GBs": STEP_BYTES * n / t / 1e9,
               "step_GBs_with_bookkeeping": STEP_BYTES_BOOK * n / t / 1e9}
        if n >= (1 << 20):  # a plain device copy of the board + meta bytes (read + write 48 B)
            src = torch.empty((n, 24), dtype=torch.uint8, device="cuda:0")
            dst = torch.empty_like(src)
            tc = timed(lambda: dst.copy_(src), 10)
            row["copy_GBs"] = 48 * n / tc / 1e9
            del src, dst
        if n <= (1 << 22):
            # graph-replayed launches after >= 30 ms of the same work (the clock settles, as in
            # bench.py); K = 64 up to 1M boards, 16 at 4M (a 2.5 GB ring)
            kk = 64 if n <= (1 << 20) else 16
            rb = g2048.ReplayBuffer(n * kk, device="cuda:0")
            gl = 8
            gr = graph_of(lambda: env.rollout(kk, replay=rb), gl)
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.03:
                gr.replay()
                torch.cuda.synchronize()
            tr = timed(gr.replay, 4) / gl
            row.update(rollout_k=kk, rollout_step_us=tr / kk * 1e6,
                       rollout_steps_per_s=n * kk / tr,
                       rollout_GBs=ROLLOUT_BYTES * n * kk / tr / 1e9)
            del rb, gr
        out.append(row)
        print(json.dumps(row), flush=True)
        del env, g
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
