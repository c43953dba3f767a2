#!/usr/bin/env python3
"""Soak of the one-launch-per-step kernels: 4 000 graph-replayed random-policy steps with every
output and the ring append at 64k boards, then three 1 000-board slices (boards, counters, ring
rows) against the oracle; then 2 000 graph-replayed training-loop iterations of the fused conv
float64 learner (greedy-branch forward + fused eps-greedy step + update) with the env's error
counter and the weights' finiteness checked."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import g2048  # noqa: E402
from g2048.learner import DQNLearner, Trainer  # noqa: E402
from oracle import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
n, steps, seed = 65536, 4000, 13
rows = 64
env = g2048.VecEnv2048(n, seed=seed, device=dev)
rb = g2048.ReplayBuffer(rows * n, device=dev)
r = torch.empty(n, dtype=torch.int32, device=dev)
d = torch.empty(n, dtype=torch.uint8, device=dev)
lg = torch.empty(n, dtype=torch.uint8, device=dev)
g = bench.capture(lambda: env.step(None, replay=rb, reward=r, done=d, legal=lg), 100)  # 1 + 100
t0 = time.perf_counter()
for _ in range((steps - 1) // 100):
    g.replay()
for _ in range(steps - 1 - 100 * ((steps - 1) // 100)):
    env.step(None, replay=rb, reward=r, done=d, legal=lg)
torch.cuda.synchronize()
print(f"{steps} steps x {n} boards in {time.perf_counter() - t0:.2f} s", flush=True)
env.check_errors()
bad = 0
for i0 in (0, n // 2 - 500, n - 1000):
    k = 1000
    ref = O.OracleEnv(k, seed=seed, board_offset=i0)
    ref_rb = O.OracleReplay(k * rows)
    for _ in range(steps):
        o = ref.step(O.MODE_RANDOM, replay=ref_rb)
    sl = slice(i0, i0 + k)
    ok = (np.array_equal(env.board[sl].cpu().numpy(), ref.board) and
          np.array_equal(env.score_moves()[sl].cpu().numpy().view(np.uint32), ref.meta) and
          np.array_equal(env.ep[sl].cpu().numpy().view(np.uint32), ref.ep) and
          np.array_equal(r[sl].cpu().numpy(), o["reward"]) and
          np.array_equal(lg[sl].cpu().numpy(), o["legal"]))
    ridx = torch.from_numpy((np.arange(rows)[:, None] * n + np.arange(i0, i0 + k)[None, :])
                            .reshape(-1)).to(dev)
    for name in ("s", "s2", "a", "r", "d"):
        ok = ok and np.array_equal(getattr(rb, name).index_select(0, ridx).cpu().numpy(),
                                   getattr(ref_rb, name))
    bad += 0 if ok else 1
    print(f"  slice {i0}: {'ok' if ok else 'MISMATCH'}", flush=True)
del env, rb
torch.cuda.empty_cache()

env = g2048.VecEnv2048(n, seed=17, device=dev)
rb = g2048.ReplayBuffer(1 << 20, device=dev)
L = DQNLearner(rb, net="conv", dtype=torch.float64, batch_size=8192, target_sync_every=100)
T = Trainer(env, rb, L, updates_per_step=1, min_fill=0)
T.prefill(16)
t0 = time.perf_counter()
for _ in range(2000):
    T.step()
torch.cuda.synchronize()
env.check_errors()
finite = all(bool(torch.isfinite(p).all()) for p in list(L.model.parameters()) + list(L.target.parameters()))
eps = T.current_epsilon()
print(f"2000 training-loop iterations in {time.perf_counter() - t0:.2f} s, updates {int(L.step_dev)}, "
      f"finite {finite}, episodes {int(env.ep[:, 0].sum())}, eps mean {float(eps.mean()):.3f}, "
      f"loss {float(L.last_loss):.1f}", flush=True)
bad += 0 if (finite and int(L.step_dev) == 2000) else 1
print("slices / loop bad:", bad, flush=True)
sys.exit(1 if bad else 0)
