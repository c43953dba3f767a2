#!/usr/bin/env python3
"""The reference dense net's forward over 64k board rows: the HIP kernel (g2048_densenet_forward)
against torch's four GEMMs, float32 and float64 (events over 20 calls after a warm-up)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
import torch  # noqa: E402

import g2048  # noqa: E402
from g2048 import qnet  # noqa: E402
from g2048.nets import det_init, make_net  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rows = torch.randint(0, 12, (n, 16), dtype=torch.uint8, device="cuda")


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for dt, peak in ((torch.float32, 157.3), (torch.float64, 78.6)):
    m = det_init(make_net("dense", dt, "cuda"), 0.3)
    f = qnet.DenseForward(m)
    out = torch.empty((n, 4), dtype=dt, device="cuda")
    x = rows.to(dt)
    with torch.no_grad():
        th = t(lambda: m(x))
    hip = t(lambda: f(rows, out=out))
    fl = 2.0 * 402432 * n
    print(f"{dt}: HIP {hip:.1f} us ({fl / hip / 1e6:.1f} TF, {fl / hip / 1e6 / peak:.3f} of {peak}), "
          f"torch {th:.1f} us", flush=True)
