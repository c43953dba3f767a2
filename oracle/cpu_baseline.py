"""CPU baseline legs of bench.py -- TEST INFRASTRUCTURE ONLY (the timed CPU side, never the
product path).

env:     the C oracle (oracle2048.c: src/board.py + src/dqn_lib.py:91-107 restated) stepping a
         block of boards with the random policy, in P independent processes, one per host core
         ("P = nproc processes pinned"); aggregate env steps/s.
learner: the reference train_step (src/dqn_lib.py:119-164) in float64 on the host cores:
         sample B rows of an oracle-filled replay ring + encode (oracle o2048_replay_sample_f64 =
         extract_samples_*, src/dqn_lib.py:33-84), online(s'), target(s'), Bellman target,
         online(s), MSELoss(sum), backward, Adam(lr 1e-2) -- the reference's nn.Sequential nets
         (src/configs/double_dqn_conv.py:19-28, double_dqn_dense.py:7-15), torch CPU with
         torch.set_num_threads(P).  updates/s.

Run standalone as `python -m oracle.cpu_baseline env <cpu> <seconds>` (one pinned worker).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def host_cores() -> int:
    """Cores this process may use: the affinity set, capped by OMP_NUM_THREADS when set (the
    GPU box exports the box's CPU share there)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(n, 1)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _env_worker(cpu: int, seconds: float, n: int = 4096, seed: int = 0x2048) -> None:
    try:
        os.sched_setaffinity(0, {cpu})
    except OSError:
        pass
    sys.path.insert(0, _ROOT)
    from oracle import oracle as O

    env = O.OracleEnv(n, seed=seed + cpu, board_offset=cpu * n)
    env.step(O.MODE_RANDOM)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        env.step(O.MODE_RANDOM)
        steps += n
    dt = time.perf_counter() - t0
    print(json.dumps({"cpu": cpu, "steps": steps, "seconds": dt}), flush=True)


def env_baseline(seconds: float = 8.0, cores: int | None = None) -> dict:
    """P pinned oracle processes for `seconds` each, started together; aggregate env steps/s."""
    cores = cores or host_cores()
    cpus = sorted(os.sched_getaffinity(0))[:cores]
    procs = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_baseline", "env", str(c),
                               str(seconds)], cwd=_ROOT, stdout=subprocess.PIPE, text=True)
             for c in cpus]
    recs = []
    for p in procs:
        out, _ = p.communicate(timeout=seconds + 120)
        if p.returncode != 0:
            raise RuntimeError(f"cpu baseline worker failed (rc {p.returncode})")
        recs.append(json.loads(out.strip().splitlines()[-1]))
    value = sum(r["steps"] / r["seconds"] for r in recs)
    return {"value": value, "unit": "env steps/s", "cores": len(recs), "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"oracle/oracle2048.c random-policy steps (src/board.py semantics), "
                      f"{len(recs)} pinned processes x 4096 boards x {seconds:.0f} s, "
                      f"{sum(r['steps'] for r in recs)} steps in total"}


# ------------------------------------------------------------------ learner (float64, torch CPU)
def reference_net(net: str):
    """The reference's Sequential (conv: src/configs/double_dqn_conv.py:19-28; dense:
    src/configs/double_dqn_dense.py:7-15; dense64: BASELINE configs[2]) in float64."""
    from torch import nn

    if net == "conv":
        m = nn.Sequential(nn.Conv2d(1, 64, kernel_size=2), nn.ReLU(),
                          nn.Conv2d(64, 64, kernel_size=2), nn.ReLU(), nn.Flatten(),
                          nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 4))
    elif net == "dense":
        m = nn.Sequential(nn.Linear(16, 512), nn.ReLU(), nn.Linear(512, 512), nn.ReLU(),
                          nn.Linear(512, 256), nn.ReLU(), nn.Linear(256, 4))
    elif net == "dense64":
        m = nn.Sequential(nn.Linear(16, 64), nn.ReLU(), nn.Linear(64, 4))
    else:
        raise ValueError(net)
    return m.double()


def learner_baseline(net: str = "conv", batch: int = 8192, updates: int = 3,
                     threads: int | None = None, fill_boards: int = 4096,
                     fill_steps: int = 4) -> dict:
    """Reference train_step (intended zero_grad -> backward -> step order) on the host cores."""
    import copy

    import torch

    sys.path.insert(0, _ROOT)
    from oracle import oracle as O

    threads = threads or host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        model = reference_net(net)
        target = copy.deepcopy(model)
        opt = torch.optim.Adam(model.parameters(), lr=1e-2)
        cap = fill_boards * fill_steps
        env, rb = O.OracleEnv(fill_boards, seed=7), O.OracleReplay(cap)
        for _ in range(fill_steps):
            env.step(O.MODE_RANDOM, replay=rb)
        conv = net == "conv"
        gamma = torch.tensor(0.8, dtype=torch.float32)

        def one(epoch):
            _, s, a, r, s2, d = rb.sample_f64(B=batch, seed=11, epoch=epoch)
            shape = (batch, 1, 4, 4) if conv else (batch, 16)
            s, s2 = torch.from_numpy(s).view(shape), torch.from_numpy(s2).view(shape)
            a, r, d = torch.from_numpy(a), torch.from_numpy(r), torch.from_numpy(d)
            with torch.no_grad():
                a_star = torch.argmax(model(s2), 1)
                nq = target(s2).gather(1, a_star[:, None])[:, 0]
                y = r + (1 - d) * gamma.double() * nq
            opt.zero_grad()
            q = model(s).gather(1, a[:, None])[:, 0]
            loss = ((q - y) ** 2).sum()
            loss.backward()
            opt.step()
            return float(loss.detach())

        one(0)  # warm-up (allocator, Adam state)
        t0 = time.perf_counter()
        for k in range(updates):
            one(k + 1)
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return {"value": updates / dt, "unit": "updates/s", "cores": threads, "kind": "port",
            "dtype": "fp64", "batch": batch, "net": net,
            "sample": f"{updates} float64 train_steps of the reference {net} Sequential at "
                      f"B={batch} on torch CPU ({threads} threads), sampled from a "
                      f"{cap}-row oracle-filled ring ({dt:.1f} s); the batch is drawn and "
                      f"encoded by the oracle's C sampler (o2048_replay_sample_f64), which "
                      f"replaces the reference's Python extract_samples_* loops "
                      f"(src/dqn_lib.py:33-84), so this leg is faster than the reference's "
                      f"own train_step"}


if __name__ == "__main__":
    if len(sys.argv) >= 4 and sys.argv[1] == "env":
        _env_worker(int(sys.argv[2]), float(sys.argv[3]))
    else:
        print(json.dumps(env_baseline(2.0)))
        print(json.dumps(learner_baseline("conv", 5000, 1)))
        print(json.dumps(learner_baseline("dense", 5000, 1)))
