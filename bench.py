#!/usr/bin/env python3
"""Benchmark of the 2048 hot path on MI355X (contract: see DESIGN.md "Measurement").

Default workload = BASELINE.json configs[1]: 65 536 vectorised boards per GPU, env step only
(uniform random actions drawn in-kernel from Philox), one g2048_env_step launch per step,
replayed from hipGraphs of `--graph-steps` steps.  value = env steps/s over all ranks.
Extra fields report the K-steps-per-launch rollout kernel and (with --train) DQN updates/s.

Multi-GPU: one process per GPU (torchrun), boards sharded by board_offset = rank * N, no
collective on the env path (weak scaling); timing = max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "2048 env steps/sec + DQN updates/sec at 64k parallel boards, 1→8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# algorithmic bytes per env step of k_step (random mode, reward + done + legal outputs):
# board 16 R + 16 W, meta 16 R + 16 W, reward 4 W, done 1 W, legal 1 W
STEP_BYTES = 70
# rollout kernel with replay append, per step: transition s 16 + s' 16 + a 1 + r 4 + d 1
ROLLOUT_BYTES = 38


PMC_FILE = os.path.join(ROOT, "profiles", "r01", "pmc_step.json")


def pmc_traffic(kernel: str, boards: int):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (tools/gpu_pmc.sh:
    separate FETCH_SIZE / WRITE_SIZE runs, FETCH_SIZE x2 gfx950 correction), or None."""
    try:
        with open(PMC_FILE) as f:
            rec = json.load(f).get(f"{kernel}@{boards}")
    except (OSError, ValueError):
        return None, None
    if not rec:
        return None, None
    return rec["hbm_bytes_per_launch"], os.path.relpath(PMC_FILE, ROOT)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--boards", type=int, default=65536)
    p.add_argument("--graph-steps", type=int, default=100)
    p.add_argument("--seed", type=int, default=0x2048)
    p.add_argument("--rollout-k", type=int, default=64, help="steps per rollout launch (0 = skip)")
    p.add_argument("--train", default="dense64,conv",
                   help="learner workloads to time (comma list of dense64,conv,dense; '' = none)")
    p.add_argument("--train-updates", type=int, default=200)
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--replay", type=int, default=1 << 20)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    return p.parse_args()


# RCCL ("nccl") in production; G2048_BENCH_BACKEND=gloo rehearses several ranks on one GPU
BACKEND = os.environ.get("G2048_BENCH_BACKEND", "nccl")


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a torchrun environment: start N ranks (one process per GPU)
    through torch.distributed.run as a CHILD process -- nothing here has touched the GPU -- and
    return its exit code."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__), *sys.argv[1:]]
    import subprocess

    return subprocess.call(cmd)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1) if world > 1 else 0)
    if world > 1:
        torch.cuda.set_device(dev)
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(BACKEND)
    return world, rank, dev


def barrier(world, dev):
    if world > 1:
        if BACKEND == "nccl":
            dist.barrier(device_ids=[dev.index])
        else:
            dist.barrier()


def max_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return float(t.item())


def capture(fn, n_steps: int):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # one eager call on the side stream before capture
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n_steps):
            fn()
    return g


def bench_env(args, world, rank, dev):
    import g2048

    n = args.boards
    env = g2048.VecEnv2048(n, seed=args.seed, device=dev, board_offset=rank * n)
    reward = torch.empty(n, dtype=torch.int32, device=dev)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    legal = torch.empty(n, dtype=torch.uint8, device=dev)

    def one_step():
        env.step(None, reward=reward, done=done, legal=legal)

    G = max(1, min(args.graph_steps, args.steps))
    graphs = [(capture(one_step, G), args.steps // G)]  # (capture executes one eager step)
    if args.steps % G:
        graphs.append((capture(one_step, args.steps % G), 1))
    # warm-up: the W untimed steps run as graph replays too, so the timed region starts with the
    # GPU already in its steady state (eager launches leave it idle between steps); every captured
    # graph is replayed at least once whatever W is, so the timed region never holds the first
    # replay of a fresh graph
    for g, _ in graphs:
        g.replay()
    for _ in range(args.warmup // G):
        graphs[0][0].replay()
    for _ in range(args.warmup % G):
        one_step()
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for g, reps in graphs:
        for _ in range(reps):
            g.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(world, dev)
    wall = time.perf_counter() - t0
    ev_s = e0.elapsed_time(e1) / 1e3
    wall_max = max_over_ranks(wall, world, dev)

    # single-launch kernel duration (events bracketing one eager launch, median of 200)
    durs = []
    for _ in range(200):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        one_step()
        b.record(stream)
        b.synchronize()
        durs.append(a.elapsed_time(b) / 1e3)
    durs.sort()
    single = durs[len(durs) // 2]
    env.check_errors()
    return dict(wall=wall_max, ev_s=ev_s, single_launch_s=single, n=n, G=G)


def launch_floor(n: int, dev, G: int = 100, reps: int = 20) -> float:
    """Per-launch time of a graph-replayed device copy of the step's board + meta bytes (32 B in,
    32 B out per board): the floor any one-launch-per-step kernel over n boards pays here."""
    src = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    g = capture(lambda: dst.copy_(src), G)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / 1e3 / (G * reps)


def bench_rollout(args, world, rank, dev):
    """K random steps per launch with fused replay append (replay pre-fill path)."""
    import g2048

    n, k = args.boards, args.rollout_k
    env = g2048.VecEnv2048(n, seed=args.seed + 1, device=dev, board_offset=rank * n)
    rb = g2048.ReplayBuffer(n * k, device=dev)
    env.rollout(k, replay=rb)
    torch.cuda.synchronize()
    reps = 20
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        env.rollout(k, replay=rb)
    e1.record(stream)
    torch.cuda.synchronize()
    s = e0.elapsed_time(e1) / 1e3 / reps
    return dict(launch_s=s, steps_per_s=n * k / s, bytes_per_launch=n * k * ROLLOUT_BYTES)


def bench_train(args, world, rank, dev, net):
    """BASELINE configs[2]/[3] (configs[4] at --gpus 8): N boards + Double-DQN, replay 1M,
    B=8192, fp32, graph-captured update with RCCL gradient all-reduce when world > 1.
    Times (a) learner updates alone and (b) the full loop iteration = Q forward of the boards
    on the greedy branch + fused epsilon-greedy step/append + 1 update, early (eps ~ 1) and late
    (eps = min_epsilon) in the schedule."""
    import g2048
    from g2048.learner import DQNLearner, Trainer, flops_per_update

    n = args.boards
    C = max(args.replay // n, 1) * n
    env = g2048.VecEnv2048(n, seed=args.seed + 7, device=dev, board_offset=rank * n)
    rb = g2048.ReplayBuffer(C, device=dev)
    L = DQNLearner(rb, net=net, dtype=torch.float32, batch_size=args.batch, target_sync_every=100)
    T = Trainer(env, rb, L, updates_per_step=1, min_fill=0)
    T.prefill(C // n)  # replay pre-filled by random-policy rollout steps (one launch)
    for _ in range(5):
        T.step()
    L.update()  # the learner's own graph (the Trainer may run a graphed loop): captured here
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    K = args.train_updates
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world, dev)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(K):
        L.update()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(world, dev)
    upd_wall = max_over_ranks(time.perf_counter() - t0, world, dev)
    upd_ev = e0.elapsed_time(e1) / 1e3
    K2 = max(K // 2, 1)
    barrier(world, dev)
    t0 = time.perf_counter()
    for _ in range(K2):
        T.step()
    torch.cuda.synchronize()
    barrier(world, dev)
    loop_wall = max_over_ranks(time.perf_counter() - t0, world, dev)
    # (b) ran at the start of the eps schedule (eps ~ 1: the conv forward runs on the few
    # greedy-branch boards only, the dense step skips all-explore groups).  (c) the same loop
    # late in training: every board past eps_decay_episodes, eps = min_epsilon (Q of ~all boards).
    eps_early = float(T.current_epsilon().mean())
    env.ep[:, 0] = int(T.eps_decay)
    T.step()
    torch.cuda.synchronize()
    eps_late = float(T.current_epsilon().mean())
    barrier(world, dev)
    t0 = time.perf_counter()
    for _ in range(K2):
        T.step()
    torch.cuda.synchronize()
    barrier(world, dev)
    late_wall = max_over_ranks(time.perf_counter() - t0, world, dev)
    loss = float(L.last_loss)
    env.check_errors()
    fl = flops_per_update(net, args.batch)
    return {"updates_per_s": K / upd_wall, "update_ms": upd_ev / K * 1e3,
            "learner_tflops": fl / (upd_ev / K) / 1e12,
            "loop_iter_ms": loop_wall / K2 * 1e3,
            "loop_env_steps_per_s": sum_over_ranks(n * K2 / loop_wall, world, dev),
            "loop_updates_per_s": K2 / loop_wall, "loop_epsilon_mean": eps_early,
            "loop_late_iter_ms": late_wall / K2 * 1e3,
            "loop_late_env_steps_per_s": sum_over_ranks(n * K2 / late_wall, world, dev),
            "loop_late_epsilon_mean": eps_late,
            "batch": args.batch, "replay": C, "dtype": "fp32", "loss": loss,
            "params": L.n_params}


def cpu_baseline(args):
    """The oracle (plain-C restatement of src/board.py + dqn_lib.play_one_step) on ONE host core,
    bounded sample: 4096 boards stepped with random actions for ~args.cpu_seconds."""
    from oracle import oracle as O

    O.build()
    n = 4096
    env = O.OracleEnv(n, seed=args.seed)
    env.step(O.MODE_RANDOM)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        env.step(O.MODE_RANDOM)
        steps += n
    dt = time.perf_counter() - t0
    return dict(value=steps / dt, unit="env steps/s", cores=1, kind="port",
                sample=f"oracle/oracle2048.c random-policy steps, {n} boards x {steps // n} steps "
                       f"({dt:.1f} s, 1 thread)")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world, rank, dev = setup_dist(args)
    torch.cuda.set_device(dev)
    # the extra fields run first: the headline env-step timing then starts on a GPU that has
    # been busy for a while (a cold start measured 2.96 instead of 2.72 us per step)
    ro = bench_rollout(args, world, rank, dev) if args.rollout_k > 0 else None
    if ro:
        ro_total = sum_over_ranks(ro["steps_per_s"], world, dev)
    train = {}
    for net in [x for x in args.train.split(",") if x]:
        train[net] = bench_train(args, world, rank, dev, net)
    r = bench_env(args, world, rank, dev)
    total_steps = sum_over_ranks(r["n"] * args.steps, world, dev)
    value = total_steps / r["wall"]
    per_step_s = r["ev_s"] / args.steps
    achieved = STEP_BYTES * r["n"] / per_step_s / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    traffic, traffic_src = pmc_traffic("k_step", r["n"])
    floor_s = launch_floor(r["n"], dev)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": r["wall"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (fresh boards from Philox spawns, uniform random actions)",
            "config": {"workload": "BASELINE configs[1]: 64k vectorised boards, env-step-only "
                                   "(no learner), random policy",
                       "boards_per_gpu": r["n"], "global_boards": r["n"] * world,
                       "parallelism": f"dp{world} (boards sharded, no collective)",
                       "launch": f"1 g2048_env_step per step, hipGraph of {r['G']} steps"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "k_step<MODE_RANDOM>",
                         "bytes_per_launch": STEP_BYTES * r["n"],
                         "launch_us_graph": per_step_s * 1e6,
                         "launch_us_single_eager": r["single_launch_s"] * 1e6,
                         # at 64k boards the step is bound by the launch floor, not by HBM:
                         "launch_floor_us": floor_s * 1e6,
                         "floor_frac": floor_s / per_step_s},
            "cpu_baseline": cpu,
        }
        if ro:
            line["rollout"] = {"kernel": "k_rollout (K steps/launch, replay append)",
                               "k": args.rollout_k, "env_steps_per_s": ro_total,
                               "launch_ms": ro["launch_s"] * 1e3,
                               "replay_write_GBs": ro["bytes_per_launch"] / ro["launch_s"] / 1e9}
        if train:
            line["learner"] = train
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
