#!/usr/bin/env python3
"""Benchmark of the 2048 hot path on MI355X (contract: DESIGN.md section 6).

Headline (BASELINE.json configs[1]): 65 536 vectorised boards per GPU, env step only, uniform
random actions drawn in-kernel from Philox.  One bench "step" = one g2048_env_rollout launch that
moves every board `--rollout-k` (64) times and appends each transition (s, a, r, s', done) to an
HBM replay ring of N * K rows -- the fused play_one_step + deque.append of src/dqn_lib.py:91-107
with the boards resident in VGPRs.  value = env steps/s over all ranks = N * K * world * steps /
(max over ranks of the timed wall time).

Extra fields: the one-launch-per-step kernel (g2048_env_step, hipGraph-replayed) at the same N,
DQN updates/s + full training-loop iterations at B = 8192 for the dense-64 / conv / dense-ref
nets in fp32 (fused HIP kernels where they exist) and fp64 (the reference's precision), the CPU
baselines (oracle env on every host core; the reference train_step in fp64 on torch CPU).

Multi-GPU: one process per GPU (`--gpus N` starts them through torch.distributed.run when no
torchrun environment is present), boards sharded by board_offset = rank * N, no collective on
the env path (weak scaling), the learner's gradients all-reduced over RCCL.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "2048 env steps/sec + DQN updates/sec at 64k parallel boards, 1→8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TF = 157.3   # dense f32 (vector / MFMA) peak, MI355X_MICROARCH.md
FP64_PEAK_TF = 78.6    # dense f64 peak
# Algorithmic bytes per env step:
#   rollout (the headline kernel): the replay append s 16 + s' 16 + a 1 + r 4 + d 1 = 38 B; the
#   board / meta / episode counters are read and written once per launch (not per step)
ROLLOUT_BYTES = 38
#   one launch per step, random mode: board 16 R + 16 W + reward 4 + done 1 = 37 B;
#   with the bookkeeping the kernel moves as well (the score row 4 R + 4 W, legal 1): 46 B --
#   54 B up to ABI v4, whose meta held {score, moves} per board (8 R + 8 W every step)
STEP_BYTES = 37
STEP_BYTES_BOOKKEEPING = 46
PROFILE_DIR = os.path.join(ROOT, "profiles", "r06")
PMC_FILE = os.path.join(PROFILE_DIR, "pmc.json")
# the learner kernels' PMC passes (tools/gpu_pmc_learner.sh -> tools/pmc_learner.py)
PMC_LEARNER_FILE = os.path.join(ROOT, "profiles", "r06", "pmc_learner.json")
# the kernels of one update of each fused learner (the per-update launches; k_pack / k_adam run
# only at setup or on the data-parallel path)
UPDATE_KERNELS = {
    ("conv", "fp64"): ("k_conv64_train_a", "k_conv64_train_b", "k_conv64_reduce"),
    ("conv", "fp32"): ("k_conv_targets_persist", "k_conv_train_fwd", "k_conv_train_bwd",
                       "k_reduce_pre"),
    ("dense", "fp64"): ("k_dense_sample", "k_dense_forward", "k_dense_rows", "k_dense_wgrad",
                        "k_dense_reduce"),
    ("dense", "fp32"): ("k_dense_sample", "k_dense_forward", "k_dense_rows", "k_dense_wgrad",
                        "k_dense_reduce"),
    ("dense64", "fp32"): ("k_mlp_update", "k_mlp_reduce"),
    ("dense64", "fp64"): ("k_dense64_update_f64", "k_dense64_reduce_f64"),
}
INFINITY_CACHE_BYTES = 256 << 20  # MI355X_MICROARCH.md: die-level L3, 256 MiB
RESIDENCY_RULE = ("MI355X_MICROARCH.md, Infinity Cache: a line stays resident while everything "
                  "loaded or stored between two uses of it fits in about 256 MiB")


def pmc_record(key: str):
    """Memory-side bytes per launch (+ issue counters) of one kernel@shape from the committed
    rocprofv3 PMC passes (tools/gpu_pmc.sh: separate FETCH_SIZE / WRITE_SIZE / SQ passes, run as
    their own rocprofv3 commands -- NOT measured by this process), with the file's provenance."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    r = d.get(key)
    if r is not None:
        r = dict(r, source=f"{os.path.relpath(PMC_FILE, ROOT)} ({d.get('_provenance', 'rocprofv3 --pmc passes, tools/gpu_pmc.sh')})")
    return r


def traffic_fields(rec, algorithmic: float) -> dict:
    """`traffic` (bytes per launch from the committed PMC passes) and where it came from."""
    if not rec or "hbm_bytes_per_launch" not in rec:
        return {"traffic": None, "traffic_source": None}
    t = rec["hbm_bytes_per_launch"]
    return {"traffic": t, "traffic_over_algorithmic": t / algorithmic,
            "traffic_source": rec["source"] + "; FETCH_SIZE + WRITE_SIZE at the memory side of "
                              "L2 (Infinity-Cache hits included), per launch"}


def learner_algorithmic_bytes(batch: int, params: int, elt: int) -> int:
    """Bytes one update must move (learner): the B sampled transitions (s, s' 16 + 16,
    a 1, r 4, d 1 = 38 B each), both nets' weights read once, Adam's moments and the parameters
    read and written (m, v, p: 6 x params), and the rows / targets written (8 + elt per sample)."""
    return batch * (38 + 8 + elt) + params * elt * (2 + 6)


def learner_roofline(net: str, dtype: str, batch: int, update_s: float, params: int,
                     algo_flop: float, peak_tf: float) -> dict:
    """The roofline object of one learner leg: bound "mfma" (the update is GEMM-shaped work on
    f32 / f64 MFMA); achieved = the ALGORITHMIC FLOPs (5 forward-equivalents of the direct net,
    SURVEY 8d) over the event-timed update; executed_mfma_flop = the matrix FLOPs the kernels
    really issue (Winograd conv2 issues fewer; 0 for the dense-64 f64 update, which runs on VALU),
    and traffic = FETCH + WRITE bytes of the update's kernels, both from the committed PMC passes
    (profiles/r06/pmc_learner.json, a separate rocprofv3 run)."""
    elt = 4 if dtype == "fp32" else 8
    algo_b = learner_algorithmic_bytes(batch, params, elt)
    out = {"bound": "mfma", "achieved": algo_flop / update_s / 1e12, "peak": peak_tf,
           "unit": "TFLOP/s", "frac": algo_flop / update_s / 1e12 / peak_tf,
           "algorithmic_flop": algo_flop, "algorithmic_bytes": algo_b, "update_us": update_s * 1e6,
           "executed_mfma_flop": None, "traffic": None}
    try:
        with open(PMC_LEARNER_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return out
    tag = f"{net}.{dtype}@{batch}"
    recs = {k: d.get(f"{k}@{tag}") for k in UPDATE_KERNELS.get((net, dtype), ())}
    if not recs or any(r is None for r in recs.values()):
        return out
    if all("hbm_bytes_per_launch" in r for r in recs.values()):
        t = sum(r["hbm_bytes_per_launch"] for r in recs.values())
        out.update(traffic=t, traffic_over_algorithmic=t / algo_b,
                   traffic_per_kernel={k: r["hbm_bytes_per_launch"] for k, r in recs.items()})
    if all("mfma_flop" in r for r in recs.values()):
        ex = sum(r["mfma_flop"] for r in recs.values())
        out.update(executed_mfma_flop=ex, executed_mfma_tflops=ex / update_s / 1e12,
                   executed_mfma_frac=ex / update_s / 1e12 / peak_tf)
    out["traffic_source"] = (f"{os.path.relpath(PMC_LEARNER_FILE, ROOT)} "
                             f"({d.get('_provenance', '')}); kernels {', '.join(recs)}")
    return out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200, help="timed rollout launches")
    p.add_argument("--warmup", type=int, default=20, help="untimed rollout launches")
    p.add_argument("--boards", type=int, default=65536)
    p.add_argument("--rollout-k", type=int, default=64, help="env steps per rollout launch")
    p.add_argument("--rollout-k-extra", default="256",
                   help="further K values timed beside the headline (rollout_k_sweep field)")
    p.add_argument("--large-n", default="4194304x16",
                   help="boards x K of a large-N rollout timed beside the headline "
                        "(rollout_large_n field; '' skips it)")
    p.add_argument("--hbm-ring-launches", type=int, default=8,
                   help="rollout_64k_hbm leg: the headline launch into a ring of this many "
                        "launches' rows (> 256 MiB: streamed to HBM); 0 or 1 skips it")
    p.add_argument("--step-steps", type=int, default=2000,
                   help="timed one-launch-per-step env steps (0 = skip that leg)")
    p.add_argument("--graph-steps", type=int, default=100)
    p.add_argument("--settle-ms", type=float, default=60.0,
                   help="untimed back-to-back replays of the timed graph before each timed region "
                        "(the clock ramps over the first ~10 ms of load; see DESIGN 6)")
    p.add_argument("--seed", type=int, default=0x2048)
    p.add_argument("--train", default="dense64,conv,dense,dense@5000",
                   help="learner legs to time: comma list of dense64 / conv / dense, each "
                        "optionally @batch (default --batch); '' = none")
    p.add_argument("--train-dtypes", default="fp32,fp64")
    p.add_argument("--train-updates", type=int, default=200)
    p.add_argument("--batch", type=int, default=8192)
    p.add_argument("--replay", type=int, default=1 << 20)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=8.0)
    return p.parse_args()


# RCCL ("nccl") in production; G2048_BENCH_BACKEND=gloo rehearses several ranks on one GPU
BACKEND = os.environ.get("G2048_BENCH_BACKEND", "nccl")
CTRL = None  # gloo side group (setup_dist): the ranks' agreement on a failed learner leg
CTRL_TIMEOUT_S = float(os.environ.get("G2048_BENCH_CTRL_TIMEOUT_S", "600"))


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a torchrun environment: start N ranks (one process per GPU)
    through torch.distributed.run as a CHILD process -- nothing here has touched the GPU -- and
    return its exit code."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def pick_device(local: int, world: int, backend: str, n_dev: int) -> int:
    """The GPU index of local rank `local`.  Under RCCL ("nccl") every rank needs its own GPU:
    more ranks than visible devices is refused (RCCL cannot put two ranks on one device, and
    stacking them would silently measure a different workload).  The gloo rehearsal
    (G2048_BENCH_BACKEND=gloo) may share devices round-robin."""
    if world == 1:
        return 0
    if backend == "nccl":
        if local >= n_dev or world > n_dev:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} ranks under RCCL but only {n_dev} "
                             "visible GPU(s): one rank per GPU is required")
        return local
    return local % max(n_dev, 1)


def setup_dist(args):
    """One process per GPU.  world > 1: an RCCL ("nccl") process group (gloo in the one-GPU
    rehearsal), plus a gloo side group for the ranks' agreement on a failed leg.  G2048_BENCH_DIST=1
    at world 1 builds the same groups around ONE rank, so every distributed path of this file --
    the RCCL barrier, max-over-ranks, thread-local captures, the learner's captured SUM all-reduce
    with 1 / world in Adam, the fixed-count settle and the GPU all_gather of the lockstep check --
    runs on a one-GPU box before the driver's multi-GPU run (tests/test_bench_rccl_gpu.py)."""
    global CTRL
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", pick_device(local, world, BACKEND, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1 or os.environ.get("G2048_BENCH_DIST") == "1":
        if world == 1:  # a one-rank group: a local rendezvous of its own
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(BACKEND)
        # control plane on the host: a rank whose learner leg failed may have left the RCCL
        # communicator unusable (or its peers blocked in a replayed collective)
        CTRL = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=CTRL_TIMEOUT_S))
    return world, rank, dev


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def barrier(world, dev):
    if distributed():
        if BACKEND == "nccl":
            dist.barrier(device_ids=[dev.index])
        else:
            dist.barrier()


def max_over_ranks(x: float, world: int, dev) -> float:
    if not distributed():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int, dev) -> float:
    if not distributed():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return float(t.item())


def any_rank_failed(failed: bool) -> bool:
    """The ranks' agreement after a learner leg, over the gloo side group: True if ANY rank
    failed it.  A rank whose peers never arrive (one of them failed and the others are blocked in
    a collective it will not join) times out here after CTRL_TIMEOUT_S and exits non-zero, which
    makes torch.distributed.run stop every rank: the job fails loudly instead of hanging."""
    if CTRL is None:
        return failed
    t = torch.tensor([1 if failed else 0], dtype=torch.int32)
    try:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=CTRL)
    except Exception as e:  # noqa: BLE001 -- a timeout or a dead peer
        print(f"bench.py rank {dist.get_rank()}: no agreement on the learner leg ({e}); "
              "exiting non-zero", file=sys.stderr, flush=True)
        os._exit(3)
    return bool(t.item())


def timed(world, dev, fn, reps: int):
    """(max-over-ranks wall seconds, this rank's HIP-event seconds) of `reps` calls of fn,
    bracketed by a barrier + synchronize on both sides; the events sit on the stream the
    kernels are launched on (torch's current stream, which the g2048 wrappers use)."""
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(world, dev)
    wall = time.perf_counter() - t0
    return max_over_ranks(wall, world, dev), e0.elapsed_time(e1) / 1e3


def settle(replay, ms: float, max_calls: int = 4000) -> float:
    """Keep the GPU busy with `replay` (untimed) for at least `ms` of wall time, so the timed
    region starts at the clock a sustained run holds: gfx950 ramps its clock over the first
    ~10 ms of load (64k-board rollout: 30.3 us per launch right after a short warm-up, 27.4 us
    after ~10 ms).  Returns the wall milliseconds spent."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    calls = 0
    while (time.perf_counter() - t0) * 1e3 < ms and calls < max_calls:
        replay()
        calls += 1
        if calls % 8 == 0:
            torch.cuda.synchronize()  # pace the host: the queue stays short
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def capture(fn, n_steps: int):
    """A hipGraph of n_steps calls of fn (g2048/dist.py: graph_capture -- thread-local in a
    process holding an RCCL group, whose watchdog thread queries events while this thread
    records; no garbage collection during the capture)."""
    from g2048.dist import graph_capture, quiesce_for_capture

    quiesce_for_capture()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # one eager call on the side stream before capture
    torch.cuda.current_stream().wait_stream(s)
    with graph_capture(g):
        for _ in range(n_steps):
            fn()
    return g


# ------------------------------------------------------------------ headline: the rollout kernel
def bench_rollout(args, world, rank, dev, k_override=None, n_override=None, ring_launches=1):
    """W untimed + `steps` timed k_rollout launches (K env steps of every board each, replay
    append into an N*K*ring_launches-row ring), replayed from hipGraphs of --graph-steps launches
    (the kernel reads its step clock and ring row from device memory, so a replay is a fresh
    rollout): back to back on the GPU, so the events' time per launch is the kernel's own duration
    (what rocprofv3 --kernel-trace reports), not kernel + host enqueue gap.  With ring_launches R
    > 1 each launch writes ring rows the previous R - 1 launches did not touch."""
    import g2048

    n = args.boards if n_override is None else n_override
    k = args.rollout_k if k_override is None else k_override
    env = g2048.VecEnv2048(n, seed=args.seed, device=dev, board_offset=rank * n)
    rb = g2048.ReplayBuffer(n * k * ring_launches, device=dev)

    def launch():
        env.rollout(k, replay=rb)

    steps = args.steps
    G = max(1, min(args.graph_steps, steps))
    graphs = [(capture(launch, G), steps // G)]
    if steps % G:
        graphs.append((capture(launch, steps % G), 1))
    for g, _ in graphs:  # no timed replay is the first replay of its graph
        g.replay()
    for _ in range(max(args.warmup, 1)):
        launch()
    settle_ms = settle(graphs[0][0].replay, args.settle_ms)

    def run_all():
        for g, reps in graphs:
            for _ in range(reps):
                g.replay()

    wall, ev = timed(world, dev, run_all, 1)
    env.check_errors()
    assert int(rb.count) == n * k * ring_launches
    # the bytes a launch's lines see between two uses: the ring (rows of R launches) + env state
    ws = ROLLOUT_BYTES * n * k * ring_launches + n * (16 + 8 + 16) + 8 * ((n + 63) // 64)
    return dict(wall=wall, ev_s=ev, n=n, k=k, settle_ms=settle_ms, board_offset=rank * n,
                working_set=ws)


def rollout_roofline(r, steps, rec):
    """The roofline object of one rollout leg: algorithmic 38 B per env step over the HIP-event
    launch time.  bound "hbm" only when the working set exceeds the Infinity Cache (else the
    bytes need never reach HBM and the launch is bound by instruction issue)."""
    launch_s = r["ev_s"] / steps
    algo = ROLLOUT_BYTES * r["n"] * r["k"]
    achieved = algo / launch_s / 1e9
    # the same bytes over the wall time per launch that `value` / `ms_per_step` use (host clock
    # around the whole timed region: graph launch latency and the final sync included)
    wall_s = r["wall"] / steps
    hbm = r["working_set"] > INFINITY_CACHE_BYTES
    out = {"bound": "hbm" if hbm else "issue",
           "resident": "hbm-streamed" if hbm else "infinity-cache",
           "working_set_bytes": r["working_set"], "residency_rule": RESIDENCY_RULE,
           "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS,
           "frac_source": ("HIP events on the kernel's stream around the timed launches (the "
                           "kernel's own duration, as rocprofv3 reports it); `frac_wall` is the "
                           "same bytes over ms_per_step, the clock `value` uses"),
           "frac_events": achieved / HBM_PEAK_GBS,
           "frac_wall": algo / wall_s / 1e9 / HBM_PEAK_GBS,
           "launch_us_wall": wall_s * 1e6,
           "frac_note": ("of the HBM spec; the bytes stream to HBM" if hbm else
                         "algorithmic bytes over the HBM spec, but the working set stays in the "
                         "Infinity Cache: not an HBM-bandwidth claim (see `issue`)"),
           "bytes_per_step": ROLLOUT_BYTES, "bytes_per_launch": algo,
           "launch_us": launch_s * 1e6, "settle_ms": r["settle_ms"]}
    out.update(traffic_fields(rec, algo))
    if rec and rec.get("issue"):
        out["issue"] = rec["issue"]
    return out


# ------------------------------------------------------------------ one launch per step
def bench_step(args, world, rank, dev):
    """g2048_env_step (random actions, reward / done / legal outputs) replayed from hipGraphs of
    --graph-steps launches; every captured graph is replayed once before the timed region."""
    import g2048

    n, steps = args.boards, args.step_steps
    env = g2048.VecEnv2048(n, seed=args.seed + 1, device=dev, board_offset=rank * n)
    reward = torch.empty(n, dtype=torch.int32, device=dev)
    done = torch.empty(n, dtype=torch.uint8, device=dev)
    legal = torch.empty(n, dtype=torch.uint8, device=dev)

    def one_step():
        env.step(None, reward=reward, done=done, legal=legal)

    G = max(1, min(args.graph_steps, steps))
    graphs = [(capture(one_step, G), steps // G)]
    if steps % G:
        graphs.append((capture(one_step, steps % G), 1))
    for g, _ in graphs:  # warm: no timed replay is the first replay of its graph
        g.replay()
    for _ in range(3):
        graphs[0][0].replay()
    settle(graphs[0][0].replay, args.settle_ms)

    def run_all():
        for g, reps in graphs:
            for _ in range(reps):
                g.replay()

    wall, ev = timed(world, dev, run_all, 1)
    env.check_errors()
    # the launch floor here: a graph-replayed device copy of the kernel's board + score bytes
    src = torch.zeros((n, 20), dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    gf = capture(lambda: dst.copy_(src), 100)
    gf.replay()
    _, fl = timed(1, dev, gf.replay, 20)
    per = ev / steps
    return {"kernel": "k_step<MODE_RANDOM> (g2048_env_step, one launch per env step)",
            "env_steps_per_s": sum_over_ranks(n * steps / wall, world, dev),
            "launch_us_graph": per * 1e6,
            "launch_floor_us": fl / 2000 * 1e6,
            "bytes_per_step": STEP_BYTES,
            "bytes_per_step_with_bookkeeping": STEP_BYTES_BOOKKEEPING,
            "hbm_frac": STEP_BYTES * n / per / 1e9 / HBM_PEAK_GBS,
            "note": "launch-bound at 64k boards (2.4 MB per launch): compare the launch floor"}


# ------------------------------------------------------------------ learner
def bench_train(args, world, rank, dev, net, dtype, batch):
    """BASELINE configs[2]/[3] (configs[4] at --gpus 8): N boards + Double-DQN, replay 1M,
    B = 8192, gradient all-reduce over RCCL when world > 1.  (a) learner updates alone,
    (b) the training-loop iteration = Q of the greedy-branch boards + fused eps-greedy step /
    append + 1 update, early (eps ~ 1) and late (eps = min_epsilon) in the schedule."""
    import g2048
    from g2048.learner import DQNLearner, Trainer, flops_per_update

    n = args.boards
    C = max(args.replay // n, 1) * n
    env = g2048.VecEnv2048(n, seed=args.seed + 7, device=dev, board_offset=rank * n)
    rb = g2048.ReplayBuffer(C, device=dev)
    tdt = torch.float32 if dtype == "fp32" else torch.float64
    # in a process group (also a one-rank one, G2048_BENCH_DIST=1): the data-parallel update, with
    # the gradient SUM all-reduce captured in the update's graph under RCCL
    L = DQNLearner(rb, net=net, dtype=tdt, batch_size=batch, target_sync_every=100,
                   data_parallel=True if distributed() else None)
    T = Trainer(env, rb, L, updates_per_step=1, min_fill=0)
    T.prefill(C // n)  # replay pre-filled by random-policy rollout steps (one launch)
    for _ in range(5):
        T.step()
    L.update()  # the learner's own graphs (the Trainer may run a graphed loop): captured here
    torch.cuda.synchronize()
    K = args.train_updates if dtype == "fp32" else max(args.train_updates // 4, 10)
    # untimed updates for --settle-ms (the clock ramp, as for the rollout legs: a fp64 conv update
    # timed right after a short warm-up reads ~160 us, sustained ~151 us)
    if not distributed():
        settle_ms = settle(L.update, args.settle_ms, max_calls=2000)
    else:  # every rank must run the same number of updates (each holds a collective)
        t0 = time.perf_counter()
        for _ in range(int(args.settle_ms)):  # one update per settle ms
            L.update()
        torch.cuda.synchronize()
        settle_ms = (time.perf_counter() - t0) * 1e3
    upd_wall, upd_ev = timed(world, dev, L.update, K)
    K2 = max(K // 2, 1)
    loop_wall, _ = timed(world, dev, T.step, K2)
    eps_early = float(T.current_epsilon().mean())
    env.ep[:, 0] = int(T.eps_decay)  # every board past the decay: eps = min_epsilon
    T.step()
    torch.cuda.synchronize()
    eps_late = float(T.current_epsilon().mean())
    late_wall, _ = timed(world, dev, T.step, K2)
    loss = float(L.last_loss)
    env.check_errors()
    lockstep = None
    if distributed():  # the replicas (online + target nets) must agree bit for bit on every rank
        flat = torch.cat([p.detach().reshape(-1) for p in
                          list(L.model.parameters()) + list(L.target.parameters())])
        flat = flat if BACKEND == "nccl" else flat.cpu()
        got = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(got, flat)
        lockstep = all(torch.equal(got[0], g) for g in got[1:])
    fl = flops_per_update(net, batch)
    peak = FP32_PEAK_TF if dtype == "fp32" else FP64_PEAK_TF
    tf = fl / (upd_ev / K) / 1e12
    return {"updates_per_s": K / upd_wall, "update_ms": upd_ev / K * 1e3,
            "learner_tflops": tf, "flop_frac": tf / peak, "peak_tflops": peak,
            "path": ("fused HIP kernels" if L.fused else "torch-ROCm GEMMs after the HIP "
                     "gather+encode kernel"),
            "loop_iter_ms": loop_wall / K2 * 1e3,
            "loop_env_steps_per_s": sum_over_ranks(n * K2 / loop_wall, world, dev),
            "loop_updates_per_s": K2 / loop_wall, "loop_epsilon_mean": eps_early,
            "loop_late_iter_ms": late_wall / K2 * 1e3,
            "loop_late_env_steps_per_s": sum_over_ranks(n * K2 / late_wall, world, dev),
            "loop_late_epsilon_mean": eps_late,
            "batch": batch, "replay": C, "dtype": dtype, "loss": loss, "settle_ms": settle_ms,
            "params": L.n_params, "graphed_loop": T.graph, "ranks_lockstep": lockstep,
            "data_parallel": L.dp, "captured_allreduce": L.capture_collective,
            "grad_scale": L.grad_scale,
            "roofline": learner_roofline(net, dtype, batch, upd_ev / K, L.n_params, fl, peak)}


# ------------------------------------------------------------------ CPU baselines
def cpu_baselines(args):
    """The oracle env on every host core + the reference train_step in fp64 on torch CPU
    (oracle/cpu_baseline.py; its C library was built by __graft_entry__.build())."""
    from oracle import cpu_baseline as CB

    env = CB.env_baseline(args.cpu_seconds)
    env["learner"] = [CB.learner_baseline("conv", b, updates=2) for b in (5000, 8192)]
    # BASELINE configs[0]: the dense net at its own batch (src/configs/double_dqn_dense.py:17)
    env["learner"].append(CB.learner_baseline("dense", 5000, updates=2))
    return env


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world, rank, dev = setup_dist(args)
    ro = bench_rollout(args, world, rank, dev)
    n, k = ro["n"], ro["k"]
    value = n * k * world * args.steps / ro["wall"]
    ranges = [[ro["board_offset"], n]]
    if distributed():  # every rank's global board range: disjoint Philox subsequences
        got = [None] * world
        dist.all_gather_object(got, ranges[0])
        ranges = got
    # the same launch at further K: a launch's first steps run slower than its steady state
    # (DESIGN.md 4.2), so the per-step time falls with K
    ksweep = []
    for kx in [int(x) for x in args.rollout_k_extra.split(",") if x]:
        rx = bench_rollout(args, world, rank, dev, k_override=kx)
        lx = rx["ev_s"] / args.steps
        ksweep.append({"k": kx, "env_steps_per_s": n * kx * world * args.steps / rx["wall"],
                       "launch_us": lx * 1e6, "frac": ROLLOUT_BYTES * n * kx / lx / 1e9 / HBM_PEAK_GBS,
                       "resident": "infinity-cache" if rx["working_set"] <= INFINITY_CACHE_BYTES
                       else "hbm-streamed"})
    # the headline launch (64k boards x K) into a ring of --hbm-ring-launches launches' rows:
    # every launch writes rows the previous ones did not, so the ring streams to HBM
    hbm64 = None
    if args.hbm_ring_launches > 1:
        rh = bench_rollout(args, world, rank, dev, ring_launches=args.hbm_ring_launches)
        hbm64 = {"boards_per_gpu": n, "k": k, "ring_rows": n * k * args.hbm_ring_launches,
                 "kernel": "k_rollout_lean",
                 "env_steps_per_s": n * k * world * args.steps / rh["wall"],
                 "roofline": rollout_roofline(rh, args.steps, pmc_record(
                     f"k_rollout@{n}x{k}r{args.hbm_ring_launches}"))}
        torch.cuda.empty_cache()
    # the same launch at large N (boards x K): past 256k boards the ring streams to HBM and
    # g2048_env_rollout dispatches the warp-specialised k_rollout_ws
    large = None
    if args.large_n:
        nl, _, kl = args.large_n.partition("x")
        nl, kl = int(nl), int(kl or 16)
        rl = bench_rollout(args, world, rank, dev, k_override=kl, n_override=nl)
        kern = "k_rollout_ws" if nl >= (1 << 18) else "k_rollout_lean"
        roof = rollout_roofline(rl, args.steps, pmc_record(f"{kern}@{nl}x{kl}"))
        large = {"boards_per_gpu": nl, "k": kl, "kernel": kern,
                 "env_steps_per_s": nl * kl * world * args.steps / rl["wall"],
                 "launch_us": roof["launch_us"], "achieved_GBs": roof["achieved"],
                 "frac": roof["frac"], "roofline": roof}
        torch.cuda.empty_cache()
    step = bench_step(args, world, rank, dev) if args.step_steps > 0 else None
    train = {}
    failed = False
    for leg in [x for x in args.train.split(",") if x]:
        net, _, b = leg.partition("@")  # "dense@5000": that net at that batch
        for dt in [x for x in args.train_dtypes.split(",") if x]:
            if failed:
                train[f"{leg}.{dt}"] = {"error": "skipped after an earlier learner leg failed"}
                continue
            mine = False
            try:
                train[f"{leg}.{dt}"] = bench_train(args, world, rank, dev, net, dt,
                                                   int(b) if b else args.batch)
            except Exception as e:
                # one process without a group fails loudly.  In a process group the learner legs
                # are the only ones that capture RCCL collectives: the failing leg is reported in
                # the line and the remaining learner legs are skipped on EVERY rank (agreed over
                # the gloo side group), so the env-step headline measured above still prints
                if not distributed():
                    raise
                traceback.print_exc()
                train[f"{leg}.{dt}"] = {"error": f"{type(e).__name__}: {e}"[:400]}
                mine = True
            if any_rank_failed(mine):
                failed = True
                if not mine:
                    train[f"{leg}.{dt}"] = {"error": "failed on another rank",
                                            "this_rank": train[f"{leg}.{dt}"]}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baselines(args)
    roof = rollout_roofline(ro, args.steps, pmc_record(f"k_rollout@{n}x{k}"))
    roof["kernel"] = ("k_rollout_lean (g2048_env_rollout: ring in one buffer window, auto-reset, "
                      "no episode log)")
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ro["wall"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (fresh boards from Philox spawns, uniform random actions)",
            "config": {"workload": "BASELINE configs[1]: 64k vectorised boards per GPU, env step "
                                   "only (no learner), random policy; one step = one rollout "
                                   f"launch moving every board {k} times with replay append",
                       "boards_per_gpu": n, "global_boards": n * world,
                       "env_steps_per_launch": n * k, "replay_rows": n * k,
                       "rank_boards": ranges,
                       "parallelism": f"dp{world} (boards sharded, no collective)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "dist": {"process_group": distributed(),
                     "backend": dist.get_backend() if distributed() else None,
                     "capture_error_mode": _capture_mode_name()},
        }
        if hbm64:
            line["rollout_64k_hbm"] = hbm64
        if ksweep:
            line["rollout_k_sweep"] = ksweep
        if large:
            line["rollout_large_n"] = large
        if step:
            line["step_kernel"] = step
        if train:
            line["learner"] = train
        print(json.dumps(line), flush=True)
    if distributed():
        dist.destroy_process_group()


def _capture_mode_name() -> str:
    from g2048.dist import capture_error_mode
    return capture_error_mode()


if __name__ == "__main__":
    main()
