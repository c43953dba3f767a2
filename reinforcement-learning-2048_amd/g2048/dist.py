"""Data-parallel plumbing for the learner (one process per GPU, RCCL over xGMI).

The reference is single-process (no distributed backend).  The build shards the
BOARDS across ranks (board_offset = rank * N, no exchange on the env path) and keeps one learner
replica per rank whose gradients are averaged with ONE all-reduce of a flat bucket per update:
conv 33 476 params = 134 KB fp32, dense-64 5.4 KB, dense-ref 1.6 MB -- all latency-bound on
xGMI, so a single bucket (one ring pass) beats per-tensor collectives.
Backend-agnostic: the CPU tests run it over gloo.
"""
from __future__ import annotations

import contextlib
import gc
import os

import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None):
    """torchrun-style init (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*).  Returns
    (world, rank, device).  backend None -> "nccl" (RCCL) when a GPU is visible, else "gloo"."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if use_gpu:
            torch.cuda.set_device(dev)
            dist.init_process_group(backend or "nccl", device_id=dev)
        else:
            dist.init_process_group(backend or "gloo")
    return world, rank, dev


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def broadcast_params(model: torch.nn.Module, src: int = 0, group=None) -> None:
    """Identical initial weights on every rank (target nets then stay in lockstep)."""
    if world_size(group) > 1:
        with torch.no_grad():
            for p in model.parameters():
                dist.broadcast(p.data, src=src, group=group)


class FlatGradBucket:
    """All parameter .grad tensors as views of ONE flat buffer, so zeroing and the gradient
    all-reduce are single operations (and stay valid inside a captured hipGraph)."""

    def __init__(self, model: torch.nn.Module, dtype=None):
        params = list(model.parameters())
        self.params = params
        self.numel = sum(p.numel() for p in params)
        dtype = dtype or params[0].dtype
        self.flat = torch.zeros(self.numel, dtype=dtype, device=params[0].device)
        off = 0
        for p in params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero_(self):
        self.flat.zero_()

    def allreduce_mean_(self, group=None) -> None:
        w = world_size(group)
        if w > 1:
            dist.all_reduce(self.flat, group=group)
            self.flat.div_(w)

    def allreduce_sum_(self, group=None) -> None:
        """The SUM all-reduce alone (also at world 1: the captured data-parallel update is tested
        on one GPU with a world-1 RCCL group); the caller's Adam applies 1 / world."""
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(self.flat, group=group)

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * self.flat.element_size()


def captures_collectives(group=None) -> bool:
    """Whether the gradient all-reduce can be captured into the update's hipGraph: RCCL (the
    "nccl" backend on ROCm) launches its collective kernels on the caller's stream, so a graph
    replays them; gloo runs on the host and stays between two graph replays."""
    return (dist.is_available() and dist.is_initialized()
            and dist.get_backend(group) == dist.Backend.NCCL)


def nccl_group_exists() -> bool:
    """Whether this process holds a ProcessGroupNCCL (RCCL) default group."""
    return (dist.is_available() and dist.is_initialized()
            and dist.get_backend() == dist.Backend.NCCL)


def capture_error_mode(group=None) -> str:
    """torch.cuda.graph's capture_error_mode for ANY hipGraph captured in this process.

    ProcessGroupNCCL's watchdog thread polls the events of every eager collective
    (hipEventQuery, ~every 100 ms) until it sees them complete.  Under a "global"-mode capture
    that query, made by another thread, is an unsafe call: it invalidates the capture
    (hipErrorStreamCaptureInvalidated) and fails in the watchdog ("operation not permitted when
    stream is capturing"), which then tears the process group down -- seen in round 5 on a
    global-mode capture next to a world-1 RCCL group.  "thread_local" confines the capture's
    rules to the capturing thread, so the watchdog's queries are legal whenever they land.  So
    every capture in a process that holds an NCCL group is thread-local; elsewhere torch's
    default "global" (which also catches an unsafe call from a helper thread of ours)."""
    return "thread_local" if (captures_collectives(group) or nccl_group_exists()) else "global"


@contextlib.contextmanager
def graph_capture(graph: "torch.cuda.CUDAGraph", group=None, **kw):
    """torch.cuda.graph(graph) for every capture of this package: the capture-error mode of
    capture_error_mode(), and no garbage collection while it records.  A collection that runs in
    the middle of a capture can free an OLD graph (an earlier learner's, a bench leg's) whose
    destructor calls hipGraphExecDestroy -- an unsafe call in any capture mode on the capturing
    thread, which invalidates the capture ("operation failed due to a previous error during
    capture"; seen once in the round-6 driver command's conv leg).  So: collect first, then keep
    the collector off until the capture ends."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph, capture_error_mode=capture_error_mode(group), **kw):
            yield graph
    finally:
        if was:
            gc.enable()


def quiesce_for_capture(group=None) -> None:
    """Before a hipGraph capture in an RCCL process: drain the device, so the side-stream warm-up
    (and its eager collectives) are complete when the capture starts.  The watchdog race itself
    is closed by the thread-local capture mode (capture_error_mode), not by waiting."""
    if captures_collectives(group) or nccl_group_exists():
        torch.cuda.synchronize()


def shard_offset(rank: int, boards_per_rank: int) -> int:
    """Global id of a rank's first board: Philox subsequences never overlap across ranks."""
    return rank * boards_per_rank
