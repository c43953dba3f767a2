"""A* replay pre-fill (src/state_space_search.py), host search + device ring.

`A_star` mirrors the reference's A_star (:46-101) on one board: best-first on
-merge_score // 2 with the reference's tie, closed-list and child-order rules (the search
runs in C++ in libg2048.so, `g2048_astar_search`; see csrc/g2048_astar.hip).
`generate_replay_buffer_using_A_star` mirrors :103-131: one fresh board per game, search, trace
the path back, and append its transitions to a device ReplayBuffer.

The reference appends (child board, move, parent score - child score, child board, done = 0)
-- s' = s, a negated reward and no terminal flag ("buggy in the reference").
`compat=True` (default) reproduces that; `compat=False` appends the intended transitions
(parent board, move, merge gain, child board, done = child has no legal move).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as N

SPAWN = {"philox": N.ASTAR_SPAWN_PHILOX, "first-empty": N.ASTAR_SPAWN_FIRST_EMPTY}


def A_star(board, goal_tile: int = 2048, seed: int = 0, game: int = 0, spawn: str = "philox",
           start_score: int = 0, max_expansions: int = 0, max_path: int = 1 << 16) -> dict:
    """board: 16 log2 exponents (row-major) or a 4x4 array of tile values; goal_tile: a tile
    value (power of two).  Returns the reference's result fields plus the path:
    success, path_length (inf when not found), visited_nodes, expanded_nodes, and
    path_boards u8[len + 1, 16] (exponents, root first), path_moves u8[len], path_scores."""
    b = np.asarray(board).reshape(16)
    if b.max(initial=0) > 31:  # tile values -> exponents
        nz = b > 0
        e = np.zeros(16, np.uint8)
        e[nz] = np.log2(b[nz]).astype(np.uint8)
        b = e
    b = np.ascontiguousarray(b, dtype=np.uint8)
    goal_exp = int(goal_tile).bit_length() - 1
    if goal_tile <= 1 or (1 << goal_exp) != goal_tile:
        raise ValueError("goal_tile must be a power of two >= 2")
    if spawn not in SPAWN:
        raise ValueError(f"spawn must be one of {sorted(SPAWN)}")
    pb = np.zeros((max_path + 1, 16), np.uint8)
    pm = np.zeros(max_path, np.uint8)
    ps = np.zeros(max_path + 1, np.int64)
    plen, vis, exp = C.c_int64(), C.c_int64(), C.c_int64()
    ok = C.c_int()
    N.check(N.load().g2048_astar_search(
        b.ctypes.data, int(start_score), goal_exp, int(seed) & ((1 << 64) - 1), int(game), SPAWN[spawn],
        int(max_expansions), int(max_path), pb.ctypes.data, pm.ctypes.data, ps.ctypes.data,
        C.byref(plen), C.byref(vis), C.byref(exp), C.byref(ok)), "g2048_astar_search")
    n = plen.value
    return {"success": bool(ok.value), "path_length": n if ok.value else float("inf"),
            "visited_nodes": vis.value, "expanded_nodes": exp.value,
            "path_boards": pb[:n + 1].copy(), "path_moves": pm[:n].copy(),
            "path_scores": ps[:n + 1].copy()}


def path_transitions(res: dict, compat: bool = True, done=None):
    """The transitions of one search result, in the reference's trace-back order (returned
    node first): arrays (s [n,16], a [n], r [n], s2 [n,16], d [n]).  compat=False needs
    `done` (u8 [n], 1 where the child board has no legal move) in that order."""
    pb, pm, ps = res["path_boards"], res["path_moves"], res["path_scores"]
    n = len(pm)
    order = np.arange(n, 0, -1)  # child index k = n .. 1, its parent k - 1
    child, parent = pb[order], pb[order - 1]
    a = pm[order - 1]
    if compat:  # src/state_space_search.py:119-124
        r = ps[order - 1] - ps[order]
        return child, a, r, child.copy(), np.zeros(n, np.uint8)
    if done is None or len(done) != n:
        raise ValueError("compat=False needs the children's terminal flags")
    return parent, a, ps[order] - ps[order - 1], child, np.asarray(done, np.uint8)


def generate_replay_buffer_using_A_star(batch_size: int, maxlen: int, device="cuda",
                                        seed: int = 0x2048, goal_tile: int = 2048,
                                        compat: bool = True, max_expansions: int = 0):
    """src/state_space_search.py:103-131: `batch_size` searches from fresh boards (two Philox
    spawns each, as the env deals them), every path's transitions appended to a device ring of
    `maxlen` rows (the deque(maxlen) keeps the newest).  Returns (ReplayBuffer, results)."""
    from .env import ReplayBuffer, VecEnv2048

    env = VecEnv2048(int(batch_size), seed=seed, device=device)
    starts = env.board.cpu().numpy()
    results = [A_star(starts[g], goal_tile=goal_tile, seed=seed, game=g,
                      max_expansions=max_expansions) for g in range(int(batch_size))]
    dones = [None] * len(results)
    if not compat:  # terminal flag of every child board, from the device legal-mask kernel
        kids = [res["path_boards"][np.arange(len(res["path_moves"]), 0, -1)] for res in results]
        allk = np.concatenate(kids) if kids else np.zeros((0, 16), np.uint8)
        if len(allk):
            probe = VecEnv2048(len(allk), seed=seed, device=device)
            probe.board.copy_(torch.from_numpy(allk).to(probe.device))
            term = (probe.legal_mask() == 0).cpu().numpy().astype(np.uint8)
            off = np.cumsum([0] + [len(k) for k in kids])
            dones = [term[off[i]:off[i + 1]] for i in range(len(kids))]
    parts = [path_transitions(res, compat, dn) for res, dn in zip(results, dones)]
    s, a, r, s2, d = (np.concatenate([p[i] for p in parts]) for i in range(5))
    keep = slice(max(0, len(a) - int(maxlen)), len(a))  # deque(maxlen): the newest survive
    rb = ReplayBuffer(int(maxlen), device=device)
    if len(a[keep]):
        rb.load(s[keep], a[keep], r[keep], s2[keep], d[keep])
    torch.cuda.synchronize(rb.device)
    return rb, results
