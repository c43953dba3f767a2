"""ctypes wrapper over oracle/build/liboracle2048.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker for the HIP env kernels and the CPU baseline, never the product path.
Every function restates the reference (src/board.py, src/dqn_lib.py); see oracle2048.c.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle2048.so")
_lib = None

MODE_ACTIONS, MODE_RANDOM, MODE_EGREEDY_F32, MODE_EGREEDY_F64, MODE_INJECT = 0, 1, 2, 3, 4
P4_10, EGREEDY_FIXED, NO_AUTORESET = 1, 2, 4


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class _Env(C.Structure):
    _fields_ = [("n", C.c_int64), ("board_offset", C.c_uint64), ("seed", C.c_uint64),
                ("flags", C.c_uint32), ("board", C.c_void_p), ("meta", C.c_void_p),
                ("ep", C.c_void_p), ("clock", C.c_void_p), ("qsum", C.c_void_p), ("log", C.c_void_p),
                ("log_slots", C.c_int64)]


# g2048_episode / o2048_episode (40 bytes)
EPISODE_DTYPE = np.dtype([("step", "<u8"), ("q_sum", "<f8"), ("board", "<u4"), ("episode", "<u4"),
                          ("score", "<u4"), ("moves", "<u4"), ("max_exp", "<u4"),
                          ("reserved", "<u4")])
assert EPISODE_DTYPE.itemsize == 40


class _Replay(C.Structure):
    _fields_ = [("capacity", C.c_int64), ("s", C.c_void_p), ("s2", C.c_void_p),
                ("a", C.c_void_p), ("r", C.c_void_p), ("d", C.c_void_p), ("count", C.c_void_p)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp, u8p = C.c_void_p, C.POINTER(C.c_uint8)
        L.o2048_slide_row.restype = C.c_uint32
        L.o2048_slide_row.argtypes = [vp, vp]
        L.o2048_move.restype = C.c_uint32
        L.o2048_move.argtypes = [vp, C.c_int, vp]
        L.o2048_legal_mask.restype = C.c_uint8
        L.o2048_legal_mask.argtypes = [vp]
        L.o2048_philox.restype = None
        L.o2048_philox.argtypes = [vp, vp, vp]
        L.o2048_greedy_f64.restype = C.c_int
        L.o2048_greedy_f64.argtypes = [vp, C.c_uint8, C.c_int]
        L.o2048_greedy_f32.restype = C.c_int
        L.o2048_greedy_f32.argtypes = [vp, C.c_uint8, C.c_int]
        L.o2048_env_reset.restype = None
        L.o2048_env_reset.argtypes = [C.POINTER(_Env), vp, C.c_uint32]
        L.o2048_env_step.restype = C.c_int64
        L.o2048_env_step.argtypes = [C.POINTER(_Env), C.c_int, vp, vp, C.c_double, C.c_double,
                                     C.c_double, vp, vp, vp, vp, vp, vp, C.POINTER(_Replay)]
        L.o2048_replay_sample_f64.restype = None
        L.o2048_replay_sample_f64.argtypes = [C.POINTER(_Replay), vp, C.c_int64, C.c_uint64,
                                              C.c_uint64, vp, vp, vp, vp, vp, vp]
        del u8p
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def slide_row(row):
    r = np.ascontiguousarray(row, dtype=np.uint8)
    out = np.zeros(4, np.uint8)
    sc = lib().o2048_slide_row(_p(r), _p(out))
    return out, int(sc)


def move(board, action):
    b = np.ascontiguousarray(board, dtype=np.uint8).reshape(16)
    out = np.zeros(16, np.uint8)
    sc = lib().o2048_move(_p(b), int(action), _p(out))
    return out, int(sc)


def legal_mask(board) -> int:
    b = np.ascontiguousarray(board, dtype=np.uint8).reshape(16)
    return int(lib().o2048_legal_mask(_p(b)))


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, np.uint32)
    lib().o2048_philox(_p(c), _p(k), _p(out))
    return out


def greedy(q, legal, fixed=False):
    q = np.ascontiguousarray(q)
    if q.dtype == np.float32:
        return int(lib().o2048_greedy_f32(_p(q), int(legal), int(fixed)))
    q = q.astype(np.float64)
    return int(lib().o2048_greedy_f64(_p(q), int(legal), int(fixed)))


class OracleReplay:
    def __init__(self, capacity: int):
        self.capacity = capacity
        self.s = np.zeros((capacity, 16), np.uint8)
        self.s2 = np.zeros((capacity, 16), np.uint8)
        self.a = np.zeros(capacity, np.uint8)
        self.r = np.zeros(capacity, np.int32)
        self.d = np.zeros(capacity, np.uint8)
        self.count = np.zeros(1, np.uint64)
        self._c = _Replay(capacity, _p(self.s), _p(self.s2), _p(self.a), _p(self.r), _p(self.d),
                          _p(self.count))

    def sample_f64(self, idx=None, B=None, seed=0, epoch=0):
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.int64)
            B = len(idx)
        io = np.zeros(B, np.int64)
        s = np.zeros((B, 16)); s2 = np.zeros((B, 16))
        a = np.zeros(B, np.int64); r = np.zeros(B); d = np.zeros(B)
        lib().o2048_replay_sample_f64(C.byref(self._c), _p(idx), B, seed, epoch, _p(io),
                                      _p(s), _p(s2), _p(a), _p(r), _p(d))
        return io, s, a, r, s2, d


class OracleEnv:
    """N boards stepped by the oracle with exactly the semantics of g2048_env_step*."""

    def __init__(self, n: int, seed: int, flags: int = 0, board_offset: int = 0, reset=True):
        self.n = n
        self.board = np.zeros((n, 16), np.uint8)
        self.meta = np.zeros((n, 2), np.uint32)
        self.ep = np.zeros((n, 4), np.uint32)
        self.clock = np.zeros((n + 63) // 64, np.uint64)
        self.epoch = 0
        self._c = _Env(n, board_offset, seed, flags, _p(self.board), _p(self.meta), _p(self.ep),
                       _p(self.clock), None, None, 0)
        if reset:
            self.reset()

    def attach_episode_log(self, slots: int):
        """One EPISODE_DTYPE record per finished episode in per-board slot rings [n][slots]
        (g2048_env_set_episode_log)."""
        self.log = np.zeros((self.n, slots), EPISODE_DTYPE)
        self.qsum = np.zeros(self.n, np.float64)
        self._c.qsum, self._c.log, self._c.log_slots = _p(self.qsum), self.log.ctypes.data, slots
        self._log_read = np.zeros(self.n, np.int64)

    def episodes(self):
        """Records of the episodes finished since the last call, sorted by (step, board)."""
        now = self.ep[:, 0].astype(np.int64)
        S = self.log.shape[1]
        if (now - self._log_read > S).any():
            raise RuntimeError("oracle episode log overflow")
        out = [self.log[b, e % S] for b in range(self.n) for e in range(self._log_read[b], now[b])]
        self._log_read = now
        r = np.array(out, EPISODE_DTYPE)
        return r[np.lexsort((r["board"], r["step"]))] if len(r) else r

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().o2048_env_reset(C.byref(self._c), _p(m), self.epoch)
        self.epoch += 1

    def step(self, mode=MODE_RANDOM, actions=None, q=None, eps=0.0, spawn_idx=None,
             spawn_exp=None, replay: OracleReplay | None = None, eps_schedule=None):
        n = self.n
        reward = np.zeros(n, np.int32)
        done = np.zeros(n, np.uint8)
        legal = np.zeros(n, np.uint8)
        act = np.zeros(n, np.uint8)
        if actions is not None:
            actions = np.ascontiguousarray(actions, dtype=np.uint8)
        if q is not None:
            q = np.ascontiguousarray(q)
        if spawn_idx is not None:
            spawn_idx = np.ascontiguousarray(spawn_idx, dtype=np.int8)
            spawn_exp = np.ascontiguousarray(spawn_exp, dtype=np.uint8)
        dec, mn = eps_schedule if eps_schedule is not None else (0.0, 0.0)
        bad = lib().o2048_env_step(C.byref(self._c), mode, _p(actions), _p(q), float(eps),
                                   float(dec), float(mn),
                                   _p(spawn_idx), _p(spawn_exp), _p(reward), _p(done),
                                   _p(legal), _p(act),
                                   C.byref(replay._c) if replay is not None else None)
        return dict(reward=reward, done=done, legal=legal, action=act, bad=int(bad))
