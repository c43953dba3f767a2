"""VecEnv2048 / ReplayBuffer: batched, HBM-resident replacements for Board2048 and the replay deque.

Reference objects replaced (ribal-aladeeb/reinforcement-learning-2048):
  Board2048                     src/board.py:8-237   -> one row of VecEnv2048 (N boards at once)
  deque((s, a, r, s', done))    src/dqn_lib.py:172   -> ReplayBuffer (SoA ring in HBM)
All state lives in torch-allocated device tensors that the C ABI wraps by pointer
(g2048_env_wrap / g2048_replay_wrap), so the boards can be fed straight into the Q-network.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as N

ACTIONS = ("up", "down", "left", "right")  # src/board.py:129, action ints at :191

# g2048_episode (include/g2048.h), 40 bytes per finished episode
EPISODE_FIELDS = ("step", "q_sum", "board", "episode", "score", "moves", "max_exp")


def decode_episodes(raw: torch.Tensor) -> dict:
    """int64 [k, 5] records -> dict of int64 / float64 host tensors, sorted by (step, board)
    (the completion order; ties within one step broken by board id)."""
    raw = raw.cpu()
    lo = raw[:, 2:5] & 0xFFFFFFFF
    hi = (raw[:, 2:5] >> 32) & 0xFFFFFFFF
    out = {"step": raw[:, 0].clone(), "q_sum": raw[:, 1].view(torch.float64).clone(),
           "board": lo[:, 0], "episode": hi[:, 0], "score": lo[:, 1], "moves": hi[:, 1],
           "max_exp": lo[:, 2]}
    order = torch.from_numpy(np.lexsort((out["board"].numpy(), out["step"].numpy())))
    return {k: v[order] for k, v in out.items()}


class EpisodeLog:
    """Per-board rings of finished-episode records, written by the step kernels themselves
    (g2048_env_set_episode_log: board i's episode e lands in slot i*S + e%S) -- the per-episode
    bookkeeping of training_loop (src/dqn_lib.py:184-213) and Experiment.add_episode
    (src/experiments.py:112-122) with no host round trip and no atomics per step.  `read()`
    gathers the records of episodes finished since the last read, using the env's own per-board
    episode counters (ep[:, 0])."""

    def __init__(self, env: "VecEnv2048", slots_per_board: int = 8):
        self.env = env
        self.slots = int(slots_per_board)
        kw = dict(device=env.device)
        self.raw = torch.zeros((env.n, self.slots, 5), dtype=torch.int64, **kw)
        self.qsum = torch.zeros(env.n, dtype=torch.float64, **kw)
        self.read_ep = env.ep[:, 0].to(torch.int64)   # episodes already accounted for
        self.ep0 = self.read_ep.clone()               # at attach time
        N.check(N.load().g2048_env_set_episode_log(env.handle, N.ptr(self.raw), self.slots,
                                                   N.ptr(self.qsum)), "g2048_env_set_episode_log")

    def detach(self) -> None:
        N.check(N.load().g2048_env_set_episode_log(self.env.handle, None, 0, None),
                "g2048_env_set_episode_log")

    def total(self) -> int:
        """Episodes finished since the log was attached (host sync)."""
        return int((self.env.ep[:, 0].to(torch.int64) - self.ep0).sum())

    def read(self, strict: bool = True) -> dict:
        """Records of the episodes finished since the last read, sorted by (step, board) (host
        sync).  strict: raise if a board finished more than `slots` episodes since the last read
        (older records were overwritten; read more often or attach more slots)."""
        now = self.env.ep[:, 0].to(torch.int64)
        cnt = now - self.read_ep
        over = int(cnt.max()) - self.slots if cnt.numel() else 0
        if over > 0:
            if strict:
                raise RuntimeError(f"episode log overflow: a board finished {over} episodes more "
                                   f"than its {self.slots} slots since the last read")
            cnt = cnt.clamp(max=self.slots)
        first = now - cnt
        self.read_ep = now
        total = int(cnt.sum())
        if total == 0:
            return decode_episodes(self.raw.new_zeros((0, 5)))
        boards = torch.repeat_interleave(torch.arange(self.env.n, device=cnt.device), cnt)
        starts = torch.cumsum(cnt, 0) - cnt
        k = torch.arange(total, device=cnt.device) - torch.repeat_interleave(starts, cnt)
        ep = first[boards] + k
        return decode_episodes(self.raw[boards, ep % self.slots])


class VecEnv2048:
    """N independent 2048 boards on one GPU, stepped by the HIP kernels in csrc/g2048.hip.

    board  uint8 [N, 16]  log2 exponents (== Board2048.log_scale().state, src/board.py:224-231)
    meta   int32 [2, N]   row 0: score (= merge_score()); row 1: the step clock (low 32 bits) at
                          which the running episode began -- moves (= len(_action_history)) is
                          clock - start, derived (ABI v5: a one-launch step moves 4 B of meta);
                          score_moves() gives the [N, 2] {score, moves} pairs
    ep     int32 [N, 4]   {episodes finished, last score, last moves, last max exponent}
    clock  int64 [ceil(N/64)]  steps taken by each 64-board group (all equal; the Philox counter)
    """

    def __init__(self, n_boards: int, seed: int = 0x2048, device="cuda", board_offset: int = 0,
                 p4: float = 0.5, egreedy: str = "compat", autoreset: bool = True,
                 reset: bool = True):
        if p4 not in (0.5, 0.1):
            raise ValueError("p4 must be 0.5 (reference, src/board.py:12) or 0.1")
        if egreedy not in ("compat", "fixed"):
            raise ValueError("egreedy must be 'compat' (src/dqn_lib.py:25-29) or 'fixed'")
        if not 0 < int(n_boards) <= N.MAX_BOARDS:
            raise ValueError(f"n_boards must be in [1, {N.MAX_BOARDS}] (G2048_MAX_BOARDS)")
        self.device = N.require_gpu(device)
        self.n = int(n_boards)
        self.seed = int(seed)
        self.board_offset = int(board_offset)
        self.flags = ((N.P4_10 if p4 == 0.1 else 0) | (N.EGREEDY_FIXED if egreedy == "fixed" else 0)
                      | (0 if autoreset else N.NO_AUTORESET))
        lib = N.load()
        kw = dict(device=self.device)
        self.board = torch.zeros((self.n, 16), dtype=torch.uint8, **kw)
        self.meta = torch.zeros((2, self.n), dtype=torch.int32, **kw)
        self.ep = torch.zeros((self.n, 4), dtype=torch.int32, **kw)
        self.clock = torch.zeros(((self.n + 63) // 64,), dtype=torch.int64, **kw)
        self._h = C.c_void_p()
        self._destroy = lib.g2048_env_destroy
        with torch.cuda.device(self.device):
            N.check(lib.g2048_env_wrap(C.byref(self._h), self.n, self.seed, self.board_offset,
                                       self.device.index, self.flags, N.ptr(self.board),
                                       N.ptr(self.meta), N.ptr(self.ep), N.ptr(self.clock),
                                       int(reset),
                                       N.stream_of(self.device)), "g2048_env_wrap")

    def __del__(self):
        # the destroy entry point is bound at construction: at interpreter exit the module
        # globals this would otherwise go through may already be torn down
        h = getattr(self, "_h", None)
        destroy = getattr(self, "_destroy", None)
        if h and destroy is not None:
            destroy(h)
            self._h = None

    def __len__(self):
        return self.n

    @property
    def handle(self):
        return self._h

    def _stream(self):
        return N.stream_of(self.device)

    # ------------------------------------------------------------------ state
    @property
    def epoch(self) -> int:
        """Explicit-reset epoch (host state of the env; saved by checkpoints)."""
        v = C.c_uint32()
        N.check(N.load().g2048_env_get_epoch(self._h, C.byref(v)), "g2048_env_get_epoch")
        return int(v.value)

    @epoch.setter
    def epoch(self, value: int) -> None:
        N.check(N.load().g2048_env_set_epoch(self._h, int(value)), "g2048_env_set_epoch")

    def attach_episode_log(self, slots_per_board: int = 8) -> EpisodeLog:
        self.episode_log = EpisodeLog(self, slots_per_board)
        return self.episode_log

    def legal_mask(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """available_moves (src/board.py:128-145) of every current board as a u8 bit mask."""
        out = self._out(out, torch.uint8)
        N.check(N.load().g2048_env_legal_mask(self._h, N.ptr(out), self._stream()),
                "g2048_env_legal_mask")
        return out

    def available_moves_as_unit_vectors(self, dtype=torch.float32) -> torch.Tensor:
        """available_moves_as_torch_unit_vector (src/board.py:128-135) for all boards: [N, 4]."""
        m = self.legal_mask().to(torch.int32)
        bits = torch.arange(4, device=self.device, dtype=torch.int32)
        return ((m[:, None] >> bits) & 1).to(dtype)

    # ------------------------------------------------------------------ stepping
    def reset(self, mask: torch.Tensor | None = None) -> None:
        """Re-deal boards (2 spawns each, src/board.py:18-20) where mask != 0 (all if None)."""
        if mask is not None:
            mask = self._u8(mask, "mask")
        N.check(N.load().g2048_env_reset(self._h, N.ptr(mask), self._stream()), "g2048_env_reset")

    def step(self, actions: torch.Tensor | None = None, replay: "ReplayBuffer | None" = None,
             reward=None, done=None, legal=None):
        """One move on every board (peek_action + reward + done, src/board.py:185-202,
        src/dqn_lib.py:87-88,17-18).  actions None = uniform random (np.random.randint(4)).
        Returns (reward int32 [N], done uint8 [N], legal uint8 [N]) for the boards BEFORE the move."""
        if actions is not None:
            actions = self._u8(actions, "actions")
        reward = self._out(reward, torch.int32)
        done = self._out(done, torch.uint8)
        legal = self._out(legal, torch.uint8)
        N.check(N.load().g2048_env_step(self._h, N.ptr(actions), N.ptr(reward), N.ptr(done),
                                        N.ptr(legal), replay.handle if replay is not None else None,
                                        self._stream()), "g2048_env_step")
        return reward, done, legal

    def step_egreedy(self, q: torch.Tensor, epsilon, replay: "ReplayBuffer | None" = None,
                     reward=None, done=None, action=None, eps_schedule=None):
        """Fused epsilon_greedy_policy + peek_action + replay append (src/dqn_lib.py:16-30,91-107).
        q: Q-values [N, 4] (float32 or float64) of the current boards; epsilon: float or a
        float64 device scalar tensor (graph-safe); or eps_schedule = (decay_episodes, min_eps)
        for the reference's per-episode schedule per board (src/dqn_lib.py:184-188, epsilon is
        then ignored).  Returns (action, reward, done)."""
        if q.shape != (self.n, 4) or q.device != self.device or not q.is_contiguous():
            raise ValueError(f"q must be a contiguous [{self.n}, 4] tensor on {self.device}")
        if q.dtype not in (torch.float32, torch.float64):
            raise TypeError("q must be float32 or float64")
        dt = N.F32 if q.dtype == torch.float32 else N.F64
        if eps_schedule is not None:
            eps_ptr, eps_val = None, 0.0
        elif isinstance(epsilon, torch.Tensor):
            if epsilon.dtype != torch.float64 or epsilon.device != self.device or epsilon.numel() != 1:
                raise ValueError("epsilon tensor must be one float64 on the env device")
            eps_ptr, eps_val = N.ptr(epsilon), 0.0
        else:
            eps_ptr, eps_val = None, float(epsilon)
        reward = self._out(reward, torch.int32)
        done = self._out(done, torch.uint8)
        action = self._out(action, torch.uint8)
        if eps_schedule is not None:
            N.check(N.load().g2048_env_step_egreedy_schedule(
                self._h, N.ptr(q), dt, float(eps_schedule[0]), float(eps_schedule[1]),
                N.ptr(reward), N.ptr(done), N.ptr(action),
                replay.handle if replay is not None else None, self._stream()),
                "g2048_env_step_egreedy_schedule")
            return action, reward, done
        N.check(N.load().g2048_env_step_egreedy(self._h, N.ptr(q), dt, eps_ptr, eps_val,
                                                N.ptr(reward), N.ptr(done), N.ptr(action),
                                                replay.handle if replay is not None else None,
                                                self._stream()), "g2048_env_step_egreedy")
        return action, reward, done

    def eps_args(self, epsilon, eps_schedule=None):
        """(eps_dev, eps, eps_decay_episodes, eps_min) of the ABI's eps forms: a schedule
        (decay_episodes, min_eps), a float64 device scalar tensor, or a float."""
        if eps_schedule is not None:
            if not float(eps_schedule[0]) > 0.0:
                raise ValueError("eps_schedule decay_episodes must be > 0")
            return None, 0.0, float(eps_schedule[0]), float(eps_schedule[1])
        if isinstance(epsilon, torch.Tensor):
            if epsilon.dtype != torch.float64 or epsilon.device != self.device or epsilon.numel() != 1:
                raise ValueError("epsilon tensor must be one float64 on the env device")
            return N.ptr(epsilon), 0.0, 0.0, 0.0
        return None, float(epsilon), 0.0, 0.0

    def step_egreedy_dense64(self, params, epsilon=0.0, replay: "ReplayBuffer | None" = None,
                             reward=None, done=None, action=None, eps_schedule=None, q_out=None,
                             f64: bool = False):
        """play_one_step for every board with the dense 16-64-4 Q-net computed INSIDE the step
        kernel (g2048_env_step_egreedy_dense64, or _f64 with f64=True): params = the parameter
        struct of an fp32 (qnet.net_params) or float64 dense64 net.  Same epsilon forms as
        step_egreedy.  Returns (action, reward, done)."""
        eps_ptr, eps_val, dec, mn = self.eps_args(epsilon, eps_schedule)
        qdt = torch.float64 if f64 else torch.float32
        if q_out is not None and (q_out.shape != (self.n, 4) or q_out.dtype != qdt
                                  or not q_out.is_contiguous()):
            raise ValueError(f"q_out must be a contiguous {qdt} [{self.n}, 4] tensor")
        reward = self._out(reward, torch.int32)
        done = self._out(done, torch.uint8)
        action = self._out(action, torch.uint8)
        name = "g2048_env_step_egreedy_dense64_f64" if f64 else "g2048_env_step_egreedy_dense64"
        N.check(getattr(N.load(), name)(
            self._h, C.byref(params), eps_ptr, eps_val, dec, mn, N.ptr(reward), N.ptr(done),
            N.ptr(action), replay.handle if replay is not None else None, N.ptr(q_out),
            self._stream()), name)
        return action, reward, done

    def step_inject(self, actions, spawn_idx, spawn_exp):
        """Test entry: the given actions with the given spawn cells (-1 = none) / exponents."""
        actions = self._u8(actions, "actions")
        spawn_idx = self._typed(spawn_idx, torch.int8, "spawn_idx")
        spawn_exp = self._u8(spawn_exp, "spawn_exp")
        reward, done, legal = (self._out(None, torch.int32), self._out(None, torch.uint8),
                               self._out(None, torch.uint8))
        N.check(N.load().g2048_env_step_inject(self._h, N.ptr(actions), N.ptr(spawn_idx),
                                               N.ptr(spawn_exp), N.ptr(reward), N.ptr(done),
                                               N.ptr(legal), self._stream()),
                "g2048_env_step_inject")
        return reward, done, legal

    def rollout(self, k_steps: int, replay: "ReplayBuffer | None" = None,
                reward_sum: torch.Tensor | None = None):
        """k_steps random-policy steps in ONE launch (boards stay in registers)."""
        if reward_sum is not None:
            reward_sum = self._typed(reward_sum, torch.int64, "reward_sum")
        N.check(N.load().g2048_env_rollout(self._h, int(k_steps), replay.handle if replay is not None else None,
                                           N.ptr(reward_sum), self._stream()), "g2048_env_rollout")
        return reward_sum

    def error_count(self) -> int:
        c = C.c_int64()
        N.check(N.load().g2048_env_error_count(self._h, C.byref(c), self._stream()),
                "g2048_env_error_count")
        return int(c.value)

    def check_errors(self) -> None:
        """Raise like the reference does (IndexError for an action outside 0..3, src/board.py:192)."""
        n = self.error_count()
        if n:
            raise IndexError(f"{n} invalid action(s) / injected spawn(s) since the last check")

    # ------------------------------------------------------------------ views
    @property
    def score(self):          # Board2048.merge_score(), src/board.py:207
        return self.meta[0]

    @property
    def moves(self):          # len(Board2048._action_history): clock - episode start (mod 2^32)
        return self.score_moves()[:, 1]

    def score_moves(self) -> torch.Tensor:
        """int32 [N, 2] {score, moves} of every board (g2048_env_score_moves; the u32 values in
        int32, as the v4 meta layout held them)."""
        out = torch.empty((self.n, 2), dtype=torch.int32, device=self.device)
        N.check(N.load().g2048_env_score_moves(self._h, N.ptr(out), self._stream()),
                "g2048_env_score_moves")
        return out

    @property
    def steps(self):
        return self.clock.repeat_interleave(64)[:self.n]

    def max_tile(self):
        return torch.where(self.board.amax(1) > 0, 1 << self.board.amax(1).to(torch.int64), 0)

    def encode(self, dtype=torch.float32, conv: bool = True):
        """board_as_4d_tensor / board_as_flattened_tensor (src/dqn_lib.py:8-13) for all boards."""
        x = self.board.to(dtype)
        return x.view(self.n, 1, 4, 4) if conv else x

    # ------------------------------------------------------------------ helpers
    def _typed(self, t, dtype, name):
        t = torch.as_tensor(t, device=self.device)
        if t.dtype != dtype:
            t = t.to(dtype)
        if t.numel() != self.n:
            raise ValueError(f"{name} must have {self.n} elements")
        return t.contiguous()

    def _u8(self, t, name):
        return self._typed(t, torch.uint8, name)

    def _out(self, t, dtype):
        if t is None:
            return torch.empty(self.n, dtype=dtype, device=self.device)
        if t.dtype != dtype or t.numel() != self.n or not t.is_contiguous() or t.device != self.device:
            raise ValueError(f"output must be a contiguous {dtype} [{self.n}] tensor on {self.device}")
        return t


class ReplayBuffer:
    """HBM ring of transitions (s u8[16], a u8, r i32, s' u8[16], done u8): the reference's
    deque(maxlen=replay_buffer_length) of (Board2048, action, reward, Board2048, done) tuples
    (src/dqn_lib.py:106,172), 38 bytes per transition instead of two Python objects."""

    def __init__(self, capacity: int, device="cuda", sections=None):
        """sections: optional caller-owned (s, s2, a, r, d, count) device tensors to wrap
        (u8 [capacity, 16] x 2, u8 / i32 / u8 [capacity], i64 [1]); by default one allocation
        holds them all."""
        self.device = N.require_gpu(device)
        self.capacity = int(capacity)
        c = self.capacity
        if sections is None:
            # one allocation, 256-byte aligned sections s | s2 | r | a | d | count, each
            # G2048_REPLAY_SECTION_PAD bytes further (as g2048_replay_create lays them out): the
            # rollout's ring stores then always take the one-descriptor buffer path (sections
            # within 4 GiB), whereas separately allocated tensors land wherever the allocator
            # puts them; the pad keeps power-of-two capacities from putting the five store
            # streams on the same HBM channels (include/g2048.h)
            up = lambda x: (x + 255) // 256 * 256 + N.REPLAY_SECTION_PAD  # noqa: E731
            o_s2 = up(16 * c)
            o_r = o_s2 + up(16 * c)
            o_a = o_r + up(4 * c)
            o_d = o_a + up(c)
            o_c = o_d + up(c)
            self._mem = torch.zeros(o_c + 256, dtype=torch.uint8, device=self.device)
            m = self._mem
            sections = (m[0:16 * c].view(c, 16), m[o_s2:o_s2 + 16 * c].view(c, 16),
                        m[o_a:o_a + c], m[o_r:o_r + 4 * c].view(torch.int32), m[o_d:o_d + c],
                        m[o_c:o_c + 8].view(torch.int64))
        want = [((c, 16), torch.uint8), ((c, 16), torch.uint8), ((c,), torch.uint8),
                ((c,), torch.int32), ((c,), torch.uint8), ((1,), torch.int64)]
        for t, (shape, dt) in zip(sections, want):
            if (tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous()
                    or t.device != self.device):
                raise ValueError(f"replay section must be a contiguous {dt} {shape} tensor on "
                                 f"{self.device}")
        self.s, self.s2, self.a, self.r, self.d, self.count = sections
        self._h = C.c_void_p()
        self._destroy = N.load().g2048_replay_destroy
        with torch.cuda.device(self.device):
            N.check(N.load().g2048_replay_wrap(C.byref(self._h), self.capacity, self.device.index,
                                               N.ptr(self.s), N.ptr(self.s2), N.ptr(self.a),
                                               N.ptr(self.r), N.ptr(self.d), N.ptr(self.count)),
                    "g2048_replay_wrap")

    def __del__(self):
        # the destroy entry point is bound at construction: at interpreter exit the module
        # globals this would otherwise go through may already be torn down
        h = getattr(self, "_h", None)
        destroy = getattr(self, "_destroy", None)
        if h and destroy is not None:
            destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def __len__(self):  # host sync
        return int(self.count.item())

    def load(self, s, a, r, s2, d) -> None:
        """Fill the first rows from host/device arrays (tests, warm starts)."""
        n = len(a)
        self.s[:n].copy_(torch.as_tensor(s, dtype=torch.uint8).reshape(n, 16))
        self.s2[:n].copy_(torch.as_tensor(s2, dtype=torch.uint8).reshape(n, 16))
        self.a[:n].copy_(torch.as_tensor(a).to(torch.uint8))
        self.r[:n].copy_(torch.as_tensor(r).to(torch.int32))
        self.d[:n].copy_(torch.as_tensor(d).to(torch.uint8))
        self.count.fill_(n)

    def sample_encode(self, batch_size: int, dtype=torch.float32, idx: torch.Tensor | None = None,
                      seed: int = 0, epoch: int = 0, out=None, want_s2: bool = True,
                      want_s: bool = True):
        """sample_experiences (src/dqn_lib.py:67-84) with the encode of extract_samples_*
        (:33-64) fused: returns (states [B,16], actions i64 [B], rewards [B], next_states [B,16],
        dones [B], idx i64 [B]).  idx None = uniform with replacement over the filled rows."""
        if dtype not in (torch.float32, torch.float64):
            raise TypeError("dtype must be float32 or float64")
        B = int(batch_size)
        if idx is not None:
            idx = torch.as_tensor(idx, device=self.device).to(torch.int64).contiguous()
            if idx.numel() != B:
                raise ValueError("idx must have batch_size elements")
        kw = dict(device=self.device)
        if out is None:
            out = (torch.empty((B, 16), dtype=dtype, **kw), torch.empty(B, dtype=torch.int64, **kw),
                   torch.empty(B, dtype=dtype, **kw), torch.empty((B, 16), dtype=dtype, **kw),
                   torch.empty(B, dtype=dtype, **kw), torch.empty(B, dtype=torch.int64, **kw))
        s, a, r, s2, d, io = out
        if not want_s2:
            s2 = None
        if not want_s:
            s = None
        N.check(N.load().g2048_replay_sample_encode(
            self._h, N.ptr(idx), B, int(seed), int(epoch), N.F32 if dtype == torch.float32 else N.F64,
            N.ptr(s), N.ptr(s2), N.ptr(a), N.ptr(r), N.ptr(d), N.ptr(io),
            N.stream_of(self.device)), "g2048_replay_sample_encode")
        return s, a, r, s2, d, io
