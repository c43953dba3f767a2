"""Batched evaluation player: the reference's Player (src/player.py:9-84) over N games at once.

Policies (one game per board, every board plays to its end):
  random   Player.play_game(random_policy=True) (:41-62): argmax(avail * U[0,1)^4) == a uniform
           legal move.  Runs inside the fused step kernel (explore branch, legal-only draw).
  upleft   Player.basic_upleft_algorithm (:64-83): up, left; if neither moved, down, right; stop
           when all four failed in one round.  A per-board state machine (UpLeftState).
  greedy   Player.play_game(random_policy=False): argmax(avail * Q(x)) with x = state / max(state)
           (board.normalized(), src/board.py:217-221) -- NOT the F5 formula of training, NOT the
           log encoding the net was trained on (encoding="log" selects the training encoding).
           When every legal Q is negative the argmax lands on an illegal move; the board then no
           longer changes and the reference loops forever.  Here such a game stops at once and is
           flagged `stuck` (rule="legal" restricts the argmax to legal moves instead).

Results follow the reference's bookkeeping: `moves` = steps taken (history length, terminal
step included), `merge_score`, `max_tile`; `max_tile_frequency()` is notebook_utils'
get_max_tile_frequency (experiments/notebook_utils.py:14-16).  `record_games` = k keeps the
per-step history of the first k games in the reference's tuple format for games_played.p.
"""
from __future__ import annotations

import numpy as np
import torch

from . import qnet
from .env import VecEnv2048
from .nets import Conv2048

UP, DOWN, LEFT, RIGHT = 0, 1, 2, 3
LETTERS = ("u", "d", "l", "r")                     # play_game history labels (:58)
UPLEFT_LABELS = ("up", "down", "left", "r")        # basic_upleft_algorithm labels (:69-76)


# ------------------------------------------------------------------ device-agnostic policy pieces
def encode_normalized(board: torch.Tensor, dtype=torch.float64, conv: bool = True) -> torch.Tensor:
    """board.normalized().state_as_4d_tensor() (src/board.py:217-221,235-236) for u8 exponent
    boards [n, 16]: tile values / max tile value."""
    e = board.to(torch.int64)
    v = torch.where(e > 0, torch.ones_like(e) << e, torch.zeros_like(e)).to(torch.float64)
    x = (v / v.amax(dim=1, keepdim=True)).to(dtype)
    return x.view(-1, 1, 4, 4) if conv else x


def encode_log(board: torch.Tensor, dtype=torch.float32, conv: bool = True) -> torch.Tensor:
    """The training encoding (board_as_4d_tensor, src/dqn_lib.py:8-10): the exponents."""
    x = board.to(dtype)
    return x.view(-1, 1, 4, 4) if conv else x


def legal_bits(legal: torch.Tensor) -> torch.Tensor:
    """u8 legal masks [n] -> {0,1} [n, 4] (available_moves_as_torch_unit_vector)."""
    bits = torch.arange(4, device=legal.device, dtype=torch.int32)
    return (legal.to(torch.int32)[:, None] >> bits) & 1


def select_greedy(q: torch.Tensor, legal: torch.Tensor, rule: str = "reference") -> torch.Tensor:
    """reference: torch.argmax(available_moves * Q) (src/player.py:54-57), first index on ties;
    legal: argmax over the legal moves only (0 when none)."""
    avail = legal_bits(legal).to(q.dtype)
    if rule == "reference":
        return torch.argmax(avail * q, dim=1)
    if rule == "legal":
        masked = torch.where(avail > 0, q, torch.full_like(q, -torch.inf))
        a = torch.argmax(masked, dim=1)
        return torch.where(legal > 0, a, torch.zeros_like(a))
    raise ValueError("rule must be 'reference' or 'legal'")


class UpLeftState:
    """basic_upleft_algorithm (src/player.py:64-83) as a per-board state machine.

    phase 0 up, 1 left, 2 down, 3 right; `moved` = some move of the current round changed the
    board (the reference tests simple_score(), the tile sum, which only a spawn -- i.e. a move
    that changed the board -- can raise)."""

    ACTION = (UP, LEFT, DOWN, RIGHT)

    def __init__(self, n: int, device):
        self.phase = torch.zeros(n, dtype=torch.int64, device=device)
        self.moved = torch.zeros(n, dtype=torch.bool, device=device)
        self._act = torch.tensor(self.ACTION, dtype=torch.int64, device=device)

    def actions(self) -> torch.Tensor:
        return self._act[self.phase]

    def update(self, moved_now: torch.Tensor) -> torch.Tensor:
        """Advance after the move of this phase; returns the boards whose game ended."""
        m = self.moved | moved_now
        p = self.phase
        end_round = (p == 1) | (p == 3)
        finished = (p == 3) & ~m
        nxt = torch.where(end_round & m, torch.zeros_like(p), p + 1)
        self.phase = torch.where(finished, p, nxt)
        self.moved = torch.where(end_round, torch.zeros_like(m), m)
        return finished


# ------------------------------------------------------------------ results
class GameResults:
    def __init__(self, policy, max_tile, merge_score, moves, stuck, histories):
        self.policy = policy
        self.max_tile = max_tile          # int64 [n] tile value
        self.merge_score = merge_score    # int64 [n]
        self.moves = moves                # int64 [n] steps taken (history length)
        self.stuck = stuck                # bool  [n] greedy game stopped on an illegal argmax
        self.histories = histories        # list of per-game histories (first record_games)

    def __len__(self):
        return len(self.max_tile)

    def max_tile_frequency(self) -> np.ndarray:
        return np.array(np.unique(self.max_tile, return_counts=True), dtype=int)

    def summary(self) -> dict:
        return {"policy": self.policy, "games": len(self), "stuck": int(self.stuck.sum()),
                "merge_score_mean": float(self.merge_score.mean()),
                "moves_mean": float(self.moves.mean()), "max_tile_max": int(self.max_tile.max()),
                "max_tile_hist": {int(k): int(v) for k, v in zip(*self.max_tile_frequency())}}


# ------------------------------------------------------------------ the player
class BatchedPlayer:
    """n_games games on one GPU; see the module docstring for the policies."""

    def __init__(self, n_games: int, device="cuda:0", seed: int = 0, model=None,
                 encoding: str = "normalized", rule: str = "reference", p4: float = 0.5,
                 record_games: int = 0, max_moves: int = 1 << 20, check_every: int = 32):
        self.n = int(n_games)
        self.device = torch.device(device)
        self.seed = int(seed)
        self.model = model
        if encoding not in ("normalized", "log"):
            raise ValueError("encoding must be 'normalized' (src/player.py:50) or 'log'")
        self.encoding, self.rule, self.p4 = encoding, rule, p4
        self.record = int(min(record_games, self.n))
        self.max_moves = int(max_moves)
        self.check_every = int(check_every)

    def _env(self, egreedy="compat"):
        return VecEnv2048(self.n, seed=self.seed, device=self.device, p4=self.p4,
                          egreedy=egreedy, autoreset=False)

    @torch.no_grad()
    def _q(self, env):
        m = self.model
        conv = isinstance(m, Conv2048) or (isinstance(m, torch.nn.Sequential)
                                           and isinstance(m[0], torch.nn.Conv2d))
        dtype = next(m.parameters()).dtype
        if self.encoding == "log" and qnet.kind_of(m) is not None:
            return qnet.forward(m, env.board)  # fused fp32 kernels eat exponents directly
        x = (encode_normalized if self.encoding == "normalized" else encode_log)(
            env.board, dtype, conv)
        return m(x).reshape(self.n, 4)

    def play(self, policy: str = "random") -> GameResults:
        if policy == "greedy" and self.model is None:
            raise ValueError("the greedy policy needs a model")
        if policy not in ("random", "upleft", "greedy"):
            raise ValueError("policy must be 'random', 'upleft' or 'greedy'")
        env = self._env(egreedy="fixed" if policy == "random" else "compat")
        dev = self.device
        n = self.n
        fin = torch.zeros(n, dtype=torch.bool, device=dev)
        stuck = torch.zeros(n, dtype=torch.bool, device=dev)
        f_score = torch.zeros(n, dtype=torch.int64, device=dev)
        f_moves = torch.zeros(n, dtype=torch.int64, device=dev)
        f_max = torch.zeros(n, dtype=torch.int64, device=dev)
        ul = UpLeftState(n, dev) if policy == "upleft" else None
        q0 = torch.zeros((n, 4), dtype=torch.float32, device=dev) if policy == "random" else None
        rec = []  # per step: (board before, action, reward, score before, board after)
        k = self.record
        t = 0
        while True:
            before = env.board[:k].clone() if k else None
            score_before = env.score[:k].clone() if k else None
            if policy == "random":
                act, reward, done = env.step_egreedy(q0, 1.0)
                ended = done.bool()
                newly_stuck = None
            elif policy == "upleft":
                act = ul.actions()
                reward, _, legal = env.step(act)
                moved = ((legal.to(torch.int64) >> act) & 1).bool()
                ended = ul.update(moved)
                newly_stuck = None
            else:
                legal = env.legal_mask()
                act = select_greedy(self._q(env), legal, self.rule)
                reward, done, _ = env.step(act)
                ended = done.bool()
                # an illegal argmax on a live board repeats forever in the reference
                illegal = ((legal.to(torch.int64) >> act) & 1) == 0
                newly_stuck = illegal & ~ended & ~fin
                ended = ended | newly_stuck
            new = ended & ~fin
            sm = env.score_moves().to(torch.int64)
            f_score = torch.where(new, sm[:, 0], f_score)
            f_moves = torch.where(new, sm[:, 1], f_moves)
            f_max = torch.where(new, env.board.amax(dim=1).to(torch.int64), f_max)
            if newly_stuck is not None:
                stuck |= newly_stuck
            fin |= new
            if k:
                rec.append((before, act[:k].to(torch.uint8), reward[:k].clone(), score_before,
                            env.board[:k].clone()))
            t += 1
            if t % self.check_every == 0 or t >= self.max_moves:
                if bool(fin.all()) or t >= self.max_moves:
                    break
        env.check_errors()
        max_tile = torch.where(f_max > 0, torch.ones_like(f_max) << f_max, f_max)
        hist = self._histories(policy, rec, f_moves[:k].cpu().numpy()) if k else []
        return GameResults(policy, max_tile.cpu().numpy(), f_score.cpu().numpy(),
                           f_moves.cpu().numpy(), stuck.cpu().numpy(), hist)

    @staticmethod
    def _histories(policy, rec, moves):
        """Per-game history tuples in the reference's format:
        play_game:   (state before, 'u'|'d'|'l'|'r', reward, merge_score before)   (:58)
        upleft:      (state after, 'up'|'left'|'down'|'r', simple_score, merge_score) (:69-76)"""
        from .experiment import real_state
        if not rec:
            return []
        b0 = torch.stack([r[0] for r in rec]).cpu().numpy()
        ac = torch.stack([r[1] for r in rec]).cpu().numpy()
        rw = torch.stack([r[2] for r in rec]).cpu().numpy()
        sb = torch.stack([r[3] for r in rec]).cpu().numpy()
        b1 = torch.stack([r[4] for r in rec]).cpu().numpy()
        games = []
        for j in range(b0.shape[1]):
            h = []
            for t in range(int(moves[j])):
                if policy == "upleft":
                    st = real_state(b1[t, j])
                    h.append((st, UPLEFT_LABELS[int(ac[t, j])], int(st.sum()),
                              int(sb[t, j]) + int(rw[t, j])))
                else:
                    a = int(ac[t, j])
                    if policy == "random" and t == int(moves[j]) - 1:
                        a = UP  # terminal step: argmax of an all-zero vector (:54-57)
                    h.append((real_state(b0[t, j]), LETTERS[a], int(rw[t, j]), int(sb[t, j])))
            games.append(h)
        return games


def play_n_games(n: int, policy: str = "random", experiment=None, **kw) -> GameResults:
    """Player.play_n_games (src/player.py:31-39): play n games and, with an experiment, append
    the recorded histories to binary/games_played.p."""
    res = BatchedPlayer(n, **kw).play(policy)
    if experiment is not None:
        experiment.save_games_played(res.histories)
    return res
