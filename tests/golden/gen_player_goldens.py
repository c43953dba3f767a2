"""Golden fixtures for the batched evaluation player, by running the reference's Player
(src/player.py) in the build container.

    PYTHONPATH=/root/reference/src PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_player_goldens.py

player.npz
  upleft_*   Player.basic_upleft_algorithm (src/player.py:64-83) games: the initial board and
             every (board after the move, move label) it records -- pins the up/left/down/right
             state machine and its stop rule
  greedy_*   Player.play_game(random_policy=False) (src/player.py:41-62) with a deterministic
             conv net: per step the board, the legal mask, Q(normalized board) and the chosen
             action -- pins the normalized encoding (src/board.py:217-221) and
             argmax(avail * Q) without the F5 normalisation.  A game whose argmax lands on an
             illegal move never ends in the reference (the board no longer changes); the
             generator cuts it after the repeat and flags it (greedy_stuck).  Half of the games
             add +50 to the last bias (greedy_offset) so that every Q is positive and the game
             runs to its terminal board
"""
from __future__ import annotations

import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_goldens import det_init, exps_of, make_net  # noqa: E402

import board as ref_board  # noqa: E402
import dqn_lib  # noqa: E402
import player as ref_player  # noqa: E402

LABELS = {"up": 0, "down": 1, "left": 2, "right": 3, "r": 3}


def gen_upleft(n_games=40, seed=11):
    random.seed(seed)
    np.random.seed(seed)
    starts, lens, boards, acts = [], [], [], []
    orig = ref_player.Board2048

    class Recording(orig):
        made = []

        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            Recording.made.append(self.state.copy())

    ref_player.Board2048 = Recording
    try:
        for _ in range(n_games):
            Recording.made.clear()
            stub = types.SimpleNamespace(games_history=[])
            ref_player.Player.basic_upleft_algorithm(stub, k=4)
            hist = stub.games_history[-1]
            starts.append(exps_of(Recording.made[0]))
            lens.append(len(hist))
            for state, label, _simple, _merge in hist:
                boards.append(exps_of(state))
                acts.append(LABELS[label])
    finally:
        ref_player.Board2048 = orig
    return {"upleft_start": np.stack(starts), "upleft_len": np.array(lens, np.int64),
            "upleft_after": np.stack(boards), "upleft_action": np.array(acts, np.uint8)}


class _Stuck(Exception):
    pass


def gen_greedy(n_games=24, seed=5, phases=(0.5, 1.7, 2.9), offsets=(0.0, 50.0), cap=4000):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    rec_b, rec_m, rec_q, rec_a, game_len, stuck, phase_of, off_of = [], [], [], [], [], [], [], []
    peek = ref_board.Board2048.peek_action
    for g in range(n_games):
        ph = phases[g % len(phases)]
        model = make_net("conv")[0].double()  # the reference Sequential, float64
        det_init(model, ph)
        off = offsets[(g // len(phases)) % len(offsets)]
        with torch.no_grad():  # offset > 0: all Q positive, so the argmax stays on legal moves
            model[-1].bias += off
        steps = []

        def model_rec(x, model=model):
            q = model(x)
            steps.append({"q": q.detach().reshape(4).numpy().copy()})
            return q

        calls = {"n": 0, "last": None}

        def guarded(self, action):
            # the chosen move of this step (play_game calls peek_action exactly once per step
            # outside available_moves, with a tensor action)
            if isinstance(action, torch.Tensor):
                a = int(action)
                steps[-1]["board"] = exps_of(self.state)
                steps[-1]["action"] = a
                calls["n"] += 1
                key = (self.state.tobytes(), a)
                if calls["last"] == key:
                    raise _Stuck()  # same board, same action: the reference loops forever
                calls["last"] = key
                if calls["n"] > cap:
                    raise RuntimeError("greedy golden game too long")
            return peek(self, action)

        ref_board.Board2048.peek_action = guarded
        stub = types.SimpleNamespace(model=model_rec, device="cpu", games_history=[],
                                     reward_func=dqn_lib.reward_func_merge_score)
        is_stuck = False
        try:
            with torch.no_grad():
                ref_player.Player.play_game(stub, random_policy=False)
        except _Stuck:
            is_stuck = True
            steps.pop()  # the repeated step
        finally:
            ref_board.Board2048.peek_action = peek
        for st in steps:
            b = st["board"]
            rec_b.append(b)
            vals = np.where(b > 0, 1 << b.astype(np.int64), 0)
            tmp = ref_board.Board2048(populate_empty_cells=False)
            tmp.state = vals.reshape(4, 4)
            avail = tmp.available_moves_as_torch_unit_vector(device="cpu")
            rec_m.append(int(sum(int(avail[k]) << k for k in range(4))))
            rec_q.append(st["q"])
            rec_a.append(st["action"])
        game_len.append(len(steps))
        stuck.append(is_stuck)
        phase_of.append(ph)
        off_of.append(off)
    return {"greedy_board": np.stack(rec_b), "greedy_legal": np.array(rec_m, np.uint8),
            "greedy_q": np.stack(rec_q), "greedy_action": np.array(rec_a, np.uint8),
            "greedy_len": np.array(game_len, np.int64), "greedy_stuck": np.array(stuck, bool),
            "greedy_phase": np.array(phase_of, np.float64),
            "greedy_offset": np.array(off_of, np.float64)}


def main():
    out = {}
    out.update(gen_upleft())
    out.update(gen_greedy())
    np.savez_compressed(os.path.join(HERE, "player.npz"), **out)
    print({k: v.shape for k, v in out.items()})
    print("stuck greedy games:", int(out["greedy_stuck"].sum()), "of", len(out["greedy_stuck"]))


if __name__ == "__main__":
    main()
