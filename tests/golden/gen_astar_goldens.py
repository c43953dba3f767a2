"""Golden fixtures for the A* replay pre-fill (src/state_space_search.py:46-131), by running the
reference's A_star in the build container.

    PYTHONPATH=/root/reference/src PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_astar_goldens.py

The reference spawns from numpy / `random`, which no other RNG can reproduce, so the generator
pins the SEARCH with a deterministic spawn rule patched into Board2048._populate_empty_cell:
a 2 in the first empty cell (row-major).  The build's search takes the same rule as its
`spawn_mode = first-empty`.  The goal test `goal_tile in board` (2048 for these starts) is
patched to look for a smaller tile (GOALS) so that the reference finishes in seconds; the
order in which nodes are popped, skipped, closed and expanded is the reference's own.

astar.npz, per case c (start board, goal exponent):
  start[c]        u8[16] start exponents
  goal[c]         goal exponent
  visited[c], expanded[c], success[c]
  path_off[c]     offset of the case's path in path_boards / path_moves
  path_len[c]     number of moves on the returned node's path
  path_boards     u8[sum(path_len + 1), 16] boards root .. returned node
  path_moves      u8[sum(path_len)] moves (0 up, 1 down, 2 left, 3 right)
  path_scores     i64[sum(path_len + 1)] merge score of every node on the path
  rb_*            generate_replay_buffer_using_A_star's transitions for the case (s, a, r, s2,
                  d), as the reference appends them (s' = s, r = parent - child score, d = 0)
"""
from __future__ import annotations

import os

import numpy as np

import board as ref_board  # noqa: E402
import dqn_lib  # noqa: E402
import state_space_search as sss  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
MOVES = {"up": 0, "down": 1, "left": 2, "right": 3}


def first_empty_two(self):
    idx = np.argwhere(self.state.flatten() == 0)
    if len(idx):
        self.state.flat[int(idx[0][0])] = 2
    return self


def exps(state):
    s = np.asarray(state, dtype=np.int64).flatten()
    out = np.zeros(16, np.uint8)
    nz = s > 0
    out[nz] = np.log2(s[nz]).astype(np.uint8)
    return out


def board_from_exps(e):
    b = ref_board.Board2048(populate_empty_cells=False)
    b.state = np.array([0 if x == 0 else 1 << int(x) for x in e], dtype=int).reshape(4, 4)
    return b


def main():
    ref_board.Board2048._populate_empty_cell = first_empty_two
    starts = [
        [1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0],
        [0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1],
        [1, 1, 2, 0, 0, 0, 0, 3, 0, 0, 0, 0, 2, 0, 0, 0],
        [3, 2, 1, 1, 0, 0, 0, 0, 0, 4, 0, 0, 0, 0, 0, 2],
        [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2],
        [5, 4, 3, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1],
    ]
    goals = [5, 6, 7]
    rec = {k: [] for k in ("start", "goal", "visited", "expanded", "success", "path_off",
                           "path_len", "path_boards", "path_moves", "path_scores", "rb_off",
                           "rb_len", "rb_s", "rb_a", "rb_r", "rb_s2", "rb_d")}
    orig_contains = ref_board.Board2048.__contains__
    for st in starts:
        for goal in goals:
            ref_board.Board2048.__contains__ = (
                lambda self, el, _g=goal: orig_contains(self, (1 << _g) if el == 2048 else el))
            res = sss.A_star(board_from_exps(st))
            node = res["current_node"]
            chain = []
            while node is not None:
                chain.append(node)
                node = node.parent
            chain.reverse()
            rec["start"].append(np.array(st, np.uint8))
            rec["goal"].append(goal)
            rec["visited"].append(res["visited_nodes"])
            rec["expanded"].append(res["expanded_nodes"])
            rec["success"].append(int(np.isfinite(res["path_length"])))
            rec["path_off"].append(sum(len(m) for m in rec["path_moves"]))
            rec["path_len"].append(len(chain) - 1)
            rec["path_boards"].append(np.stack([exps(n.board.state) for n in chain]))
            rec["path_moves"].append(np.array([MOVES[n.move] for n in chain[1:]], np.uint8))
            rec["path_scores"].append(np.array([n.board.merge_score() for n in chain], np.int64))
            # generate_replay_buffer_using_A_star's trace-back (src/state_space_search.py:109-127)
            s, a, r, s2, d = [], [], [], [], []
            cur = res["current_node"]
            while cur.parent is not None:
                par = cur.parent
                done = int(cur.is_root())
                act = MOVES[cur.move]
                s.append(exps(cur.board.state))
                a.append(act)
                r.append(dqn_lib.reward_func_merge_score(cur.board, par.board, act, done))
                s2.append(exps(cur.board.state))
                d.append(done)
                cur = par
            rec["rb_off"].append(sum(len(x) for x in rec["rb_a"]))
            rec["rb_len"].append(len(a))
            rec["rb_s"].append(np.array(s, np.uint8).reshape(-1, 16))
            rec["rb_a"].append(np.array(a, np.uint8))
            rec["rb_r"].append(np.array(r, np.int64))
            rec["rb_s2"].append(np.array(s2, np.uint8).reshape(-1, 16))
            rec["rb_d"].append(np.array(d, np.uint8))
            print(f"start {st} goal 2^{goal}: visited {res['visited_nodes']} expanded "
                  f"{res['expanded_nodes']} path {len(chain) - 1}")
    out = {
        "start": np.stack(rec["start"]), "goal": np.array(rec["goal"], np.int32),
        "visited": np.array(rec["visited"], np.int64), "expanded": np.array(rec["expanded"], np.int64),
        "success": np.array(rec["success"], np.uint8),
        "path_off": np.array(rec["path_off"], np.int64), "path_len": np.array(rec["path_len"], np.int64),
        "path_boards": np.concatenate(rec["path_boards"]),
        "path_moves": np.concatenate(rec["path_moves"]),
        "path_scores": np.concatenate(rec["path_scores"]),
        "rb_off": np.array(rec["rb_off"], np.int64), "rb_len": np.array(rec["rb_len"], np.int64),
        "rb_s": np.concatenate(rec["rb_s"]), "rb_a": np.concatenate(rec["rb_a"]),
        "rb_r": np.concatenate(rec["rb_r"]), "rb_s2": np.concatenate(rec["rb_s2"]),
        "rb_d": np.concatenate(rec["rb_d"]),
    }
    np.savez_compressed(os.path.join(HERE, "astar.npz"), **out)


if __name__ == "__main__":
    main()
