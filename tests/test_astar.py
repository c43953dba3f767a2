"""A* replay pre-fill (src/state_space_search.py:46-131): the host search in libg2048.so against
runs of the reference's own A_star (tests/golden/gen_astar_goldens.py: deterministic
first-empty-cell spawns, smaller goal tiles), and path invariants under Philox spawns checked
with the oracle's move rule.  The search is host code: these run without a GPU."""
import os

import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "astar.npz"))


def test_search_matches_reference_runs(g):
    from g2048.astar import A_star, path_transitions

    for c in range(len(g["goal"])):
        res = A_star(g["start"][c], goal_tile=1 << int(g["goal"][c]), spawn="first-empty")
        assert res["visited_nodes"] == g["visited"][c], c
        assert res["expanded_nodes"] == g["expanded"][c], c
        assert res["success"] == bool(g["success"][c])
        o, n = int(g["path_off"][c]), int(g["path_len"][c])
        assert len(res["path_moves"]) == n
        assert np.array_equal(res["path_moves"], g["path_moves"][o:o + n])
        ob = o + c  # path_boards / path_scores hold len + 1 rows per case
        assert np.array_equal(res["path_boards"], g["path_boards"][ob:ob + n + 1])
        assert np.array_equal(res["path_scores"], g["path_scores"][ob:ob + n + 1])
        # generate_replay_buffer_using_A_star's transitions, reference (compat) format
        s, a, r, s2, d = path_transitions(res, compat=True)
        ro, rn = int(g["rb_off"][c]), int(g["rb_len"][c])
        assert np.array_equal(s, g["rb_s"][ro:ro + rn]) and np.array_equal(s2, g["rb_s2"][ro:ro + rn])
        assert np.array_equal(a, g["rb_a"][ro:ro + rn])
        assert np.array_equal(r, g["rb_r"][ro:ro + rn]) and np.array_equal(d, g["rb_d"][ro:ro + rn])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_philox_paths_are_legal_games(seed):
    """Every step of a Philox-spawn path is the oracle's move of the parent plus exactly one
    new tile (2 or 4) in a cell the move left empty, with the score growing by the move's
    merge gain; the goal tile is on the last board."""
    from g2048.astar import A_star

    start = np.zeros(16, np.uint8)
    rng = np.random.default_rng(seed)
    start[rng.choice(16, 2, replace=False)] = rng.integers(1, 3, 2)
    res = A_star(start, goal_tile=128, seed=seed, game=seed)
    assert res["success"] and res["path_length"] == len(res["path_moves"]) > 0
    pb, pm, ps = res["path_boards"], res["path_moves"], res["path_scores"]
    assert np.array_equal(pb[0], start) and ps[0] == 0
    for k in range(len(pm)):
        moved, gain = O.move(pb[k], int(pm[k]))
        assert not np.array_equal(moved, pb[k])
        diff = np.nonzero(pb[k + 1] != moved)[0]
        assert len(diff) == 1 and moved[diff[0]] == 0 and pb[k + 1][diff[0]] in (1, 2)
        assert ps[k + 1] - ps[k] == gain
    assert 7 in pb[-1]


def test_search_arguments_and_cap():
    from g2048 import _native as N
    from g2048.astar import A_star

    start = np.array([1, 1] + [0] * 14, np.uint8)
    res = A_star(start, goal_tile=2048, max_expansions=50)  # stopped by the cap
    assert not res["success"] and res["path_length"] == float("inf")
    assert res["expanded_nodes"] <= 53
    with pytest.raises(ValueError):
        A_star(start, goal_tile=3)
    with pytest.raises(N.NativeError):
        A_star(start, goal_tile=64, max_path=0)  # the path does not fit
