"""Pins the CPU oracle (oracle/) against the reference's golden vectors (tests/golden/).

The fixtures were produced by running the Python reference itself in the build container
(tests/golden/gen_goldens.py); the oracle is trusted as the checker for the HIP kernels only
because it passes every test in this file.
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

from boards import boards_for_masks


def _exps(vals):
    v = np.asarray(vals, dtype=np.int64)
    out = np.zeros(v.shape, np.uint8)
    nz = v != 0
    out[nz] = np.log2(v[nz]).astype(np.uint8)
    return out


def test_reference_row_known_answers(golden_dir):
    # tests/test_game_board.py:5-27 (reference KATs)
    ref = json.load(open(os.path.join(golden_dir, "ref_tests.json")))
    for case in ref["rows"]:
        out, score = O.slide_row(_exps(case["in"]))
        assert list(out) == list(_exps(case["out"])), case
        assert score == case["score"], case


def test_reference_available_moves(golden_dir):
    # tests/test_game_board.py:30-59
    ref = json.load(open(os.path.join(golden_dir, "ref_tests.json")))
    for case in ref["legal_boards"]:
        m = O.legal_mask(_exps(case["state"]).reshape(16))
        assert [(m >> i) & 1 for i in range(4)] == case["mask_udlr"], case


def test_row_lut_exhaustive(golden_dir):
    # all 65 536 rows, src/board.py:92-126; sha256 prefix a0a4668c74681068
    g = np.load(os.path.join(golden_dir, "row_lut.npz"))
    res = np.zeros((65536, 4), np.uint8)
    score = np.zeros(65536, np.uint32)
    for i, row in enumerate(itertools.product(range(16), repeat=4)):
        res[i], score[i] = O.slide_row(np.array(row, np.uint8))
    assert np.array_equal(res, g["result"])
    assert np.array_equal(score, g["score"])
    stream = b"".join(bytes(res[i]) + int(score[i]).to_bytes(4, "little") for i in range(65536))
    assert hashlib.sha256(stream).hexdigest() == str(g["sha256"])
    assert str(g["sha256"]).startswith("a0a4668c74681068")


def test_trajectories_injected_spawns(golden_dir):
    # dqn_lib.play_one_step (src/dqn_lib.py:91-107) trajectories replayed with the landed spawns
    g = np.load(os.path.join(golden_dir, "trajectories.npz"))
    T = len(g["a"])
    for t in range(T):
        s = g["s"][t]
        assert O.legal_mask(s) == g["legal"][t]
        slid, gain = O.move(s, int(g["a"][t]))
        assert np.array_equal(slid, g["s_slide"][t])
        env = O.OracleEnv(1, seed=0, flags=O.NO_AUTORESET, reset=False)
        env.board[0] = s
        out = env.step(O.MODE_INJECT, actions=[g["a"][t]], spawn_idx=[g["spawn_idx"][t]],
                       spawn_exp=[g["spawn_exp"][t]])
        assert out["bad"] == (1 if (g["spawn_idx"][t] < 0 and not np.array_equal(slid, s)) else 0)
        assert np.array_equal(env.board[0], g["s2"][t]), t
        assert out["reward"][0] == g["reward"][t], t
        assert out["done"][0] == g["done"][t], t
        assert g["score_after"][t] - g["score_before"][t] == g["reward"][t]


def test_trajectory_episode_bookkeeping(golden_dir):
    # episodes end with the (s, a, 0, s, 1) self-transition (F6); rewards sum to the merge score
    g = np.load(os.path.join(golden_dir, "trajectories.npz"))
    for ep in np.unique(g["episode"]):
        sel = g["episode"] == ep
        d = g["done"][sel]
        assert d[-1] == 1 and d[:-1].sum() == 0
        assert np.array_equal(g["s"][sel][-1], g["s2"][sel][-1])
        assert g["reward"][sel].sum() == g["score_after"][sel][-1]


@pytest.mark.parametrize("field,dtype", [("action", np.float64), ("action_f32", np.float32)])
def test_egreedy_compat(golden_dir, field, dtype):
    # src/dqn_lib.py:25-29 including the precedence bug (F5)
    g = np.load(os.path.join(golden_dir, "egreedy.npz"))
    q = g["q"].astype(dtype)
    for i in range(len(q)):
        assert O.greedy(q[i], int(g["mask"][i])) == g[field][i], i
    assert np.array_equal(g["done"], (g["mask"] == 0).astype(np.uint8))


@pytest.mark.parametrize("suf,dtype", [("", np.float64), ("_f32", np.float32)])
def test_egreedy_compat_nonfinite(golden_dir, suf, dtype):
    """NaN / +-inf rows: torch.min/max propagate NaN, torch.argmax takes the first NaN."""
    g = np.load(os.path.join(golden_dir, "egreedy_nonfinite.npz"))
    q = g["q"].astype(dtype)
    assert np.isnan(q).any() and np.isinf(q).any()
    for i in range(len(q)):
        assert O.greedy(q[i], int(g["mask"][i])) == g["action" + suf][i], (i, q[i], g["mask"][i])


@pytest.mark.parametrize("suf,mode", [("", O.MODE_EGREEDY_F64), ("_f32", O.MODE_EGREEDY_F32)])
def test_oracle_env_qsum_nonfinite(golden_dir, suf, mode):
    """The oracle env step's Q-sum (episode log) adds the reference's torch.max(Q)."""
    g = np.load(os.path.join(golden_dir, "egreedy_nonfinite.npz"))
    boards = boards_for_masks(g["mask"], O.legal_mask)
    env = O.OracleEnv(len(boards), seed=1, flags=O.NO_AUTORESET, reset=False)
    env.board[:] = boards
    env.attach_episode_log(2)
    q = g["q"].astype(np.float64 if mode == O.MODE_EGREEDY_F64 else np.float32)
    out = env.step(mode, q=q, eps=0.0)
    assert np.array_equal(out["action"], g["action" + suf])
    assert np.array_equal(out["done"], g["done"])
    live = g["mask"] != 0
    assert np.array_equal(env.qsum[live], g["qmax" + suf][live], equal_nan=True)


def test_philox_known_answer():
    # Random123 / rocRAND philox4x32_10 known-answer vectors (kat_vectors: philox4x32 10 rounds)
    assert list(O.philox([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(O.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E,
                                                                   0xA20BC7C6, 0x6D5451FD]
    assert list(O.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                         [0xA4093822, 0x299F31D0])) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]
