"""Evaluation-player logic on CPU against the reference's own Player runs
(tests/golden/player.npz, made by tests/golden/gen_player_goldens.py): the upleft state machine
and the greedy selection rule / normalized encoding, plus quirk handling (illegal argmax)."""
import os

import numpy as np
import pytest
import torch

from g2048.nets import det_init, make_net
from g2048.player import UpLeftState, encode_normalized, legal_bits, select_greedy
from oracle import oracle as O

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "player.npz"))


def test_upleft_state_machine_matches_reference():
    starts, lens = GOLD["upleft_start"], GOLD["upleft_len"]
    after, acts = GOLD["upleft_after"], GOLD["upleft_action"]
    off = 0
    for g in range(len(lens)):
        st = UpLeftState(1, "cpu")
        board = starts[g]
        for k in range(lens[g]):
            a = int(st.actions()[0])
            assert a == acts[off + k], (g, k)
            slid, _ = O.move(board, a)
            moved = not np.array_equal(slid, board)
            assert moved == (not np.array_equal(after[off + k], board))
            ended = bool(st.update(torch.tensor([moved]))[0])
            assert ended == (k == lens[g] - 1), (g, k)
            board = after[off + k]
        assert O.legal_mask(board) == 0  # the reference stops only on a dead board
        off += lens[g]
    assert off == len(acts)


def test_greedy_rule_matches_reference():
    b, leg, q, a = GOLD["greedy_board"], GOLD["greedy_legal"], GOLD["greedy_q"], GOLD["greedy_action"]
    # legal masks: the reference's available_moves == the oracle / kernel mask
    np.testing.assert_array_equal(leg, [O.legal_mask(x) for x in b])
    got = select_greedy(torch.from_numpy(q), torch.from_numpy(leg), "reference")
    np.testing.assert_array_equal(got.numpy(), a)


def test_greedy_normalized_encoding_reproduces_reference_q():
    b, q = GOLD["greedy_board"], GOLD["greedy_q"]
    lens, phases, offs = GOLD["greedy_len"], GOLD["greedy_phase"], GOLD["greedy_offset"]
    off = 0
    for g in range(len(lens)):
        m = det_init(make_net("conv", dtype=torch.float64), float(phases[g]))
        with torch.no_grad():
            m._modules["7"].bias += float(offs[g])
            x = encode_normalized(torch.from_numpy(b[off:off + lens[g]]), torch.float64)
            mine = m(x).numpy()
        np.testing.assert_allclose(mine, q[off:off + lens[g]], rtol=1e-12, atol=1e-12)
        off += lens[g]


def test_stuck_games_are_an_illegal_argmax():
    leg, a, lens, stuck = (GOLD["greedy_legal"], GOLD["greedy_action"], GOLD["greedy_len"],
                           GOLD["greedy_stuck"])
    assert stuck.any() and (~stuck).any()
    off = 0
    for g in range(len(lens)):
        m, act = leg[off:off + lens[g]], a[off:off + lens[g]]
        legal_pick = (m.astype(int) >> act.astype(int)) & 1
        assert legal_pick[:-1].all()
        if stuck[g]:
            assert m[-1] != 0 and legal_pick[-1] == 0
        else:
            assert m[-1] == 0 and act[-1] == 0  # terminal step: argmax of zeros
        off += lens[g]


def test_legal_rule_never_picks_illegal():
    rng = np.random.default_rng(0)
    q = torch.from_numpy(rng.standard_normal((4000, 4)) - 3.0)
    leg = torch.from_numpy(rng.integers(0, 16, 4000).astype(np.uint8))
    a = select_greedy(q, leg, "legal")
    ok = ((leg.to(torch.int64) >> a) & 1).bool() | (leg == 0)
    assert bool(ok.all())
    ref = select_greedy(q, leg, "reference")  # all-negative Q: the reference picks illegal
    assert bool((((leg.to(torch.int64) >> ref) & 1) == 0)[leg > 0].any())
    assert legal_bits(torch.tensor([5], dtype=torch.uint8)).tolist() == [[1, 0, 1, 0]]
