"""GPU parity of the batched evaluation player (g2048.player) against the oracle driven by the
same policy rules: identical games (scores, lengths, max tiles) for the random, upleft and
greedy policies, histories in the reference's tuple format."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def P():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    from g2048 import player
    return player


def _oracle_games(n, seed, policy, model=None, flags=0):
    """Play with the oracle env until every game ended; same rules as BatchedPlayer.play."""
    from g2048.player import UpLeftState, encode_normalized, select_greedy
    o = O.OracleEnv(n, seed, flags=flags | O.NO_AUTORESET)
    fin = np.zeros(n, bool)
    out = {"score": np.zeros(n, np.int64), "moves": np.zeros(n, np.int64),
           "max": np.zeros(n, np.int64), "stuck": np.zeros(n, bool)}
    ul = UpLeftState(n, "cpu") if policy == "upleft" else None
    q0 = np.zeros((n, 4), np.float32)
    while not fin.all():
        stuck = np.zeros(n, bool)
        if policy == "random":
            r = o.step(O.MODE_EGREEDY_F32, q=q0, eps=1.0)
            ended = r["done"].astype(bool)
        elif policy == "upleft":
            act = ul.actions().numpy().astype(np.uint8)
            r = o.step(O.MODE_ACTIONS, actions=act)
            moved = ((r["legal"].astype(np.int64) >> act) & 1).astype(bool)
            ended = ul.update(torch.from_numpy(moved)).numpy()
        else:
            legal = np.array([O.legal_mask(b) for b in o.board], np.uint8)
            with torch.no_grad():
                q = model(encode_normalized(torch.from_numpy(o.board.copy()), torch.float64))
            act = select_greedy(q, torch.from_numpy(legal)).numpy().astype(np.uint8)
            r = o.step(O.MODE_ACTIONS, actions=act)
            ended = r["done"].astype(bool)
            stuck = (((legal.astype(np.int64) >> act) & 1) == 0) & ~ended & ~fin
            ended = ended | stuck
        new = ended & ~fin
        out["score"][new] = o.meta[new, 0]
        out["moves"][new] = o.meta[new, 1]
        out["max"][new] = o.board[new].max(axis=1)
        out["stuck"] |= stuck
        fin |= new
    out["max"] = np.where(out["max"] > 0, 1 << out["max"], 0)
    return out


def _check_same(res, want):
    np.testing.assert_array_equal(res.merge_score, want["score"])
    np.testing.assert_array_equal(res.moves, want["moves"])
    np.testing.assert_array_equal(res.max_tile, want["max"])
    np.testing.assert_array_equal(res.stuck, want["stuck"])


def test_random_policy_matches_oracle(P):
    n = 512
    res = P.BatchedPlayer(n, device=DEV, seed=21, record_games=6).play("random")
    _check_same(res, _oracle_games(n, 21, "random", flags=O.EGREEDY_FIXED))
    assert not res.stuck.any() and res.moves.min() > 10
    f = res.max_tile_frequency()
    assert f[1].sum() == n and set(f[0]) <= {2 ** k for k in range(1, 12)}
    # histories: reference play_game tuples, every non-terminal move legal
    for g, h in enumerate(res.histories):
        assert len(h) == res.moves[g]
        assert h[-1][1] == "u" and h[-1][2] == 0
        for k, (state, letter, reward, merge) in enumerate(h):
            e = np.where(state > 0, np.log2(np.maximum(state, 1)), 0).astype(np.uint8).reshape(16)
            mask = O.legal_mask(e)
            if k < len(h) - 1:
                assert (mask >> "udlr".index(letter)) & 1
            else:
                assert mask == 0
        assert h[-1][3] == res.merge_score[g]


def test_upleft_policy_matches_oracle(P):
    n = 384
    res = P.BatchedPlayer(n, device=DEV, seed=8, record_games=3).play("upleft")
    _check_same(res, _oracle_games(n, 8, "upleft"))
    for g, h in enumerate(res.histories):
        assert len(h) == res.moves[g]
        assert [x[1] for x in h[-4:]] == ["up", "left", "down", "r"]
        assert h[-1][3] == res.merge_score[g] and h[-1][2] == int(h[-1][0].sum())


@pytest.mark.parametrize("offset", [0.0, 50.0])
def test_greedy_policy_matches_oracle(P, offset):
    from g2048.nets import det_init, make_net
    n = 256
    cpu_model = det_init(make_net("conv", dtype=torch.float64), 1.7)
    with torch.no_grad():
        cpu_model._modules["7"].bias += offset
    gpu_model = det_init(make_net("conv", dtype=torch.float64, device=DEV), 1.7)
    with torch.no_grad():
        gpu_model._modules["7"].bias += offset
    res = P.BatchedPlayer(n, device=DEV, seed=4, model=gpu_model, record_games=2).play("greedy")
    want = _oracle_games(n, 4, "greedy", model=cpu_model)
    _check_same(res, want)
    if offset > 0:
        assert not res.stuck.any()
    # the legal-only rule never gets stuck
    res2 = P.BatchedPlayer(n, device=DEV, seed=4, model=gpu_model, rule="legal").play("greedy")
    assert not res2.stuck.any() and res2.moves.min() > 1


def test_play_n_games_writes_games_played(P, tmp_path):
    from g2048.experiment import Experiment, load_pickle
    exp = Experiment("rand", root=str(tmp_path))
    res = P.play_n_games(64, "random", experiment=exp, device=DEV, record_games=5)
    games = load_pickle(exp.folder, "games_played.p")
    assert len(games) == 5 and len(games[0]) == res.moves[0]
