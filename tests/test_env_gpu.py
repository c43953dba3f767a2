"""GPU parity of the HIP env kernels (through the C ABI) against the CPU oracle and the
reference's golden vectors.  Bit-exact: this is integer / byte work."""
import itertools
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402
from boards import boards_for_masks, mask_boards  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def g2048():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    import g2048 as G
    G.load_native()
    return G


def _np(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _env_with(G, boards, **kw):
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 16)
    env = G.VecEnv2048(len(boards), device=DEV, reset=False, autoreset=False, **kw)
    env.board.copy_(torch.from_numpy(boards))
    return env


def _random_boards(n, seed):
    rng = np.random.default_rng(seed)
    fill = rng.uniform(0.2, 1.0, size=(n, 1))
    exps = rng.integers(1, 12, size=(n, 16))
    # bias toward equal neighbours so merges are common
    exps = np.where(rng.uniform(size=(n, 16)) < 0.3, np.roll(exps, 1, axis=1), exps)
    b = np.where(rng.uniform(size=(n, 16)) < fill, exps, 0).astype(np.uint8)
    b[:4] = 0
    b[4] = [1, 2, 1, 2, 2, 1, 2, 1, 1, 2, 1, 2, 2, 1, 2, 1]  # terminal checkerboard
    return b


def _mask_boards():
    return mask_boards()


# ------------------------------------------------------------------ slide / score / legal
@pytest.mark.parametrize("action", [0, 1, 2, 3])
def test_row_lut_all_directions(g2048, golden_dir, action):
    """All 65 536 rows (exponents 0..15) through every direction vs the reference LUT
    (src/board.py:92-126 via tests/golden/row_lut.npz)."""
    g = np.load(os.path.join(golden_dir, "row_lut.npz"))
    rows = np.array(list(itertools.product(range(16), repeat=4)), dtype=np.uint8)
    n = len(rows)
    boards = np.zeros((n, 4, 4), np.uint8)
    if action == 2:
        boards[:, 0, :] = rows
    elif action == 3:
        boards[:, 0, :] = rows[:, ::-1]
    elif action == 0:
        boards[:, :, 0] = rows
    else:
        boards[:, :, 0] = rows[:, ::-1]
    env = _env_with(g2048, boards.reshape(n, 16))
    changed = ~np.all(g["result"] == rows, axis=1)
    r, d, lg = env.step_inject(torch.full((n,), action, dtype=torch.uint8),
                               torch.full((n,), 15, dtype=torch.int8),
                               torch.full((n,), 2, dtype=torch.uint8))
    out = _np(env.board).reshape(n, 4, 4)
    got = {2: out[:, 0, :], 3: out[:, 0, ::-1], 0: out[:, :, 0], 1: out[:, ::-1, 0]}[action]
    assert np.array_equal(got, g["result"])
    assert np.array_equal(_np(r), np.where(changed, g["score"], 0).astype(np.int32))
    assert np.array_equal((_np(lg) >> action) & 1, changed.astype(np.uint8))
    assert np.array_equal(out[:, 3, 3], np.where(changed, 2, 0))
    assert env.error_count() == 0


@pytest.mark.parametrize("action", [0, 1, 2, 3])
def test_high_exponent_rows_vs_oracle(g2048, action):
    """Rows over exponents {0, 1, 14, 15, 16, 17} (tiles up to 131072, the largest a 4x4 game
    reaches; the reference LUT stops at 2^15) through every direction: board, merge score
    (a 65536 + 65536 merge scores 131072) and legal bit equal the oracle's
    src/board.py:92-126 restatement.  Parity beyond 2^15 rests on the oracle's value arithmetic."""
    from oracle import oracle as O
    exps = [0, 1, 14, 15, 16, 17]
    rows = np.array(list(itertools.product(exps, repeat=4)), dtype=np.uint8)
    n = len(rows)
    boards = np.zeros((n, 4, 4), np.uint8)
    if action == 2:
        boards[:, 0, :] = rows
    elif action == 3:
        boards[:, 0, :] = rows[:, ::-1]
    elif action == 0:
        boards[:, :, 0] = rows
    else:
        boards[:, :, 0] = rows[:, ::-1]
    ref = [O.slide_row(r) for r in rows]
    ref_rows = np.array([x[0] for x in ref], np.uint8)
    ref_score = np.array([x[1] for x in ref], np.int64)
    changed = ~np.all(ref_rows == rows, axis=1)
    env = _env_with(g2048, boards.reshape(n, 16))
    r, d, lg = env.step_inject(torch.full((n,), action, dtype=torch.uint8),
                               torch.full((n,), 15, dtype=torch.int8),
                               torch.full((n,), 1, dtype=torch.uint8))
    out = _np(env.board).reshape(n, 4, 4)
    got = {2: out[:, 0, :], 3: out[:, 0, ::-1], 0: out[:, :, 0], 1: out[:, ::-1, 0]}[action]
    assert np.array_equal(got, ref_rows)
    assert np.array_equal(_np(r).astype(np.int64), np.where(changed, ref_score, 0))
    assert int(ref_score.max()) == 2 * 262144  # [17, 17, 17, 17]: two 2^17 + 2^17 merges
    assert np.array_equal((_np(lg) >> action) & 1, changed.astype(np.uint8))
    assert env.error_count() == 0


def test_legal_mask_vs_oracle(g2048):
    b = _random_boards(20000, 1)
    env = _env_with(g2048, b)
    _, d, lg = env.step(torch.zeros(len(b), dtype=torch.uint8, device=DEV))
    exp = np.array([O.legal_mask(x) for x in b], np.uint8)
    assert np.array_equal(_np(lg), exp)
    assert np.array_equal(_np(d), (exp == 0).astype(np.uint8))


def test_reference_available_moves(g2048, golden_dir):
    import json
    ref = json.load(open(os.path.join(golden_dir, "ref_tests.json")))
    boards = []
    for case in ref["legal_boards"]:
        v = np.array(case["state"]).reshape(16)
        boards.append(np.where(v > 0, np.log2(np.maximum(v, 1)), 0).astype(np.uint8))
    env = _env_with(g2048, np.stack(boards))
    _, _, lg = env.step(torch.zeros(len(boards), dtype=torch.uint8, device=DEV))
    for m, case in zip(_np(lg), ref["legal_boards"]):
        assert [(int(m) >> i) & 1 for i in range(4)] == case["mask_udlr"]


def test_trajectories_injected(g2048, golden_dir):
    """Every step of the reference's play_one_step trajectories, replayed with the landed
    spawns: s', reward, done and legal mask bit-exact (src/dqn_lib.py:91-107)."""
    g = np.load(os.path.join(golden_dir, "trajectories.npz"))
    T = len(g["a"])
    env = _env_with(g2048, g["s"])
    r, d, lg = env.step_inject(torch.from_numpy(g["a"]), torch.from_numpy(g["spawn_idx"]),
                               torch.from_numpy(g["spawn_exp"]))
    assert np.array_equal(_np(env.board), g["s2"])
    assert np.array_equal(_np(r), g["reward"])
    assert np.array_equal(_np(d), g["done"])
    assert np.array_equal(_np(lg), g["legal"])
    # merge score accumulates like Board2048._mergescore
    assert np.array_equal(_np(env.score).astype(np.int64), g["reward"].astype(np.int64))
    assert env.error_count() == 0
    assert T > 2000


# ------------------------------------------------------------------ RNG modes vs oracle
@pytest.mark.parametrize("n,flags", [(4000, 0), (4096, O.P4_10), (777, 0), (1, 0), (63, O.P4_10)])
def test_random_steps_with_replay_vs_oracle(g2048, n, flags):
    seed = 0xC0FFEE + n
    kw = dict(p4=0.1 if flags & O.P4_10 else 0.5)
    env = g2048.VecEnv2048(n, seed=seed, device=DEV, board_offset=5 * n, **kw)
    rb = g2048.ReplayBuffer(3 * n, device=DEV)
    ref = O.OracleEnv(n, seed=seed, flags=flags, board_offset=5 * n)
    ref_rb = O.OracleReplay(3 * n)
    assert np.array_equal(_np(env.board), ref.board)
    for step in range(120):
        r, d, lg = env.step(None, replay=rb)
        o = ref.step(O.MODE_RANDOM, replay=ref_rb)
        if step % 17 == 0 or step == 119:
            assert np.array_equal(_np(env.board), ref.board), step
            assert np.array_equal(_np(r), o["reward"]), step
            assert np.array_equal(_np(d), o["done"]), step
            assert np.array_equal(_np(lg), o["legal"]), step
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    assert np.array_equal(_np(env.ep).view(np.uint32), ref.ep)
    assert np.array_equal(_np(env.clock).view(np.uint64), ref.clock)
    assert (ref.clock == 120).all()
    for name in ["s", "s2", "a", "r", "d"]:
        assert np.array_equal(_np(getattr(rb, name)), getattr(ref_rb, name)), name
    assert int(_np(rb.count)[0]) == int(ref_rb.count[0]) == 3 * n
    if n >= 64:
        assert ref.ep[:, 0].sum() > 0  # some episodes finished and auto-reset


def test_steps_across_clock_moves(g2048):
    """Single random-policy steps interleaved with rollouts and eps-greedy steps on one env (the
    three kernels share the group clock and the quad-based draws), and a state restored to an
    earlier clock (a checkpoint resume), all against the oracle; a partial last group
    (n % 64 != 0)."""
    n, seed = 64 * 37 + 21, 0x5EED
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    ref = O.OracleEnv(n, seed=seed)
    gen = np.random.default_rng(11)

    def check(tag):
        torch.cuda.synchronize()
        assert np.array_equal(_np(env.board), ref.board), tag
        assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta), tag
        assert np.array_equal(_np(env.clock).view(np.uint64), ref.clock), tag

    def steps(k, tag):
        for j in range(k):
            r, d, lg = env.step(None)
            o = ref.step(O.MODE_RANDOM)
            assert np.array_equal(_np(r), o["reward"]), (tag, j)
            assert np.array_equal(_np(d), o["done"]), (tag, j)
            assert np.array_equal(_np(lg), o["legal"]), (tag, j)
        check(tag)

    steps(2, "a")
    env.rollout(3)
    for _ in range(3):
        ref.step(O.MODE_RANDOM)
    steps(5, "b")  # clock 5..9: across a quad boundary
    q = gen.normal(size=(n, 4)).astype(np.float32)
    env.step_egreedy(torch.from_numpy(q).to(DEV), 0.5)
    ref.step(O.MODE_EGREEDY_F32, q=q, eps=0.5)
    steps(6, "c")
    saved = [t.clone() for t in (env.board, env.meta, env.ep, env.clock)]
    ref_saved = [a.copy() for a in (ref.board, ref.meta, ref.ep, ref.clock)]
    steps(7, "d")
    for t, v in zip((env.board, env.meta, env.ep, env.clock), saved):
        t.copy_(v)
    ref.board[...], ref.meta[...], ref.ep[...], ref.clock[...] = ref_saved
    steps(7, "e")
    steps(9, "f")


def test_actions_in_vs_oracle(g2048):
    n, seed = 3000, 99
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    ref = O.OracleEnv(n, seed=seed)
    gen = np.random.default_rng(5)
    for step in range(60):
        a = gen.integers(0, 4, size=n).astype(np.uint8)
        r, d, lg = env.step(torch.from_numpy(a).to(DEV))
        o = ref.step(O.MODE_ACTIONS, actions=a)
        assert np.array_equal(_np(r), o["reward"]), step
    assert np.array_equal(_np(env.board), ref.board)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)


@pytest.mark.parametrize("qdtype", [np.float32, np.float64])
@pytest.mark.parametrize("egreedy", ["compat", "fixed"])
@pytest.mark.parametrize("eps", [0.0, 0.3, 1.0])
def test_egreedy_fused_vs_oracle(g2048, qdtype, egreedy, eps):
    n, seed = 2500, 17
    flags = O.EGREEDY_FIXED if egreedy == "fixed" else 0
    env = g2048.VecEnv2048(n, seed=seed, device=DEV, egreedy=egreedy)
    rb = g2048.ReplayBuffer(4 * n, device=DEV)
    ref = O.OracleEnv(n, seed=seed, flags=flags)
    ref_rb = O.OracleReplay(4 * n)
    gen = np.random.default_rng(3)
    mode = O.MODE_EGREEDY_F32 if qdtype == np.float32 else O.MODE_EGREEDY_F64
    eps_t = torch.tensor([eps], dtype=torch.float64, device=DEV)
    for step in range(40):
        q = (gen.normal(size=(n, 4)) * gen.choice([0.1, 10.0, 1e3], size=(n, 1))).astype(qdtype)
        q[: n // 5] = -np.abs(q[: n // 5])
        a, r, d = env.step_egreedy(torch.from_numpy(q).to(DEV), eps_t if step % 2 else eps,
                                   replay=rb)
        o = ref.step(mode, q=q, eps=eps, replay=ref_rb)
        assert np.array_equal(_np(a), o["action"]), step
        assert np.array_equal(_np(r), o["reward"]), step
        assert np.array_equal(_np(d), o["done"]), step
    assert np.array_equal(_np(env.board), ref.board)
    for name in ["s", "s2", "a", "r", "d"]:
        assert np.array_equal(_np(getattr(rb, name)), getattr(ref_rb, name)), name


def test_egreedy_golden_rows(g2048, golden_dir):
    """The reference's epsilon_greedy_policy (src/dqn_lib.py:16-30, eps=0) on fixed Q rows:
    boards built to carry each row's legal mask."""
    g = np.load(os.path.join(golden_dir, "egreedy.npz"))
    # one board per legal mask value (found by search), reused for every row with that mask
    by_mask = {}
    for b in _mask_boards():
        by_mask.setdefault(O.legal_mask(b), b)
    assert len(by_mask) == 16
    boards = np.stack([by_mask[int(m)] for m in g["mask"]])
    for dt, field in [(np.float64, "action"), (np.float32, "action_f32")]:
        env = _env_with(g2048, boards)
        a, _, d = env.step_egreedy(torch.from_numpy(g["q"].astype(dt)).to(DEV), 0.0)
        assert np.array_equal(_np(a), g[field])
        assert np.array_equal(_np(d), g["done"])


def test_egreedy_nonfinite_golden_rows(g2048, golden_dir):
    """Q rows with NaN / +-inf / f32-overflowing products: the actions the reference's
    epsilon_greedy_policy takes (torch's NaN-propagating min/max, first-NaN argmax) and the
    torch.max(Q) it adds to the episode's Q-sum (src/dqn_lib.py:24-30)."""
    g = np.load(os.path.join(golden_dir, "egreedy_nonfinite.npz"))
    boards = boards_for_masks(g["mask"], O.legal_mask)
    live = g["mask"] != 0  # a terminal step resets the running Q-sum to 0
    for dt, suf in [(np.float64, ""), (np.float32, "_f32")]:
        env = _env_with(g2048, boards)
        log = env.attach_episode_log(2)
        a, _, d = env.step_egreedy(torch.from_numpy(g["q"].astype(dt)).to(DEV), 0.0)
        assert np.array_equal(_np(a), g["action" + suf])
        assert np.array_equal(_np(d), g["done"])
        qs = _np(log.qsum)
        assert np.array_equal(qs[live], g["qmax" + suf][live], equal_nan=True)


@pytest.mark.parametrize("n,p4", [(2048, 0.5), (2048 + 77, 0.1), (1, 0.5), (65, 0.5)])
def test_rollout_equals_single_steps(g2048, n, p4):
    """K random steps in one launch == K single steps: odd and even starting clocks (the pair
    block is split across launches), odd and even K, a partial last workgroup, both p4 modes,
    an episode log attached (terminal records + q-sum resets come from the rollout too), and a
    ring that wraps inside the launch."""
    seed = 4242
    e1 = g2048.VecEnv2048(n, seed=seed, device=DEV, p4=p4)
    e2 = g2048.VecEnv2048(n, seed=seed, device=DEV, p4=p4)
    l1, l2 = e1.attach_episode_log(64), e2.attach_episode_log(64)
    r1, r2 = g2048.ReplayBuffer(48 * n, device=DEV), g2048.ReplayBuffer(48 * n, device=DEV)
    rs = torch.zeros(n, dtype=torch.int64, device=DEV)
    acc = torch.zeros(n, dtype=torch.int64, device=DEV)
    total = 0
    for k in (3, 37, 64, 1, 0, 2):
        e1.rollout(k, replay=r1, reward_sum=rs)
        for _ in range(k):
            r, _, _ = e2.step(None, replay=r2)
            acc += r
        total += k
        assert torch.equal(e1.board, e2.board) and torch.equal(e1.meta, e2.meta), k
        assert torch.equal(e1.clock, e2.clock), k
    assert int(e1.clock.min()) == int(e1.clock.max()) == total
    assert torch.equal(e1.ep, e2.ep) and torch.equal(rs, acc)
    for name in ["s", "s2", "a", "r", "d", "count"]:
        assert torch.equal(getattr(r1, name), getattr(r2, name)), name
    g1, g2 = l1.read(), l2.read()
    if n >= 64:
        assert g1["step"].numel() > 0
    for f in g1:
        assert torch.equal(g1[f], g2[f]), f
    assert torch.equal(l1.qsum, l2.qsum)


def test_rollout_no_autoreset_equals_single_steps(g2048):
    """Without auto-reset (and no episode log: the rollout's general loop, not its lean one)
    finished boards stay terminal; K steps in one launch == K single steps, ring included."""
    n, seed = 2048 + 77, 515
    e1 = g2048.VecEnv2048(n, seed=seed, device=DEV, autoreset=False)
    e2 = g2048.VecEnv2048(n, seed=seed, device=DEV, autoreset=False)
    r1, r2 = g2048.ReplayBuffer(300 * n, device=DEV), g2048.ReplayBuffer(300 * n, device=DEV)
    for k in (1, 150, 99):
        e1.rollout(k, replay=r1)
        for _ in range(k):
            e2.step(None, replay=r2)
        assert torch.equal(e1.board, e2.board) and torch.equal(e1.meta, e2.meta), k
    assert torch.equal(e1.ep, e2.ep)
    assert int(e1.ep[:, 0].max()) > 0  # some boards finished (and stayed finished)
    for name in ["s", "s2", "a", "r", "d", "count"]:
        assert torch.equal(getattr(r1, name), getattr(r2, name)), name


def _rollout_ring(g2048, n, k, rb, seed=31):
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    env.step(None, replay=rb)  # odd start
    env.rollout(k, replay=rb)
    torch.cuda.synchronize()
    return env


def test_rollout_ring_layouts(g2048):
    """The rollout's ring stores through its three address paths give the same rows: one
    allocation (one buffer window), separately allocated sections in shuffled order (a window
    based at the lowest section), and a ring whose sections span more than 4 GiB (global
    stores)."""
    n, k = 4096 + 77, 21
    ref = g2048.ReplayBuffer(32 * n, device=DEV)
    e0 = _rollout_ring(g2048, n, k, ref)
    # separately allocated sections, in an order that puts d lowest and s highest
    c = 32 * n
    d = torch.zeros(c, dtype=torch.uint8, device=DEV)
    r = torch.zeros(c, dtype=torch.int32, device=DEV)
    a = torch.zeros(c, dtype=torch.uint8, device=DEV)
    s2 = torch.zeros((c, 16), dtype=torch.uint8, device=DEV)
    s = torch.zeros((c, 16), dtype=torch.uint8, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    sep = g2048.ReplayBuffer(c, device=DEV, sections=(s, s2, a, r, d, cnt))
    e1 = _rollout_ring(g2048, n, k, sep)
    # 2^27 + n rows (5.1 GB): past the 4 GiB window, the global-store instance
    big = g2048.ReplayBuffer((1 << 27) // n * n + n, device=DEV)
    e2 = _rollout_ring(g2048, n, k, big)
    rows = (k + 1) * n
    for e in (e1, e2):
        assert torch.equal(e.board, e0.board) and torch.equal(e.meta, e0.meta)
        assert torch.equal(e.ep, e0.ep)
    for name in ["s", "s2", "a", "r", "d"]:
        want = getattr(ref, name)[:rows]
        assert torch.equal(getattr(sep, name)[:rows], want), name
        assert torch.equal(getattr(big, name)[:rows], want), name
        assert int(getattr(big, name)[rows:].abs().sum() if name == "r"
                   else getattr(big, name)[rows:].sum()) == 0, name
    assert int(ref.count) == int(sep.count) == int(big.count) == rows
    del big
    torch.cuda.empty_cache()


@pytest.mark.parametrize("autoreset", [True, False])
def test_empty_board_is_terminal(g2048, autoreset):
    """An all-empty board has no legal move, so the random-policy step (lean_step) must report
    done (the oracle: legal == 0 -> done, src/dqn_lib.py:17-18) and, with auto-reset, deal a
    fresh board -- through the single step and the rollout, ring rows included."""
    n, seed = 777, 2024
    b = _random_boards(n, 9)
    b[::3] = 0  # every third board empty (b[:4] are empty already)
    flags = 0 if autoreset else O.NO_AUTORESET
    for use_rollout in (False, True):
        env = g2048.VecEnv2048(n, seed=seed, device=DEV, reset=False, autoreset=autoreset)
        env.board.copy_(torch.from_numpy(b))
        rb = g2048.ReplayBuffer(8 * n, device=DEV)
        ref = O.OracleEnv(n, seed=seed, flags=flags, reset=False)
        ref.board[:] = b
        ref_rb = O.OracleReplay(8 * n)
        if use_rollout:
            env.rollout(5, replay=rb)
        else:
            for _ in range(5):
                env.step(None, replay=rb)
        outs = [ref.step(O.MODE_RANDOM, replay=ref_rb) for _ in range(5)]
        assert outs[0]["done"][::3].all() and outs[0]["legal"][::3].max() == 0
        assert np.array_equal(_np(env.board), ref.board), use_rollout
        assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta), use_rollout
        assert np.array_equal(_np(env.ep).view(np.uint32), ref.ep), use_rollout
        for name in ["s", "s2", "a", "r", "d", "count"]:
            assert np.array_equal(_np(getattr(rb, name)), getattr(ref_rb, name)), (name, use_rollout)
        if not autoreset:
            assert not ref.board[::3].any()  # finished boards stay as they are
    # the single step's outputs agree with each other: done == (legal == 0)
    env = g2048.VecEnv2048(n, seed=seed, device=DEV, reset=False, autoreset=autoreset)
    env.board.copy_(torch.from_numpy(b))
    _, d, lg = env.step(None)
    assert np.array_equal(_np(d), (_np(lg) == 0).astype(np.uint8))


def test_rollout_vs_oracle(g2048):
    """The rollout against the CPU oracle directly (random-policy draws: half a Philox block per
    step), starting from an odd clock."""
    n, seed = 1000, 77
    env = g2048.VecEnv2048(n, seed=seed, device=DEV, board_offset=3 * n)
    rb = g2048.ReplayBuffer(40 * n, device=DEV)
    ref = O.OracleEnv(n, seed=seed, board_offset=3 * n)
    ref_rb = O.OracleReplay(40 * n)
    env.step(None, replay=rb)
    ref.step(O.MODE_RANDOM, replay=ref_rb)
    env.rollout(50, replay=rb)
    for _ in range(50):
        ref.step(O.MODE_RANDOM, replay=ref_rb)
    assert np.array_equal(_np(env.board), ref.board)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    assert np.array_equal(_np(env.ep).view(np.uint32), ref.ep)
    assert np.array_equal(_np(env.clock).view(np.uint64), ref.clock)
    for name in ["s", "s2", "a", "r", "d", "count"]:
        assert np.array_equal(_np(getattr(rb, name)), getattr(ref_rb, name)), name


def test_large_random_steps_vs_oracle(g2048):
    """Past 2^20 boards the step runs 256-thread workgroups (k_step<.., 256>), without the
    episode-counter prefetch above 2^18 boards: n = 2^20 + 77 (partial last block), random
    mode, replay append, checked against the oracle."""
    n, seed = (1 << 20) + 77, 5
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    rb = g2048.ReplayBuffer(3 * n, device=DEV)
    ref = O.OracleEnv(n, seed=seed)
    ref_rb = O.OracleReplay(3 * n)
    for step in range(3):
        r, d, _ = env.step(None, replay=rb)
        o = ref.step(O.MODE_RANDOM, replay=ref_rb)
        assert np.array_equal(_np(r), o["reward"]), step
        assert np.array_equal(_np(d), o["done"]), step
    assert np.array_equal(_np(env.board), ref.board)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    assert np.array_equal(_np(env.clock).view(np.uint64), ref.clock)
    for name in ["s", "s2", "a", "r", "d", "count"]:
        assert np.array_equal(_np(getattr(rb, name)), getattr(ref_rb, name)), name


def test_sample_encode_vs_oracle(g2048):
    n, seed = 1000, 7
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    rb = g2048.ReplayBuffer(8 * n, device=DEV)
    ref = O.OracleEnv(n, seed=seed)
    ref_rb = O.OracleReplay(8 * n)
    for _ in range(5):  # partially filled ring: count = 5n
        env.step(None, replay=rb)
        ref.step(O.MODE_RANDOM, replay=ref_rb)
    B = 4099
    idx = torch.randint(0, 5 * n, (B,), device=DEV)
    for dt in (torch.float32, torch.float64):
        s, a, r, s2, d, io = rb.sample_encode(B, dt, idx=idx)
        _, os_, oa, or_, os2, od = ref_rb.sample_f64(idx.cpu().numpy())
        assert np.array_equal(_np(s).astype(np.float64), os_)
        assert np.array_equal(_np(s2).astype(np.float64), os2)
        assert np.array_equal(_np(a), oa)
        assert np.array_equal(_np(r).astype(np.float64), or_)
        assert np.array_equal(_np(d).astype(np.float64), od)
    # in-kernel Philox indices: same draw as the oracle, inside [0, count)
    s, a, r, s2, d, io = rb.sample_encode(B, torch.float64, seed=123, epoch=9)
    oio, os_, oa, or_, os2, od = ref_rb.sample_f64(None, B=B, seed=123, epoch=9)
    assert np.array_equal(_np(io), oio) and np.array_equal(_np(s), os_)
    assert oio.max() < 5 * n and oio.min() >= 0


# ------------------------------------------------------------------ edge cases
def test_invalid_action_is_counted_noop(g2048):
    env = g2048.VecEnv2048(512, device=DEV, seed=1)
    before = env.board.clone()
    a = torch.zeros(512, dtype=torch.uint8, device=DEV)
    a[7] = 9
    r, _, _ = env.step(a)
    assert torch.equal(env.board[7], before[7]) and int(r[7]) == 0
    with pytest.raises(IndexError):
        env.check_errors()
    assert env.error_count() == 0


def test_reset_mask_and_episode_stats(g2048):
    n = 1000
    env = g2048.VecEnv2048(n, device=DEV, seed=2)
    ref = O.OracleEnv(n, seed=2)
    mask = (np.arange(n) % 3 == 0).astype(np.uint8)
    for _ in range(300):
        env.step(None)
        ref.step(O.MODE_RANDOM)
    env.reset(torch.from_numpy(mask).to(DEV))
    ref.reset(mask)
    assert np.array_equal(_np(env.board), ref.board)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    assert np.array_equal(_np(env.ep).view(np.uint32), ref.ep)


def test_spawn_distribution(g2048):
    """Spawn rule F3 (parity unpinned by the reference's tests; pinned here statistically):
    2 tiles per fresh board, value 4 with p = 0.5 (or 0.1), uniform over the 16 cells."""
    n = 1 << 18
    for p4 in (0.5, 0.1):
        env = g2048.VecEnv2048(n, device=DEV, seed=31, p4=p4)
        b = _np(env.board)
        assert np.all((b > 0).sum(1) == 2)
        vals = b[b > 0]
        assert set(np.unique(vals)) <= {1, 2}
        frac4 = (vals == 2).mean()
        assert abs(frac4 - p4) < 5 * np.sqrt(p4 * (1 - p4) / len(vals))
        cells = (b > 0).sum(0)
        expct = 2 * n / 16
        chi2 = ((cells - expct) ** 2 / expct).sum()
        assert chi2 < 45  # 15 dof, p ~ 1e-4


def test_sharded_boards_match_single_env(g2048):
    """Sharding (board_offset) reproduces the boards of one big env exactly."""
    n, seed = 2048, 77
    whole = g2048.VecEnv2048(2 * n, seed=seed, device=DEV)
    a = g2048.VecEnv2048(n, seed=seed, device=DEV, board_offset=0)
    b = g2048.VecEnv2048(n, seed=seed, device=DEV, board_offset=n)
    for _ in range(25):
        whole.step(None)
        a.step(None)
        b.step(None)
    assert torch.equal(whole.board, torch.cat([a.board, b.board]))


@pytest.mark.parametrize("qdtype", [np.float32, np.float64])
def test_egreedy_per_board_schedule_vs_oracle(g2048, qdtype):
    """src/dqn_lib.py:184-188 per board: eps_b from the board's own episode count."""
    n, seed = 3000, 23
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    rb = g2048.ReplayBuffer(4 * n, device=DEV)
    ref = O.OracleEnv(n, seed=seed)
    ref_rb = O.OracleReplay(4 * n)
    eps_counts = np.random.default_rng(1).integers(0, 1500, size=n).astype(np.int32)
    env.ep[:, 0] = torch.from_numpy(eps_counts).to(DEV)
    ref.ep[:, 0] = eps_counts.view(np.uint32)
    gen = np.random.default_rng(4)
    mode = O.MODE_EGREEDY_F32 if qdtype == np.float32 else O.MODE_EGREEDY_F64
    for step in range(30):
        q = gen.normal(size=(n, 4)).astype(qdtype)
        a, r, d = env.step_egreedy(torch.from_numpy(q).to(DEV), None, replay=rb,
                                   eps_schedule=(1000.0, 0.01))
        o = ref.step(mode, q=q, replay=ref_rb, eps_schedule=(1000.0, 0.01))
        assert np.array_equal(_np(a), o["action"]), step
        assert np.array_equal(_np(r), o["reward"]), step
    assert np.array_equal(_np(env.board), ref.board)
    assert np.array_equal(_np(rb.s2), ref_rb.s2)


@pytest.mark.parametrize("qdt", [np.float32, np.float64])
def test_episode_log_matches_oracle(g2048, qdt):
    """In-kernel episode log (g2048_env_set_episode_log) == oracle records, field by field,
    over eps-greedy steps with the per-board schedule (many episodes per board), read in chunks."""
    n, steps = 512, 300
    env = g2048.VecEnv2048(n, seed=11, device=DEV)
    log = env.attach_episode_log(8)
    o = O.OracleEnv(n, 11)
    o.attach_episode_log(8)
    rng = np.random.default_rng(3)
    mode = O.MODE_EGREEDY_F32 if qdt == np.float32 else O.MODE_EGREEDY_F64
    total = 0
    for t in range(steps):
        q = rng.standard_normal((n, 4)).astype(qdt)
        env.step_egreedy(torch.from_numpy(q).to(DEV), None, eps_schedule=(40.0, 0.05))
        o.step(mode, q=q, eps_schedule=(40.0, 0.05))
        if t % 100 == 99:
            got, want = log.read(), o.episodes()
            assert len(got["step"]) == len(want)
            total += len(want)
            for f in ("step", "board", "episode", "score", "moves", "max_exp"):
                np.testing.assert_array_equal(got[f].numpy(), want[f].astype(np.int64), err_msg=f)
            np.testing.assert_array_equal(got["q_sum"].numpy(), want["q_sum"])  # same f64 sums
    assert total > 500 and log.total() == total
    np.testing.assert_array_equal(_np(env.ep), o.ep.view(np.int32))
    assert log.read()["step"].numel() == 0  # nothing new since the last read


def test_episode_log_rollout_and_overflow(g2048):
    n = 256
    env = g2048.VecEnv2048(n, seed=5, device=DEV)
    log = env.attach_episode_log(1)
    env.rollout(400)
    with pytest.raises(RuntimeError, match="overflow"):
        log.read()
    env2 = g2048.VecEnv2048(n, seed=5, device=DEV)
    log2 = env2.attach_episode_log(16)
    env2.rollout(200)
    o = O.OracleEnv(n, 5)
    o.attach_episode_log(16)
    for _ in range(200):
        o.step(O.MODE_RANDOM)
    got, want = log2.read(), o.episodes()
    for f in ("step", "board", "episode", "score", "moves", "max_exp"):
        np.testing.assert_array_equal(got[f].numpy(), want[f].astype(np.int64), err_msg=f)
    assert float(got["q_sum"].abs().sum()) == 0.0  # random policy: max_q_value = 0 (:19)
    log2.detach()
    before = _np(log2.raw).copy()
    env2.rollout(50)
    np.testing.assert_array_equal(_np(log2.raw), before)  # detached: nothing written


def test_legal_mask_kernel(g2048):
    boards = np.concatenate([_mask_boards(), _random_boards(2000, 9)])
    env = _env_with(g2048, boards)
    got = _np(env.legal_mask())
    want = np.array([O.legal_mask(b) for b in boards], np.uint8)
    np.testing.assert_array_equal(got, want)
    assert set(np.unique(got)) == set(range(16))
    uv = _np(env.available_moves_as_unit_vectors())
    np.testing.assert_array_equal(uv, ((want[:, None] >> np.arange(4)) & 1).astype(np.float32))


def test_epoch_roundtrip(g2048):
    a = g2048.VecEnv2048(64, seed=2, device=DEV)
    a.reset()
    a.reset()
    assert a.epoch == 3  # construction reset + 2
    b = g2048.VecEnv2048(64, seed=2, device=DEV)
    b.epoch = a.epoch
    a.reset()
    b.reset()
    np.testing.assert_array_equal(_np(a.board), _np(b.board))


@pytest.mark.parametrize("mode", ["scalar", "schedule"])
def test_fused_dense64_step_matches_forward_plus_step(g2048, mode):
    """g2048_env_step_egreedy_dense64 (Q computed in the step kernel) == g2048_dense64_forward +
    g2048_env_step_egreedy, bit for bit: Q, actions, boards, rewards, replay, episode log."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    n = 4096 + 77
    m = det_init(make_net("dense64", torch.float32, DEV), 0.7)
    p = qnet.net_params(m)
    kw = dict(eps_schedule=(30.0, 0.05)) if mode == "schedule" else {}
    envs, rbs, logs = [], [], []
    for _ in range(2):
        e = g2048.VecEnv2048(n, seed=9, device=DEV)
        rbs.append(g2048.ReplayBuffer(8 * n, device=DEV))
        logs.append(e.attach_episode_log(16))
        e.rollout(30)
        envs.append(e)
    qf = torch.empty((n, 4), dtype=torch.float32, device=DEV)
    for t in range(60):
        a0, r0, d0 = envs[0].step_egreedy_dense64(p, 0.2, replay=rbs[0], q_out=qf, **kw)
        q = qnet.forward(m, envs[1].board)
        a1, r1, d1 = envs[1].step_egreedy(q, 0.2, replay=rbs[1], **kw)
        torch.cuda.synchronize()
        assert torch.equal(qf, q), t
        assert torch.equal(a0, a1) and torch.equal(r0, r1) and torch.equal(d0, d1), t
    for name in ("board", "meta", "ep", "clock"):
        assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), name
    for name in ("s", "s2", "a", "r", "d", "count"):
        assert torch.equal(getattr(rbs[0], name), getattr(rbs[1], name)), name
    g0, g1 = logs[0].read(), logs[1].read()
    for f in g0:
        assert torch.equal(g0[f], g1[f]), f


@pytest.mark.parametrize("mode", ["eps1", "schedule"])
def test_fused_dense64_step_skips_explorers(g2048, mode):
    """Without q_out the dense-64 step skips the MLP of every 64-board group whose boards all
    take the explore branch (the model runs only on the greedy branch, src/dqn_lib.py:20-24).
    Groups of all-new boards (eps = 1) sit next to groups with eps 0.9 and 0.05: the trajectory
    is still bitwise forward + step, episode q-sums included."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    n = 4096 + 77
    m = det_init(make_net("dense64", torch.float32, DEV), 0.7)
    p = qnet.net_params(m)
    kw = dict(eps_schedule=(30.0, 0.05)) if mode == "schedule" else {}
    eps = 1.0 if mode == "eps1" else 0.0
    grp = torch.arange(n, device=DEV) // 64 % 3
    ep0 = torch.where(grp == 0, 0, torch.where(grp == 1, 3, 100)).to(torch.int32)
    envs, rbs, logs = [], [], []
    for _ in range(2):
        e = g2048.VecEnv2048(n, seed=21, device=DEV)
        rbs.append(g2048.ReplayBuffer(8 * n, device=DEV))
        e.rollout(30)
        e.ep[:, 0] = ep0
        logs.append(e.attach_episode_log(16))  # (counts from the episodes set here)
        envs.append(e)
    for t in range(60):
        a0, r0, d0 = envs[0].step_egreedy_dense64(p, eps, replay=rbs[0], **kw)
        q = qnet.forward(m, envs[1].board)
        a1, r1, d1 = envs[1].step_egreedy(q, eps, replay=rbs[1], **kw)
        torch.cuda.synchronize()
        assert torch.equal(a0, a1) and torch.equal(r0, r1) and torch.equal(d0, d1), t
    for name in ("board", "meta", "ep", "clock"):
        assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), name
    for name in ("s", "s2", "a", "r", "d", "count"):
        assert torch.equal(getattr(rbs[0], name), getattr(rbs[1], name)), name
    g0, g1 = logs[0].read(), logs[1].read()
    for f in g0:
        assert torch.equal(g0[f], g1[f]), f
    assert torch.equal(logs[0].qsum, logs[1].qsum)


def test_fused_dense64_step_f64(g2048):
    """g2048_env_step_egreedy_dense64_f64: the in-kernel float64 Q equals the torch float64 net to
    1e-12 relative, and stepping on it equals g2048_env_step_egreedy fed the same Q, bit for bit
    (actions, boards, rewards, replay, episode q-sums)."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    n = 4096 + 77
    m = det_init(make_net("dense64", torch.float64, DEV), 0.7)
    p = qnet.Dense64Update64(m, m, 64).on  # the float64 parameter struct
    envs, rbs, logs = [], [], []
    for _ in range(2):
        e = g2048.VecEnv2048(n, seed=19, device=DEV)
        rbs.append(g2048.ReplayBuffer(8 * n, device=DEV))
        logs.append(e.attach_episode_log(16))
        e.rollout(30)
        envs.append(e)
    qf = torch.empty((n, 4), dtype=torch.float64, device=DEV)
    for t in range(40):
        with torch.no_grad():
            ref = m(envs[1].encode(torch.float64, conv=False)).reshape(n, 4)
        a0, r0, d0 = envs[0].step_egreedy_dense64(p, 0.3, replay=rbs[0], q_out=qf, f64=True,
                                                  eps_schedule=(30.0, 0.05))
        torch.cuda.synchronize()
        torch.testing.assert_close(qf, ref, rtol=1e-12, atol=1e-12 * float(ref.abs().max()))
        a1, r1, d1 = envs[1].step_egreedy(qf.clone(), 0.3, replay=rbs[1],
                                          eps_schedule=(30.0, 0.05))
        torch.cuda.synchronize()
        assert torch.equal(a0, a1) and torch.equal(r0, r1) and torch.equal(d0, d1), t
    for name in ("board", "meta", "ep", "clock"):
        assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), name
    for name in ("s", "s2", "a", "r", "d", "count"):
        assert torch.equal(getattr(rbs[0], name), getattr(rbs[1], name)), name
    assert torch.equal(logs[0].qsum, logs[1].qsum)


@pytest.mark.parametrize("n,rows", [(64 * 20 + 37, 6), (64 * 20 + 37, 8), ((1 << 18) + 64, 8)])
def test_clock_past_2_32_vs_oracle(g2048, n, rows):
    """Step clocks crossing 2^32 (the ring row switches to its 64-bit modulo, the Philox counter
    to its high word): single steps and rollouts -- rows % 4 == 0 takes the lean kernel's quad-row
    path, 6 the other, and from 2^18 boards the warp-specialised kernel runs -- with a ring of
    `rows` rows per board, against the oracle on every output, ring row and clock; a partial last
    clock group."""
    seed = 0xC10C
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    rb = g2048.ReplayBuffer(rows * n, device=DEV)
    ref = O.OracleEnv(n, seed=seed)
    ref_rb = O.OracleReplay(rows * n)
    t0 = (1 << 32) - 5
    env.clock.fill_(t0)
    # the episodes start at t0 too: meta's start row holds the clock's low word (ABI v5), so
    # moving the clock without it would count t0 moves
    env.meta[1].fill_(t0 - (1 << 32))  # (uint32) t0 as int32
    ref.clock[:] = t0
    for step in range(4):
        r, d, lg = env.step(None, replay=rb)
        o = ref.step(O.MODE_RANDOM, replay=ref_rb)
        assert np.array_equal(_np(r), o["reward"]), step
        assert np.array_equal(_np(lg), o["legal"]), step
    env.rollout(7, replay=rb)
    for _ in range(7):
        ref.step(O.MODE_RANDOM, replay=ref_rb)
    q = np.random.default_rng(n).normal(size=(n, 4)).astype(np.float32)
    a, r, d = env.step_egreedy(torch.from_numpy(q).to(DEV), 0.5, replay=rb)  # DOMAIN_STEP draws
    o = ref.step(O.MODE_EGREEDY_F32, q=q, eps=0.5, replay=ref_rb)
    assert np.array_equal(_np(a), o["action"]) and np.array_equal(_np(r), o["reward"])
    torch.cuda.synchronize()
    assert np.array_equal(_np(env.clock).view(np.uint64), ref.clock)
    assert int(ref.clock[0]) == t0 + 12 and t0 + 12 > (1 << 32)
    assert int(_np(rb.count)[0]) == int(ref_rb.count[0]) == rows * n
    assert np.array_equal(_np(env.board), ref.board)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    for name in ["s", "s2", "a", "r", "d"]:
        assert np.array_equal(_np(getattr(rb, name)), getattr(ref_rb, name)), name


def test_meta_start_row_mid_episode_vs_oracle(g2048):
    """ABI v5 meta: a caller-set state mid-episode -- clock C, scores, and moves m given as start
    rows C - m (mod 2^32, so some starts wrap below zero) -- steps like the oracle holding
    {score, m}: single steps, a rollout and an explicit reset, with score_moves() equal to the
    oracle's pairs after each, and the start rows of boards that did not finish unchanged."""
    n, seed = 1000, 0x5EED
    rng = np.random.default_rng(3)
    env = g2048.VecEnv2048(n, seed=seed, device=DEV)
    ref = O.OracleEnv(n, seed=seed)
    clock = 123_456
    score = rng.integers(0, 1 << 20, n).astype(np.uint32)
    moves = rng.integers(0, 1 << 31, n).astype(np.uint32)  # many moves > clock: starts wrap
    moves[:5] = [0, 1, clock, clock + 1, (1 << 32) - 1]
    start = (np.uint64(clock) - moves.astype(np.uint64)) & np.uint64(0xFFFFFFFF)
    env.clock.fill_(clock)
    env.meta[0].copy_(torch.from_numpy(score.view(np.int32)))
    env.meta[1].copy_(torch.from_numpy(start.astype(np.uint32).view(np.int32)))
    ref.clock[:] = clock
    ref.meta[:, 0] = score
    ref.meta[:, 1] = moves
    ref.board[:] = _np(env.board)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    before = _np(env.meta[1]).copy()
    for _ in range(3):
        env.step(None)
        ref.step(O.MODE_RANDOM)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    ended = _np(env.ep)[:, 0] > 0
    assert np.array_equal(_np(env.meta[1])[~ended], before[~ended])
    env.rollout(9)
    for _ in range(9):
        ref.step(O.MODE_RANDOM)
    assert np.array_equal(_np(env.score_moves()).view(np.uint32), ref.meta)
    mask = (np.arange(n) % 4 == 1).astype(np.uint8)
    env.reset(torch.from_numpy(mask).to(DEV))
    ref.reset(mask)
    sm = _np(env.score_moves()).view(np.uint32)
    assert np.array_equal(sm, ref.meta) and not sm[mask == 1].any()
    assert np.array_equal(_np(env.board), ref.board)
    assert np.array_equal(_np(env.ep).view(np.uint32), ref.ep)


def test_score_moves_errors(g2048):
    """g2048_env_score_moves: NULL arguments and a misaligned output are G2048_EINVAL."""
    import ctypes as C
    from g2048 import _native as N
    env = g2048.VecEnv2048(64, device=DEV)
    lib = N.load()
    out = torch.zeros(64 * 2 + 2, dtype=torch.int32, device=DEV)
    s = N.stream_of(env.device)
    assert lib.g2048_env_score_moves(None, N.ptr(out), s) == N.G2048_EINVAL
    assert lib.g2048_env_score_moves(env._h, None, s) == N.G2048_EINVAL
    assert lib.g2048_env_score_moves(env._h, C.c_void_p(N.ptr(out) + 4), s) == N.G2048_EINVAL
    assert lib.g2048_env_score_moves(env._h, N.ptr(out), s) == N.G2048_OK
