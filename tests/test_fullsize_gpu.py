"""The benchmarked configuration itself against the CPU oracle, and the
headline rollout kernel (k_rollout_lean: ring in one buffer window, auto-reset, no episode log)
against K single steps from every clock phase.

Full size = BASELINE configs[1] exactly as bench.py times it: 65 536 boards, one rollout launch of
K = 64 steps into an N*K-row ring.  The oracle (oracle/oracle2048.c) steps three 1 000-board
slices -- start, middle, end -- as envs of their own with board_offset = the slice's first global
id: Philox draws are keyed by global board id (include/g2048.h), so a slice is exact.  Compared:
boards, meta, episode counters, clocks, and every ring row of the slice's boards.  Reference
semantics: src/dqn_lib.py:91-107 (play_one_step + append), src/board.py:41-51, 92-126."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N, K = 65536, 64
SLICES = (0, 32768 - 512, N - 1000)


@pytest.fixture(scope="module")
def g2048():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    return g2048


def _np(t):
    return t.detach().cpu().numpy()


def test_bench_rollout_full_size_vs_oracle(g2048):
    """bench_rollout's launch (65 536 boards x K = 64, N*K ring) == the oracle on three slices."""
    seed = 0x2048
    env = g2048.VecEnv2048(N, seed=seed, device=DEV)
    rb = g2048.ReplayBuffer(N * K, device=DEV)
    env.rollout(K, replay=rb)
    torch.cuda.synchronize()
    board, meta, ep = _np(env.board), _np(env.score_moves()).view(np.uint32), _np(env.ep).view(np.uint32)
    ring = {name: _np(getattr(rb, name)) for name in ["s", "s2", "a", "r", "d"]}
    assert int(rb.count) == N * K
    assert (_np(env.clock).view(np.uint64) == K).all()
    for i0 in SLICES:
        n = 1000
        ref = O.OracleEnv(n, seed=seed, board_offset=i0)
        ref_rb = O.OracleReplay(n * K)
        for _ in range(K):
            ref.step(O.MODE_RANDOM, replay=ref_rb)
        sl = slice(i0, i0 + n)
        assert np.array_equal(board[sl], ref.board), i0
        assert np.array_equal(meta[sl], ref.meta), i0
        assert np.array_equal(ep[sl], ref.ep), i0
        # ring row of (step t, board i) = t * N + i  vs  t * n + (i - i0) in the slice's ring
        rows = (np.arange(K)[:, None] * N + np.arange(i0, i0 + n)[None, :]).reshape(-1)
        for name in ["s", "s2", "a", "r", "d"]:
            assert np.array_equal(ring[name][rows], getattr(ref_rb, name)), (i0, name)
        assert ref.ep[:, 0].sum() > 0  # episodes ended and auto-reset inside the launch


@pytest.mark.parametrize("n_all", [(1 << 18) - 64, (1 << 18) + 37, (1 << 20) + 4160])
def test_rollout_large_n_vs_oracle(g2048, n_all):
    """256k / 1 M boards, ring of N*16 rows, one launch of 3 steps and four of 16 -- every clock
    phase -- against the oracle on four 1 000-board slices.  Just below 256k boards
    k_rollout_lean runs (its quad-row path; its first version, under store-queue back-pressure,
    stored some boards with the first word already rewritten by the next instruction: store_board
    in g2048.hip).  From 256k boards on (the second case, ragged: a partly live last workgroup)
    the warp-specialised k_rollout_ws runs; 2^18 + 37: its last wave holds 37 live boards."""
    k, seed = 16, 7
    env = g2048.VecEnv2048(n_all, seed=seed, device=DEV)
    rb = g2048.ReplayBuffer(n_all * k, device=DEV)
    env.rollout(3, replay=rb)
    for _ in range(3):
        env.rollout(k, replay=rb)
    rs = torch.zeros(n_all, dtype=torch.int64, device=DEV)
    env.rollout(k, replay=rb, reward_sum=rs)  # the reward-sum instance for the last launch
    torch.cuda.synchronize()
    board = _np(env.board)
    ring = {name: _np(getattr(rb, name)) for name in ["s", "s2", "a", "r", "d"]}
    # the last launch wrote all k rows: its reward sums are the rows' rewards per board
    assert np.array_equal(_np(rs), ring["r"].reshape(k, n_all).astype(np.int64).sum(0))
    for i0 in (0, 68000, n_all // 2, n_all - 1000):
        n = 1000
        ref = O.OracleEnv(n, seed=seed, board_offset=i0)
        ref_rb = O.OracleReplay(n * k)
        for _ in range(3 + 4 * k):
            ref.step(O.MODE_RANDOM, replay=ref_rb)
        assert np.array_equal(board[i0:i0 + n], ref.board), i0
        rows = (np.arange(k)[:, None] * n_all + np.arange(i0, i0 + n)[None, :]).reshape(-1)
        for name in ["s", "s2", "a", "r", "d"]:
            assert np.array_equal(ring[name][rows], getattr(ref_rb, name)), (i0, name)


@pytest.mark.parametrize("p4", [0.5, 0.1])
def test_ws_rollout_equals_single_steps(g2048, p4):
    """The large-N kernel (k_rollout_ws: compute and store waves handing transitions over through
    an LDS ring, nt stores) == single steps at 1 M + 64 boards, both p(4) modes, reward sums on
    and off, launches of 5 / 16 / 11 steps (every clock phase, a ring that wraps inside a launch),
    and no hand-over timeouts (the env's error counter stays 0)."""
    n, seed = (1 << 20) + 64, 99
    e1 = g2048.VecEnv2048(n, seed=seed, device=DEV, p4=p4)
    e2 = g2048.VecEnv2048(n, seed=seed, device=DEV, p4=p4)
    r1, r2 = g2048.ReplayBuffer(24 * n, device=DEV), g2048.ReplayBuffer(24 * n, device=DEV)
    rs = torch.zeros(n, dtype=torch.int64, device=DEV)
    acc = torch.zeros(n, dtype=torch.int64, device=DEV)
    for j, k in enumerate((5, 16, 11)):
        e1.rollout(k, replay=r1, reward_sum=rs if j % 2 else None)
        for _ in range(k):
            r, _, _ = e2.step(None, replay=r2)
            if j % 2:
                acc += r
        assert torch.equal(e1.board, e2.board) and torch.equal(e1.meta, e2.meta), k
        assert torch.equal(e1.clock, e2.clock) and torch.equal(e1.ep, e2.ep), k
    assert torch.equal(rs, acc)
    for name in ["s", "s2", "a", "r", "d", "count"]:
        assert torch.equal(getattr(r1, name), getattr(r2, name)), name
    assert int(e1.ep[:, 0].sum()) > 0
    e1.check_errors()


@pytest.mark.parametrize("qdtype", [np.float32, np.float64])
def test_egreedy_step_full_size_vs_oracle(g2048, qdtype):
    """One fused epsilon-greedy step (g2048_env_step_egreedy, src/dqn_lib.py:16-30,91-107) at
    65 536 boards, eps = 0.3, random Q rows, ring append == the oracle on three slices."""
    seed = 4096
    env = g2048.VecEnv2048(N, seed=seed, device=DEV)
    rb = g2048.ReplayBuffer(4 * N, device=DEV)
    env.rollout(7, replay=None)  # some history (odd clock)
    q = np.random.default_rng(11).normal(size=(N, 4)).astype(qdtype)
    a, r, d = env.step_egreedy(torch.from_numpy(q).to(DEV), 0.3, replay=rb)
    torch.cuda.synchronize()
    board = _np(env.board)
    mode = O.MODE_EGREEDY_F32 if qdtype == np.float32 else O.MODE_EGREEDY_F64
    for i0 in SLICES:
        n = 1000
        ref = O.OracleEnv(n, seed=seed, board_offset=i0)
        for _ in range(7):
            ref.step(O.MODE_RANDOM)
        ref_rb = O.OracleReplay(4 * n)
        # the oracle's ring holds rows of step 7 at (7 mod 4) * n
        o = ref.step(mode, q=np.ascontiguousarray(q[i0:i0 + n]), eps=0.3, replay=ref_rb)
        sl = slice(i0, i0 + n)
        assert np.array_equal(_np(a)[sl], o["action"]), i0
        assert np.array_equal(_np(r)[sl], o["reward"]), i0
        assert np.array_equal(_np(d)[sl], o["done"]), i0
        assert np.array_equal(board[sl], ref.board), i0
        rows = 3 * N + np.arange(i0, i0 + n)
        for name in ["s", "s2", "a", "r", "d"]:
            assert np.array_equal(_np(getattr(rb, name))[rows],
                                  getattr(ref_rb, name)[3 * n:4 * n]), (i0, name)


@pytest.mark.parametrize("p4", [0.5, 0.1])
def test_lean_rollout_equals_single_steps(g2048, p4):
    """The headline kernel (no episode log, auto-reset, ring in one window; reward sums on and
    off) == single steps, from every clock phase mod 4 (its draws come one Philox block per
    4-step quad) and with a ring that wraps inside a launch, in both p(4) modes."""
    n, seed = 4096 + 64, 777
    e1 = g2048.VecEnv2048(n, seed=seed, device=DEV, p4=p4)
    e2 = g2048.VecEnv2048(n, seed=seed, device=DEV, p4=p4)
    r1, r2 = g2048.ReplayBuffer(10 * n, device=DEV), g2048.ReplayBuffer(10 * n, device=DEV)
    rs = torch.zeros(n, dtype=torch.int64, device=DEV)
    acc = torch.zeros(n, dtype=torch.int64, device=DEV)
    for j, k in enumerate((1, 6, 3, 9, 2, 17, 64, 5, 0, 11)):
        e1.rollout(k, replay=r1, reward_sum=rs if j % 2 else None)
        for _ in range(k):
            r, _, _ = e2.step(None, replay=r2)
            if j % 2:
                acc += r
        assert torch.equal(e1.board, e2.board) and torch.equal(e1.meta, e2.meta), k
        assert torch.equal(e1.clock, e2.clock) and torch.equal(e1.ep, e2.ep), k
    assert torch.equal(rs, acc)
    for name in ["s", "s2", "a", "r", "d", "count"]:
        assert torch.equal(getattr(r1, name), getattr(r2, name)), name
    assert int(e1.ep[:, 0].sum()) > 0


@pytest.mark.parametrize("p4", [0.5, 0.1])
def test_random_step_spawn_uniform(g2048, p4):
    """The random policy's spawn (ABI v3: the k-th empty cell in move-space line-major order) is
    uniform over the cells the slide left empty, for every move, and a 4 with p(4) (src/board.py:
    41-51, F3; parity unpinned by the reference's tests, pinned here statistically): 2^18 copies of
    a board that every move changes, one random step each (distinct board ids -> distinct draws);
    chi^2 of the landing cell per move over its 8 empty cells (7 dof, bound ~ p 1e-4)."""
    base = np.array([1, 0, 2, 0, 0, 3, 0, 4, 5, 0, 6, 0, 0, 7, 0, 8], np.uint8)
    n = 1 << 18
    env = g2048.VecEnv2048(n, seed=123, device=DEV, p4=p4)
    env.board.copy_(torch.from_numpy(np.tile(base, (n, 1))).to(DEV))
    env.meta.zero_()
    rb = g2048.ReplayBuffer(n, device=DEV)
    env.step(None, replay=rb)
    after, acts = _np(env.board), _np(rb.a)
    vals = []
    for mv in range(4):
        slid, _ = O.move(base, mv)
        empt = np.flatnonzero(slid == 0)
        rows = after[acts == mv]
        assert len(empt) == 8 and len(rows) > n // 5
        assert np.array_equal(np.where(slid != 0, rows, 0), np.tile(slid, (len(rows), 1)))
        new = (rows != 0) & (slid == 0)
        assert (new.sum(1) == 1).all()  # exactly one tile spawned, into an empty cell
        cnt = new[:, empt].sum(0).astype(np.float64)
        exp = len(rows) / 8
        assert ((cnt - exp) ** 2 / exp).sum() < 35, (mv, cnt)
        vals.append(rows[new])
    vals = np.concatenate(vals)
    frac4 = (vals == 2).mean()
    assert set(np.unique(vals)) <= {1, 2}
    assert abs(frac4 - p4) < 5 * np.sqrt(p4 * (1 - p4) / len(vals)), frac4


def test_max_boards_vs_oracle(g2048):
    """The ABI's largest env (include/g2048.h: G2048_MAX_BOARDS = 2^31 - 256 boards; 80 GB of
    board / meta / episode state plus 12 GB of step outputs in HBM): three single steps with
    every output and a 3-step rollout (the general kernel, no ring), against the oracle on three
    1 000-board slices -- the first
    boards, the middle and the last, whose global ids pass 2^30 and byte offsets 2^34.  Every
    index is 64-bit; this is where a 32-bit one would show.  (A 2^32 - 64 limit, the ABI's
    before this test, failed at the first launch: a grid of 2^32 work-items.)"""
    torch.cuda.empty_cache()
    n_all, seed = 2147483392, 0x5151
    env = g2048.VecEnv2048(n_all, seed=seed, device=DEV)
    reward = torch.empty(n_all, dtype=torch.int32, device=DEV)
    done = torch.empty(n_all, dtype=torch.uint8, device=DEV)
    legal = torch.empty(n_all, dtype=torch.uint8, device=DEV)
    n = 1000
    slices = (0, (1 << 30) - 500, n_all - n)
    refs = {i0: O.OracleEnv(n, seed=seed, board_offset=i0) for i0 in slices}
    for i0, ref in refs.items():
        assert np.array_equal(_np(env.board[i0:i0 + n]), ref.board), i0
    for step in range(3):
        env.step(None, reward=reward, done=done, legal=legal)
        torch.cuda.synchronize()
        for i0, ref in refs.items():
            o = ref.step(O.MODE_RANDOM)
            sl = slice(i0, i0 + n)
            assert np.array_equal(_np(reward[sl]), o["reward"]), (step, i0)
            assert np.array_equal(_np(done[sl]), o["done"]), (step, i0)
            assert np.array_equal(_np(legal[sl]), o["legal"]), (step, i0)
    env.rollout(3)
    torch.cuda.synchronize()
    for i0, ref in refs.items():
        for _ in range(3):
            ref.step(O.MODE_RANDOM)
        sl = slice(i0, i0 + n)
        assert np.array_equal(_np(env.board[sl]), ref.board), i0
        assert np.array_equal(_np(env.score_moves()[sl]).view(np.uint32), ref.meta), i0
        assert np.array_equal(_np(env.ep[sl]).view(np.uint32), ref.ep), i0
    clock = env.clock[-1:]
    assert int(clock) == 6
    env.check_errors()
    del env, reward, done, legal
    torch.cuda.empty_cache()
