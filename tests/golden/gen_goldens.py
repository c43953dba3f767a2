"""Generate the golden fixtures under tests/golden/ by running the Python reference.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  Nothing here travels to the GPU box except the .npz / .json
outputs it writes (data: inputs and the reference's outputs).

    PYTHONPATH=/root/reference/src PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_goldens.py

Fixtures (all boards are stored as log2 exponents, 0 = empty, row-major):
  ref_tests.json       the reference's own known answers (tests/test_game_board.py:7-23,
                       :33-52) re-evaluated through board.py
  row_lut.npz          all 16**4 rows (exponents 0..15), itertools.product order ->
                       board._apply_action_to_vector result + merge-score gain
                       (src/board.py:92-126, score at :114)
  trajectories.npz     random-policy episodes through dqn_lib.play_one_step(eps=1)
                       (src/dqn_lib.py:91-107) with every landed spawn recorded
                       (src/board.py:41-51) so the env can be replayed with injected spawns
  egreedy.npz          dqn_lib.epsilon_greedy_policy(eps=0) on fixed Q rows / legal masks
                       (src/dqn_lib.py:16-30, operator-precedence formula at :25-27)
  egreedy_nonfinite.npz  the same policy on Q rows holding NaN / +-inf / f32-overflowing values
                       (torch's NaN-propagating min/max and first-NaN argmax) + torch.max(Q)
  learner_<net>.npz    dqn_lib.train_step on a seeded buffer, B=512, deterministic weights
                       (src/dqn_lib.py:119-164) + restated intermediates, correct-order
                       grads and one Adam step (lr 1e-2)
  learner_{conv,dense64}_vanilla.npz  the same with use_double_dqn=False (src/dqn_lib.py:133-144)
  learner_dense_b5000.npz  dense-ref (double_dqn_dense.py) at B=5000, BASELINE configs[0]'s batch
"""
from __future__ import annotations

import copy
import hashlib
import itertools
import json
import math
import os
import random
import sys
from collections import deque

import numpy as np
import torch

REF_SRC = "/root/reference/src"
if REF_SRC not in sys.path:
    sys.path.insert(0, REF_SRC)

import board as ref_board  # noqa: E402
import dqn_lib  # noqa: E402
from board import Board2048  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def exps_of(state: np.ndarray) -> np.ndarray:
    s = np.asarray(state, dtype=np.int64).reshape(-1)
    out = np.zeros(16, dtype=np.uint8)
    nz = s != 0
    out[nz] = np.log2(s[nz]).astype(np.uint8)
    assert np.array_equal(np.where(nz, 1 << out.astype(np.int64), 0), s)
    return out


def values_of(exps) -> np.ndarray:
    e = np.asarray(exps, dtype=np.int64)
    return np.where(e == 0, 0, np.left_shift(1, e))


# ---------------------------------------------------------------- ref_tests.json
def gen_ref_tests():
    # Data transcribed from the reference's own tests (tests/test_game_board.py:7-23, :33-52).
    rows = [
        ([0, 0, 0, 0], [0, 0, 0, 0]), ([0, 0, 0, 2], [2, 0, 0, 0]), ([0, 0, 2, 2], [4, 0, 0, 0]),
        ([2, 0, 0, 0], [2, 0, 0, 0]), ([2, 0, 2, 0], [4, 0, 0, 0]), ([2, 2, 2, 2], [4, 4, 0, 0]),
        ([2, 2, 4, 4], [4, 8, 0, 0]), ([2, 2, 0, 0], [4, 0, 0, 0]), ([2, 0, 0, 2], [4, 0, 0, 0]),
        ([0, 0, 2, 2], [4, 0, 0, 0]), ([2, 4, 2, 4], [2, 4, 2, 4]), ([2, 2, 4, 2], [4, 4, 2, 0]),
        ([2, 4, 4, 2], [2, 8, 2, 0]), ([2, 4, 4, 4], [2, 8, 4, 0]), ([4, 8, 16, 32], [4, 8, 16, 32]),
    ]
    boards = [
        ([[2, 4, 8, 0], [0, 0, 0, 0], [2, 4, 16, 32], [0, 0, 0, 0]], ["up", "down", "right"]),
        ([[2, 4, 2, 4], [2, 4, 2, 4], [2, 4, 2, 4], [2, 4, 2, 4]], ["up", "down"]),
        ([[2, 4, 2, 4], [4, 2, 4, 2], [2, 4, 2, 4], [4, 2, 4, 2]], []),
    ]
    out = {"rows": [], "legal_boards": []}
    b = Board2048(populate_empty_cells=False)
    for inp, expected in rows:
        b._mergescore = 0
        res = b._apply_action_to_vector(np.array(inp))
        assert list(res) == expected
        out["rows"].append({"in": inp, "out": [int(x) for x in res], "score": int(b._mergescore)})
    for state, moves in boards:
        b = Board2048(populate_empty_cells=False)
        b.state = np.array(state)
        got = sorted(b.available_moves().keys())
        assert got == sorted(moves)
        mask = [int(m in got) for m in ["up", "down", "left", "right"]]
        out["legal_boards"].append({"state": state, "moves": sorted(moves), "mask_udlr": mask})
    with open(os.path.join(OUT, "ref_tests.json"), "w") as f:
        json.dump(out, f, indent=1)


# ---------------------------------------------------------------- row_lut.npz
def gen_row_lut():
    b = Board2048(populate_empty_cells=False)
    res = np.zeros((65536, 4), dtype=np.uint8)
    score = np.zeros(65536, dtype=np.uint32)
    for i, row in enumerate(itertools.product(range(16), repeat=4)):
        b._mergescore = 0
        r = b._apply_action_to_vector(values_of(row))
        res[i] = exps_of(np.concatenate([r, np.zeros(12, dtype=np.int64)]))[:4]
        score[i] = int(b._mergescore)
    stream = b"".join(bytes(res[i]) + int(score[i]).to_bytes(4, "little") for i in range(65536))
    digest = hashlib.sha256(stream).hexdigest()
    np.savez_compressed(os.path.join(OUT, "row_lut.npz"), result=res, score=score,
                        sha256=np.array(digest))
    print("row LUT sha256", digest)


# ---------------------------------------------------------------- trajectories.npz
class SpawnLog:
    """Wraps Board2048._populate_empty_cell (src/board.py:41-51) to RECORD the cell and
    value each call writes; it calls the original, so the RNG stream is untouched."""

    def __init__(self):
        self.log = {}
        self.orig = Board2048._populate_empty_cell

    def __enter__(self):
        log, orig = self.log, self.orig

        def wrapped(board_self):
            before = board_self.state.copy()
            orig(board_self)
            diff = np.argwhere(before != board_self.state)
            assert len(diff) == 1
            r, c = diff[0]
            log.setdefault(id(board_self), []).append(
                (before.copy(), board_self.state.copy(), int(r * 4 + c), int(board_self.state[r, c])))
            return board_self

        Board2048._populate_empty_cell = wrapped
        return self

    def __exit__(self, *a):
        Board2048._populate_empty_cell = self.orig


def gen_trajectories(n_episodes=24, seed0=2048):
    cols = {k: [] for k in ["s", "a", "legal", "s_slide", "spawn_idx", "spawn_exp", "s2",
                             "reward", "done", "episode", "score_before", "score_after"]}
    init = []
    with SpawnLog() as sl:
        for ep in range(n_episodes):
            random.seed(seed0 + ep)
            np.random.seed(seed0 + ep)
            board = Board2048()
            ents = sl.log[id(board)]
            assert len(ents) == 2
            init.append([ents[0][2], int(np.log2(ents[0][3])), ents[1][2], int(np.log2(ents[1][3]))])
            buf = deque(maxlen=10)
            done = False
            while not done:
                legal = board.available_moves_as_torch_unit_vector()
                legal_bits = sum(int(legal[i].item() != 0) << i for i in range(4))
                sl.log.clear()
                nb, action, reward, done, _ = dqn_lib.play_one_step(
                    board, 1.0, None, buf, "cpu",
                    reward_function=dqn_lib.reward_func_merge_score,
                    board_to_tensor_function=dqn_lib.board_as_4d_tensor)
                done = bool(int(done))
                ents = sl.log.get(id(nb), [])
                changed = not np.array_equal(nb.state, board.state)
                if changed:
                    before, after, idx, val = ents[-1]
                    assert np.array_equal(after, nb.state)
                    s_slide, sidx, sexp = exps_of(before), idx, int(np.log2(val))
                else:
                    s_slide, sidx, sexp = exps_of(board.state), -1, 0
                cols["s"].append(exps_of(board.state))
                cols["a"].append(int(action))
                cols["legal"].append(legal_bits)
                cols["s_slide"].append(s_slide)
                cols["spawn_idx"].append(sidx)
                cols["spawn_exp"].append(sexp)
                cols["s2"].append(exps_of(nb.state))
                cols["reward"].append(int(reward))
                cols["done"].append(int(done))
                cols["episode"].append(ep)
                cols["score_before"].append(int(board.merge_score()))
                cols["score_after"].append(int(nb.merge_score()))
                board = nb
    dt = {"s": np.uint8, "a": np.uint8, "legal": np.uint8, "s_slide": np.uint8,
          "spawn_idx": np.int8, "spawn_exp": np.uint8, "s2": np.uint8, "reward": np.int32,
          "done": np.uint8, "episode": np.int32, "score_before": np.int64, "score_after": np.int64}
    arrs = {k: np.array(v, dtype=dt[k]) for k, v in cols.items()}
    arrs["init_spawns"] = np.array(init, dtype=np.int16)  # [E, 4] = idx0, exp0, idx1, exp1
    np.savez_compressed(os.path.join(OUT, "trajectories.npz"), **arrs)
    print("trajectories", len(arrs["a"]), "steps,", int(arrs["done"].sum()), "terminal,",
          int((arrs["spawn_idx"] < 0).sum()), "no-op")


# ---------------------------------------------------------------- egreedy.npz
class _StubBoard:
    def __init__(self, mask):
        self.mask = mask

    def available_moves_as_torch_unit_vector(self, device=None):
        return torch.tensor([float((self.mask >> i) & 1) for i in range(4)], dtype=torch.float32)


def gen_egreedy(n=4000, seed=7):
    rng = np.random.default_rng(seed)
    q = rng.normal(size=(n, 4)) * rng.choice([0.01, 1.0, 30.0, 1e3], size=(n, 1))
    q[: n // 8] = -np.abs(q[: n // 8])                   # all-negative rows (F5)
    q[n // 8: n // 4] = np.round(q[n // 8: n // 4])      # ties
    q[n // 4: n // 4 + 64] = 0.0
    mask = rng.integers(0, 16, size=n).astype(np.uint8)
    mask[:32] = 0
    action = np.zeros(n, dtype=np.uint8)
    done = np.zeros(n, dtype=np.uint8)
    for i in range(n):
        qt = torch.tensor(q[i], dtype=torch.float64)
        a, d, _ = dqn_lib.epsilon_greedy_policy(
            _StubBoard(int(mask[i])), 0.0, lambda x, qt=qt: qt, "cpu",
            board_to_tensor_function=lambda b, dev: None)
        action[i] = a
        done[i] = int(d)
    # the same rows evaluated in float32 (the fast mode computes Q in fp32)
    action32 = np.zeros(n, dtype=np.uint8)
    for i in range(n):
        qt = torch.tensor(q[i], dtype=torch.float32)
        a, _, _ = dqn_lib.epsilon_greedy_policy(
            _StubBoard(int(mask[i])), 0.0, lambda x, qt=qt: qt, "cpu",
            board_to_tensor_function=lambda b, dev: None)
        action32[i] = a
    np.savez_compressed(os.path.join(OUT, "egreedy.npz"), q=q, mask=mask, action=action,
                        action_f32=action32, done=done)


def gen_egreedy_nonfinite(n=3000, seed=11):
    """Rows with NaN, +inf, -inf and values whose min*max overflows float32 (finite in float64):
    the reference's epsilon_greedy_policy (src/dqn_lib.py:24-30) in f64 and f32, with the
    torch.max(Q) it returns (the Q-sum of the episode log)."""
    rng = np.random.default_rng(seed)
    pool = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1.0, -2.0, 0.5, 3.0, 1e30, -1e30, 7e-39],
                    dtype=np.float64)
    q = rng.normal(size=(n, 4))
    pick = rng.random(size=(n, 4)) < 0.45
    q[pick] = pool[rng.integers(0, len(pool), size=int(pick.sum()))]
    # every row has at least one non-finite or overflowing entry
    first = rng.integers(0, 4, size=n)
    q[np.arange(n), first] = pool[rng.integers(0, 3, size=n)]
    q[n - 16:] = np.nan                                   # all-NaN rows
    mask = rng.integers(0, 16, size=n).astype(np.uint8)
    mask[n - 16:] = np.arange(16)
    out = {"q": q, "mask": mask}
    for dt, suf in [(torch.float64, ""), (torch.float32, "_f32")]:
        action = np.zeros(n, dtype=np.uint8)
        qmax = np.zeros(n, dtype=np.float64)
        for i in range(n):
            qt = torch.tensor(q[i], dtype=dt)
            a, d, mq = dqn_lib.epsilon_greedy_policy(
                _StubBoard(int(mask[i])), 0.0, lambda x, qt=qt: qt, "cpu",
                board_to_tensor_function=lambda b, dev: None)
            action[i] = a
            qmax[i] = float(mq)
        out["action" + suf] = action
        out["qmax" + suf] = qmax
    out["done"] = (mask == 0).astype(np.uint8)
    np.savez_compressed(os.path.join(OUT, "egreedy_nonfinite.npz"), **out)
    print("egreedy_nonfinite", n, "rows;", int(np.isnan(q).any(axis=1).sum()), "with NaN")


# ---------------------------------------------------------------- learner_<net>.npz
def det_init(model, phase: float, freq: float = 1.3):
    """Deterministic weights: p.flat[k] = sin(freq k + phase) / sqrt(fan_in)."""
    with torch.no_grad():
        for p in model.parameters():
            k = torch.arange(p.numel(), dtype=torch.float64)
            fan_in = int(np.prod(p.shape[1:])) if p.dim() > 1 else 4
            p.copy_((torch.sin(freq * k + phase) / math.sqrt(fan_in)).reshape(p.shape).to(p.dtype))


def make_net(kind):
    nn = torch.nn
    if kind == "conv":
        import configs.double_dqn_conv as cfg  # src/configs/double_dqn_conv.py:19-28
        return copy.deepcopy(cfg.model), dqn_lib.board_as_4d_tensor, dqn_lib.extract_samples_conv
    if kind == "dense":
        import configs.double_dqn_dense as cfg  # src/configs/double_dqn_dense.py:7-15
        return copy.deepcopy(cfg.model), dqn_lib.board_as_flattened_tensor, dqn_lib.extract_samples_dense
    if kind == "dense64":  # BASELINE.json configs[2]: 16 -> 64 -> 4
        m = nn.Sequential(nn.Linear(16, 64), nn.ReLU(), nn.Linear(64, 4)).double()
        return m, dqn_lib.board_as_flattened_tensor, dqn_lib.extract_samples_dense
    raise ValueError(kind)


def build_buffer(n_trans=2000, seed=99):
    random.seed(seed)
    np.random.seed(seed)
    buf = deque(maxlen=n_trans)
    board = Board2048()
    while len(buf) < n_trans:
        nb, _, _, done, _ = dqn_lib.play_one_step(board, 1.0, None, buf, "cpu")
        board = Board2048() if int(done) else nb
    s = np.stack([exps_of(t[0].state) for t in buf])
    a = np.array([int(t[1]) for t in buf], dtype=np.int64)
    r = np.array([int(t[2]) for t in buf], dtype=np.int64)
    s2 = np.stack([exps_of(t[3].state) for t in buf])
    d = np.array([int(t[4]) for t in buf], dtype=np.int64)
    return buf, dict(buf_s=s, buf_a=a, buf_r=r, buf_s2=s2, buf_d=d)


def gen_learner(kind, buf, bufarrs, B=512, gamma=0.8, lr=1e-2, seed=1234, use_double=True,
                name=None, tgt_phase=0.2, freq=1.3):
    """One reference train_step (src/dqn_lib.py:119-164) on a seeded minibatch -> learner_<name>.npz.
    use_double=False takes the vanilla branch (:133-144): y = r + (1-d)*gamma*max_a Q_tgt(s')."""
    name = name or kind
    model, to_tensor, extract = make_net(kind)
    target = copy.deepcopy(model)
    det_init(model, 0.5, freq)
    det_init(target, tgt_phase, freq)
    init_params = [p.detach().clone() for p in model.parameters()]
    loss_fn = torch.nn.MSELoss(reduction="sum")
    opt = torch.optim.Adam(model.parameters(), lr=lr)

    np.random.seed(seed)
    idx = np.random.randint(len(buf), size=B)  # src/dqn_lib.py:68 (re-drawn below)
    np.random.seed(seed)
    loss_ref = dqn_lib.train_step(B, gamma, model, target, buf, loss_fn, opt, "cpu", use_double,
                                  to_tensor, extract)
    # F1: the reference's zero_grad-before-step leaves params untouched
    compat_unchanged = all(torch.equal(p, q) for p, q in zip(model.parameters(), init_params))
    assert compat_unchanged

    # restated intermediates on the same minibatch (no-grad target; F10)
    s = torch.from_numpy(bufarrs["buf_s"][idx].astype(np.float64))
    s2 = torch.from_numpy(bufarrs["buf_s2"][idx].astype(np.float64))
    if kind == "conv":
        s, s2 = s.reshape(B, 1, 4, 4), s2.reshape(B, 1, 4, 4)
    a = torch.from_numpy(bufarrs["buf_a"][idx])
    r = torch.from_numpy(bufarrs["buf_r"][idx])
    d = torch.from_numpy(bufarrs["buf_d"][idx])
    with torch.no_grad():
        q_on_s2 = model(s2)
        a_star = torch.argmax(q_on_s2, dim=1)
        q_tgt_s2 = target(s2)
        if use_double:
            y = (r + (1 - d) * gamma * q_tgt_s2.gather(1, a_star[:, None])[:, 0]).double()
        else:
            y = r + ((1 - d) * gamma * torch.max(q_tgt_s2, 1).values)
    q_on_s = model(s)
    q = q_on_s.gather(1, a[:, None])[:, 0]
    loss = ((q - y) ** 2).sum()
    assert float(loss) == float(loss_ref), (float(loss), float(loss_ref))
    # intended order: zero_grad -> backward -> step
    opt2 = torch.optim.Adam(model.parameters(), lr=lr)
    opt2.zero_grad()
    loss.backward()
    grads = [p.grad.detach().clone() for p in model.parameters()]
    opt2.step()
    after = [p.detach().clone() for p in model.parameters()]

    flat = lambda ts: torch.cat([t.reshape(-1) for t in ts]).numpy()
    out = dict(idx=idx.astype(np.int64), gamma=np.float64(gamma), lr=np.float64(lr),
               loss_ref=np.float64(float(loss_ref)), loss=np.float64(float(loss)),
               q_on_s=q_on_s.detach().numpy(), q_on_s2=q_on_s2.numpy(), q_tgt_s2=q_tgt_s2.numpy(),
               a_star=a_star.numpy(), y=y.numpy(), q=q.detach().numpy(),
               n_params=np.int64(sum(p.numel() for p in model.parameters())),
               param_shapes=np.array(json.dumps([list(p.shape) for p in model.parameters()])))
    if not use_double:  # (the keys are absent from the Double-DQN fixtures, which predate them)
        out["use_double_dqn"] = np.bool_(False)
        out["tgt_phase"] = np.float64(tgt_phase)
        out["init_freq"] = np.float64(freq)
    g, pa = flat(grads), flat(after)
    if g.size <= 50000:
        out.update(grads=g, params_after=pa)
    else:  # dense-ref (403 716 params): strided sample + digests keep the fixture small
        sel = np.arange(0, g.size, 97)
        out.update(grad_sel=sel, grads_sampled=g[sel], params_after_sampled=pa[sel],
                   grad_sum=np.float64(g.sum()), grad_sumsq=np.float64((g * g).sum()),
                   params_after_sum=np.float64(pa.sum()))
    out.update(bufarrs)
    np.savez_compressed(os.path.join(OUT, f"learner_{name}.npz"), **out)
    print(f"learner {name}: loss {float(loss_ref):.6f}")


if __name__ == "__main__":
    torch.set_num_threads(8)
    gen_ref_tests()
    gen_row_lut()
    gen_trajectories()
    gen_egreedy()
    gen_egreedy_nonfinite()
    buf, arrs = build_buffer()
    for k in ["conv", "dense", "dense64"]:
        gen_learner(k, buf, arrs)
    # round 3: the vanilla-DQN branch (src/dqn_lib.py:133-144) and BASELINE configs[0]'s batch
    # (double_dqn_dense.py:17, batch_size=5000; rows drawn with replacement from the 2000)
    # (weights at another frequency / target phase, so that max_a Q_tgt(s') differs from
    # Q_tgt(s', argmax Q_on(s')) on most rows: with the Double-DQN fixtures' weights the two nets'
    # argmax agree on every row, and a vanilla fixture would not tell the branches apart)
    gen_learner("conv", buf, arrs, use_double=False, name="conv_vanilla", tgt_phase=2.9, freq=3.7)
    gen_learner("dense64", buf, arrs, use_double=False, name="dense64_vanilla", tgt_phase=2.9,
                freq=3.7)
    gen_learner("dense", buf, arrs, B=5000, name="dense_b5000")
