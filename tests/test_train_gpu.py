"""GPU tests of the device-resident training loop (g2048.train / Trainer): bit-exact resume
from binary/checkpoint.pt, episode records and game snapshots in the reference's artefact
format, checked against the device state and the oracle's move rule."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    from g2048 import train
    return train


def _small(G, net="conv", **kw):
    args = dict(n_boards=1024, net=net, batch_size=256, replay_buffer_length=32 * 1024,
                min_fill=2048, target_sync_every=5, no_episodes_to_reach_epsilon=4.0,
                min_epsilon=0.05, seed=3, device=DEV, track_boards=2)
    args.update(kw)
    return G.build_trainer(**args)


def _fingerprint(tr):
    torch.cuda.synchronize()
    L = tr.learner
    return {"board": tr.env.board.cpu().clone(), "meta": tr.env.meta.cpu().clone(),
            "clock": tr.env.clock.cpu().clone(),
            "ep": tr.env.ep.cpu().clone(), "replay_s": tr.replay.s.cpu().clone(),
            "count": tr.replay.count.cpu().clone(), "log": tr.log.raw.cpu().clone(),
            "params": [p.detach().cpu().clone() for p in L.model.parameters()],
            "target": [p.detach().cpu().clone() for p in L.target.parameters()],
            "loss": L.last_loss.cpu().clone()}


@pytest.mark.parametrize("net", ["conv", "dense"])
def test_resume_is_bit_exact(G, net, tmp_path):
    a = _small(G, net)
    for _ in range(12):
        a.step()
    state = a.state_dict()
    from g2048.experiment import Experiment
    exp = Experiment("ck", root=str(tmp_path))
    exp.save_checkpoint(state)
    for _ in range(9):
        a.step()
    want = _fingerprint(a)

    b = _small(G, net)
    b.load_state_dict(exp.load_checkpoint())
    for _ in range(9):
        b.step()
    got = _fingerprint(b)
    for k in ("board", "meta", "clock", "ep", "replay_s", "count", "log", "loss"):
        assert torch.equal(got[k], want[k]), k
    for x, y in zip(got["params"] + got["target"], want["params"] + want["target"]):
        assert torch.equal(x, y)
    assert b.learner.updates == a.learner.updates and b.steps == a.steps


def test_resume_round4_dense_checkpoint(G):
    """the reference dense net trained on the torch path up to round 4; its checkpoints
    (learner fused=False, kind '', torch Adam state per parameter, no sampler seed) resume on the
    fused dense-ref update: same weights, Adam moments and step, and -- the sampler seed being the
    learner's own -- the same next updates, bit for bit."""
    a = _small(G, "dense")
    assert a.learner.fused and a.learner.kind == "dense"
    for _ in range(12):
        a.step()
    st = a.state_dict()
    L = dict(st["learner"])
    flat_m, flat_v = L.pop("adam_exp_avg"), L.pop("adam_exp_avg_sq")
    step = L.pop("step_dev")
    L.pop("sample_seed")
    per, off = [], 0
    for p in a.learner.bucket.params:  # round 4: torch.optim.Adam(capturable=True) state
        n = p.numel()
        per.append({"step": step.to(torch.float32).reshape(()),
                    "exp_avg": flat_m[off:off + n].view_as(p).clone(),
                    "exp_avg_sq": flat_v[off:off + n].view_as(p).clone()})
        off += n
    L.update(fused=False, kind="", adam=per)
    old = dict(st, learner=L)
    for _ in range(5):
        a.step()
    want = _fingerprint(a)
    b = _small(G, "dense")
    b.load_state_dict(old)
    assert torch.equal(b.learner._adam.exp_avg.cpu(), flat_m)
    assert torch.equal(b.learner.step_dev.cpu(), step)
    for _ in range(5):
        b.step()
    got = _fingerprint(b)
    for k in ("board", "replay_s", "loss"):
        assert torch.equal(got[k], want[k]), k
    for x, y in zip(got["params"] + got["target"], want["params"] + want["target"]):
        assert torch.equal(x, y)
    c = _small(G, "conv")  # another net's torch-path checkpoint is still refused
    with pytest.raises(ValueError, match="another net"):
        c.load_state_dict(dict(c.state_dict(), learner=dict(c.state_dict()["learner"],
                                                            fused=False, kind="")))


def test_resume_version3_trainer_state(G):
    """A trainer state of rounds 3-5 (version 3: env meta [N, 2] {score, moves}, ABI v4) resumes
    on the ABI-v5 env (meta rows {score, episode start}): its pairs become rows with start =
    clock - moves, and the run continues bit for bit -- boards, score / moves, episode counters,
    the ring, the episode log and the learner."""
    a = _small(G, "conv")
    for _ in range(12):
        a.step()
    st = a.state_dict()
    assert st["trainer_state_version"] == 4 and tuple(st["env"]["meta"].shape) == (2, a.env.n)
    old = dict(st, trainer_state_version=3,
               env=dict(st["env"], meta=a.env.score_moves().cpu().clone()))
    for _ in range(9):
        a.step()
    want = _fingerprint(a)
    b = _small(G, "conv")
    b.load_state_dict(old)
    assert torch.equal(b.env.meta.cpu(), st["env"]["meta"])
    for _ in range(9):
        b.step()
    got = _fingerprint(b)
    for k in ("board", "meta", "clock", "ep", "replay_s", "count", "log", "loss"):
        assert torch.equal(got[k], want[k]), k
    assert torch.equal(b.env.score_moves(), a.env.score_moves())


def test_load_rejects_mismatch(G):
    a = _small(G, "conv")
    st = a.state_dict()
    b = _small(G, "conv", batch_size=128)
    with pytest.raises(ValueError):
        b.load_state_dict(st)
    c = _small(G, "conv", seed=4)
    with pytest.raises(ValueError):
        c.load_state_dict(st)
    old = dict(st)
    old.pop("trainer_state_version")  # a round-2 trainer state (no key, env meta [N, 2] + clock)
    with pytest.raises(ValueError, match="trainer state version 2 .env meta \\[N, 2\\]"):
        a.load_state_dict(old)
    old["env"] = dict(st["env"], meta=torch.zeros((a.env.n, 4), dtype=torch.int32))
    with pytest.raises(ValueError, match="trainer state version 1 .env meta \\[N, 4\\]"):
        a.load_state_dict(old)  # a round-1 trainer state (env meta [N, 4], no clock)


def _move_ok(s, a, s2, r, letters=("u", "d", "l", "r")):
    """s2 follows s under action a: the oracle slide (+ one spawned 2/4) or no change."""
    e = np.where(s > 0, np.log2(np.maximum(s, 1)), 0).astype(np.uint8).reshape(16)
    e2 = np.where(s2 > 0, np.log2(np.maximum(s2, 1)), 0).astype(np.uint8).reshape(16)
    slid, gain = O.move(e, letters.index(a))
    if np.array_equal(slid, e):
        return np.array_equal(e2, e) and r == 0
    diff = np.nonzero(slid != e2)[0]
    return (len(diff) == 1 and slid[diff[0]] == 0 and e2[diff[0]] in (1, 2) and r == gain)


def test_training_loop_artefacts(G, tmp_path):
    from g2048.experiment import Experiment, load_pickle
    tr = _small(G, "conv", n_boards=512)
    exp = Experiment("run", root=str(tmp_path))
    exp.add_hyperparameter(G.hyperparameters(tr, 600, 50))
    G.training_loop(tr, no_episodes=600, experiment=exp, snapshot_game_every_n_episodes=50,
                    save_every_episodes=200, check_every=16, max_steps=4000)
    eps = load_pickle(exp.folder, "episodes.p")
    assert len(eps) >= 600 and [e["number"] for e in eps] == list(range(len(eps)))
    # per board, the logged episodes agree with the env's own counters
    ep = tr.env.ep.cpu().numpy()
    per_board = {}
    for e in eps:
        per_board.setdefault(e["board"], []).append(e)
    for b, lst in per_board.items():
        assert [x["board_episode"] for x in lst] == list(range(len(lst)))
        assert len(lst) == ep[b, 0]
        last = lst[-1]
        assert int(last["merge_score"]) == ep[b, 1] and last["number_moves"] == ep[b, 2]
        assert int(last["max_tile"]) == 1 << ep[b, 3]
    for e in eps:
        assert e["reward"] == float(e["merge_score"]) / e["number_moves"]
        assert e["epsilon"] == max((4.0 - e["board_episode"]) / 4.0, 0.05)
    # snapshots: complete games of tracked boards, consistent move by move
    hist_dir = os.path.join(exp.folder, "binary", "board_histories")
    files = sorted(os.listdir(hist_dir))
    assert files
    by_num = {e["number"]: e for e in eps}
    for fn in files:
        num = int(fn[len("episode_"):-2])
        hist = load_pickle(exp.folder, os.path.join("board_histories", fn))
        e = by_num[num]
        assert e["board"] in (0, 1) and len(hist) == e["number_moves"]
        assert int(hist[-1][0].max()) == int(e["max_tile"])
        assert sum(h[2] for h in hist) == int(e["merge_score"])
        for k in range(len(hist) - 1):
            assert _move_ok(hist[k][0], hist[k][1], hist[k + 1][0], hist[k][2]), (fn, k)
    # resume from the folder continues from the checkpoint
    exp2, tr2 = G.resume("run", root=str(tmp_path), net="conv", batch_size=256,
                         min_fill=2048, target_sync_every=5, no_episodes_to_reach_epsilon=4.0,
                         min_epsilon=0.05, device=DEV, track_boards=2)
    assert tr2.steps == tr.steps and len(exp2.episodes) == len(eps)
    assert torch.equal(tr2.env.board.cpu(), tr.env.board.cpu())


@pytest.mark.parametrize("net", ["conv", "dense64"])
def test_graphed_loop_equals_eager(G, net):
    """Trainer(graph=True) replays one captured hipGraph per iteration (step + updates); the
    trajectory must be bitwise the eager one: boards, episode counters, ring, episode log,
    tracked-board histories, online and target weights, loss.  Covers the steps before
    min_fill (no update), 2 updates per step and target syncs between replays."""
    outs = []
    for graph in (True, False):
        tr = _small(G, net, min_fill=3 * 1024, target_sync_every=3, track_boards=3,
                    updates_per_step=2, loop_graph=graph)
        assert tr.graph is graph
        for _ in range(11):
            tr.step()
        f = _fingerprint(tr)
        f["h_s"], f["h_a"] = tr.h_s.cpu().clone(), tr.h_a.cpu().clone()
        outs.append((f, tr.learner.updates))
    (a, ua), (b, ub) = outs
    assert ua == ub == 2 * 9
    for k in a:
        if k in ("params", "target"):
            for x, y in zip(a[k], b[k]):
                assert torch.equal(x, y), k
        else:
            assert torch.equal(a[k], b[k]), k


def test_greedy_forward_loop_equals_full_forward(G):
    """The fused conv Trainer evaluates the net only for the boards whose step takes the greedy
    branch (qnet.forward_greedy); with every other board's Q computed as well (a full forward
    per step) the trajectory is bitwise the same.  Boards start at mixed episode counts, so
    eps spans 1 .. min_epsilon from the first step."""
    outs = []
    for greedy in (True, False):
        tr = _small(G, "conv", min_fill=3 * 1024, target_sync_every=3, track_boards=0)
        assert tr._q is not None
        if not greedy:
            tr._q = None
        grp = torch.arange(tr.env.n, device=DEV) % 5
        tr.env.ep[:, 0] = grp.to(torch.int32)
        for _ in range(25):
            tr.step()
        outs.append(_fingerprint(tr))
    a, b = outs
    for k in a:
        if k in ("params", "target"):
            for x, y in zip(a[k], b[k]):
                assert torch.equal(x, y), k
        else:
            assert torch.equal(a[k], b[k]), k
