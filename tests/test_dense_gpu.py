"""The reference dense Q-net's HIP forward (g2048_densenet_forward / _greedy, csrc/g2048_dense.hip):
Q against the torch model (src/configs/double_dqn_dense.py:7-15) in float32 and float64, the
greedy-branch rows bitwise the all-rows forward's, and the Trainer loop that uses it (captured
step + update, src/dqn_lib.py:167-244) bitwise the same with every board's Q computed."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    return g2048


def _boards(n, seed):
    g = torch.Generator().manual_seed(seed)
    b = torch.randint(0, 18, (n, 16), generator=g, dtype=torch.uint8)
    b[torch.rand((n, 16), generator=g) < 0.4] = 0
    return b.to(DEV)


@pytest.mark.parametrize("dtype,rtol,atol", [(torch.float32, 2e-5, 2e-5), (torch.float64, 1e-12, 1e-12)])
@pytest.mark.parametrize("n", [1, 777, 4096 + 5])
def test_dense_forward_matches_torch(G, dtype, rtol, atol, n):
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    m = det_init(make_net("dense", dtype, DEV), 0.4)
    rows = _boards(n, n)
    f = qnet.DenseForward(m)
    q = f(rows)
    with torch.no_grad():
        ref = m(rows.to(dtype))
    torch.testing.assert_close(q, ref, rtol=rtol, atol=atol * float(ref.abs().max()))
    # rows through an index list (the sampled-rows form)
    idx = torch.randperm(n, device=DEV)[: max(1, n // 3)]
    torch.testing.assert_close(f(rows, idx=idx), q[idx], rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("n,form", [(1, 0.0), (1000, 0.5), (20001, "tensor"), (65536 + 37, "schedule")])
def test_dense_forward_greedy_rows(G, dtype, n, form):
    """Q only for the boards whose next step is greedy, bitwise the all-rows forward's rows;
    explorers' rows untouched; stepping on it equals stepping on the full forward."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net
    from test_qnet_gpu import _greedy_mask

    ep0 = torch.randint(0, 8, (n,), generator=torch.Generator().manual_seed(n), dtype=torch.int32)
    envs = []
    for _ in range(2):
        e = G.VecEnv2048(n, device=DEV, seed=17 + n, board_offset=3 * n)
        e.rollout(19)
        e.ep[:, 0] = ep0.to(DEV)
        envs.append(e)
    if form == "schedule":
        kw = dict(eps_schedule=(6.0, 0.1))
        eps = np.maximum((6.0 - ep0.numpy().astype(np.float64)) / 6.0, 0.1)
    elif form == "tensor":
        kw = dict(epsilon=torch.tensor(0.3, dtype=torch.float64, device=DEV))
        eps = np.full(n, 0.3)
    else:
        kw = dict(epsilon=form)
        eps = np.full(n, float(form))
    m = det_init(make_net("dense", dtype, DEV), 0.7)
    f = qnet.DenseForward(m)
    full = f(envs[0].board)
    out = torch.full((n, 4), float("nan"), dtype=dtype, device=DEV)
    f.greedy(envs[0], out=out, **kw)
    g = _greedy_mask(envs[0], eps)
    if n > 100:
        assert 0 < int(g.sum()) < n
    assert torch.equal(out[g], full[g])
    assert bool(out[~g].isnan().all())
    eps_arg = kw.get("epsilon", 0.0)
    sched = kw.get("eps_schedule")
    a0, r0, d0 = envs[0].step_egreedy(out, eps_arg, eps_schedule=sched)
    a1, r1, d1 = envs[1].step_egreedy(full, eps_arg, eps_schedule=sched)
    assert torch.equal(a0, a1) and torch.equal(r0, r1) and torch.equal(d0, d1)
    assert torch.equal(envs[0].board, envs[1].board)


def test_dense_forward_rejects_other_nets(G):
    from g2048 import qnet
    from g2048.nets import make_net

    with pytest.raises(TypeError):
        qnet.DenseForward(make_net("dense64", torch.float32, DEV))


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_dense_trainer_graphed_greedy_equals_full_forward(G, dtype):
    """The reference dense net: the Trainer replays ONE captured graph per iteration (HIP
    greedy-branch forward + fused eps-greedy step + the fused update, g2048_densenet_update), and 25
    iterations are bitwise those of the same loop computing every board's Q (the boards start at
    mixed episode counts, so eps spans 1 .. min_epsilon)."""
    from g2048 import train
    from test_train_gpu import _fingerprint, _small

    outs = []
    for greedy in (True, False):
        tr = _small(train, "dense", min_fill=3 * 1024, target_sync_every=3, track_boards=0,
                    dtype=getattr(torch, dtype))
        assert tr.graph and tr.learner._dfwd is not None and tr.learner.kind == "dense"
        tr.greedy_forward = greedy
        grp = torch.arange(tr.env.n, device=DEV) % 5
        tr.env.ep[:, 0] = grp.to(torch.int32)
        for _ in range(25):
            tr.step()
        assert tr._loop_graph is not None and tr.learner.updates == 23
        outs.append(_fingerprint(tr))
    a, b = outs
    for k in a:
        if k in ("params", "target"):
            for x, y in zip(a[k], b[k]):
                assert torch.equal(x, y), k
        else:
            assert torch.equal(a[k], b[k]), k


def test_dense_trainer_graphed_equals_eager(G):
    """The captured iteration (step + update) against the eager loop (graph=False), same seeds:
    boards, ring, episode log bitwise; weights to fp32 roundoff of the two torch launches."""
    from g2048 import train
    from test_train_gpu import _fingerprint, _small

    outs = []
    for graph in (True, False):
        tr = _small(train, "dense", min_fill=3 * 1024, target_sync_every=3, track_boards=0,
                    loop_graph=graph)
        assert tr.graph == graph
        for _ in range(12):
            tr.step()
        outs.append(_fingerprint(tr))
    a, b = outs
    for k in ("board", "meta", "clock", "ep", "replay_s", "count", "log"):
        assert torch.equal(a[k], b[k]), k
    for x, y in zip(a["params"] + a["target"], b["params"] + b["target"]):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5)


def _dense_fixture_nets(g, dtype):
    from g2048.nets import det_init, make_net

    freq = float(g["init_freq"]) if "init_freq" in g else 1.3
    tph = float(g["tgt_phase"]) if "tgt_phase" in g else 0.2
    return (det_init(make_net("dense", dtype, DEV), 0.5, freq),
            det_init(make_net("dense", dtype, DEV), tph, freq))


@pytest.mark.parametrize("name", ["learner_dense", "learner_dense_b5000"])
def test_dense_ref_fused_matches_reference(G, golden_dir, name):
    """The fused float64 update of the reference dense net (g2048_densenet_update: six launches,
    DQNLearner(net="dense", dtype=float64)) against the reference train_step fixtures -- B = 512
    and BASELINE configs[0]'s B = 5000 (src/configs/double_dqn_dense.py:17): the loss within 1e-6
    absolute, y to 1e-12, the fixture's sampled gradient entries and their sum / sum of squares,
    and the sampled parameters after one Adam step (intended order) to 1e-10."""
    import os
    from g2048.learner import DQNLearner

    g = np.load(os.path.join(golden_dir, name + ".npz"))
    rb = G.ReplayBuffer(len(g["buf_a"]), device=DEV)
    rb.load(g["buf_s"], g["buf_a"], g["buf_r"], g["buf_s2"], g["buf_d"])
    idx = torch.from_numpy(g["idx"]).to(DEV)
    m, tg = _dense_fixture_nets(g, torch.float64)
    L = DQNLearner(rb, net="dense", dtype=torch.float64, batch_size=len(idx), lr=float(g["lr"]),
                   target_sync_every=0, model=m, sampler=lambda B, r: idx)
    assert L.fused and L.f64 and L.kind == "dense"
    L.target.load_state_dict(tg.state_dict())
    L.update()
    torch.cuda.synchronize()
    ref = float(g["loss_ref"])
    assert abs(float(L.last_loss) - ref) <= 1e-6 + 1e-13 * abs(ref), (float(L.last_loss), ref)
    assert torch.equal(L._idx, idx)
    np.testing.assert_allclose(L._y.cpu().numpy(), g["y"], rtol=1e-12, atol=1e-9)
    grad = L.grad_flat.cpu().numpy()
    sel = g["grad_sel"]
    gs = g["grads_sampled"]
    np.testing.assert_allclose(grad[sel], gs, rtol=1e-10, atol=1e-10 * max(1.0, float(np.abs(gs).max())))
    assert abs(grad.sum() - float(g["grad_sum"])) <= 1e-9 * max(1.0, abs(float(g["grad_sum"])))
    assert abs((grad ** 2).sum() - float(g["grad_sumsq"])) <= 1e-9 * float(g["grad_sumsq"])
    after = torch.cat([p.detach().reshape(-1) for p in L.model.parameters()]).cpu().numpy()
    np.testing.assert_allclose(after[sel], g["params_after_sampled"], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-9), (torch.float32, 2e-4)])
@pytest.mark.parametrize("double_dqn", [True, False])
@pytest.mark.parametrize("batch", [1, 33, 700, 5000, 8192, 20000, 65536])
def test_dense_ref_fused_equals_autograd(G, batch, double_dqn, dtype, tol):
    """Three fused updates of the reference dense net (Philox rows, Adam, target sync every 2)
    against torch autograd through dqn_lib.dqn_loss on the same rows and the same pre-update
    weights: loss and every parameter tensor's gradient to `tol` relative (float64 1e-9; float32
    2e-4 -- fp32 sums over B rows in another order); B = 1 and 33 are ragged single / double
    tiles (the weight-gradient splits then hold 0-16 rows), B = 700 leaves a ragged last tile,
    B = 65 536 is eight times the bench's batch."""
    import copy

    from g2048 import dqn_lib
    from g2048.learner import DQNLearner

    n = 4096
    env = G.VecEnv2048(n, seed=23, device=DEV)
    rb = G.ReplayBuffer(4 * n, device=DEV)
    env.rollout(4, replay=rb)
    L = DQNLearner(rb, net="dense", dtype=dtype, batch_size=batch, target_sync_every=2, seed=8,
                   use_double_dqn=double_dqn)
    assert L.fused and L.kind == "dense"
    for k in range(3):
        m0, t0 = copy.deepcopy(L.model), copy.deepcopy(L.target)
        L.update()
        torch.cuda.synchronize()
        rows = L._idx.clone()
        assert int(rows.min()) >= 0 and int(rows.max()) < 4 * n
        s, a, r, s2, d = dqn_lib.sample_experiences(batch, rb, DEV, None,
                                                    dqn_lib.extract_samples_dense, dtype=dtype,
                                                    idx=rows)
        loss, _, y = dqn_lib.dqn_loss(m0, t0, s, a, r, s2, d, L.gamma, double_dqn, None)
        loss.backward()
        assert abs(float(L.last_loss) - float(loss)) <= tol * abs(float(loss)), k
        torch.testing.assert_close(L._y, y, rtol=tol, atol=tol * float(y.abs().max()))
        off = 0
        for i, p in enumerate(m0.parameters()):
            gl, gr = L.grad_flat[off:off + p.numel()], p.grad.reshape(-1)
            assert float((gl - gr).norm()) <= tol * max(float(gr.norm()), 1e-30), (k, i)
            off += p.numel()
    assert int(L.step_dev) == 3


def test_dense_ref_fused_dp_split_equals_folded(G):
    """The data-parallel form (gradient only, then Adam64.step on the device counter) moves the
    online and target weights bitwise like the update with Adam folded into its reduction."""
    from g2048.learner import DQNLearner

    n = 2048
    env = G.VecEnv2048(n, seed=5, device=DEV)
    rb = G.ReplayBuffer(4 * n, device=DEV)
    env.rollout(4, replay=rb)
    a = DQNLearner(rb, net="dense", dtype=torch.float64, batch_size=1000, target_sync_every=2,
                   seed=2, graph=False)
    b = DQNLearner(rb, net="dense", dtype=torch.float64, batch_size=1000, target_sync_every=2,
                   seed=2, graph=False)
    b.model.load_state_dict(a.model.state_dict())
    b.target.load_state_dict(a.target.state_dict())
    b._upd.adam = None
    for _ in range(3):
        a.update()
        b._compute_grads()
        b._adam.step(b.grad_flat, b.step_dev)
        torch.cuda.synchronize()
        assert torch.equal(a.grad_flat, b.grad_flat)
        for p, q in zip(list(a.model.parameters()) + list(a.target.parameters()),
                        list(b.model.parameters()) + list(b.target.parameters())):
            assert torch.equal(p, q)
