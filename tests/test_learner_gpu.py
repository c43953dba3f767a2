"""Learner on the GPU: HIP replay gather+encode -> torch-ROCm Double-DQN, against the reference's
train_step fixtures (1e-6 absolute on loss / Q-values, float64)."""
import os

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


def fixture(golden_dir, net):
    return np.load(os.path.join(golden_dir, f"learner_{net}.npz"))


def fixture_nets(g, net, dtype=torch.float64):
    """Online / target weights of a fixture (tests/golden/gen_goldens.py det_init)."""
    from g2048.nets import det_init, make_net

    freq = float(g["init_freq"]) if "init_freq" in g else 1.3
    tph = float(g["tgt_phase"]) if "tgt_phase" in g else 0.2
    return (det_init(make_net(net, dtype, DEV), 0.5, freq),
            det_init(make_net(net, dtype, DEV), tph, freq))


def loaded_replay(G, g):
    rb = G.ReplayBuffer(len(g["buf_a"]), device=DEV)
    rb.load(g["buf_s"], g["buf_a"], g["buf_r"], g["buf_s2"], g["buf_d"])
    return rb


@pytest.mark.parametrize("net", ["conv", "dense", "dense64"])
def test_train_step_matches_reference(G, golden_dir, net):
    from g2048 import dqn_lib
    from g2048.nets import det_init, make_net

    g = fixture(golden_dir, net)
    rb = loaded_replay(G, g)
    m = det_init(make_net(net, torch.float64, DEV), 0.5)
    tg = det_init(make_net(net, torch.float64, DEV), 0.2)
    idx = torch.from_numpy(g["idx"]).to(DEV)
    ext = dqn_lib.extract_samples_conv if net == "conv" else dqn_lib.extract_samples_dense
    s, a, r, s2, d = dqn_lib.sample_experiences(len(idx), rb, DEV, None, ext, idx=idx)
    loss, q, y = dqn_lib.dqn_loss(m, tg, s, a, r, s2, d, float(g["gamma"]))
    ref = float(g["loss_ref"])
    assert abs(float(loss.detach()) - ref) <= 1e-6 + 1e-13 * abs(ref), (float(loss.detach()), ref)
    np.testing.assert_allclose(q.detach().cpu().numpy(), g["q"], rtol=1e-12, atol=1e-6)
    np.testing.assert_allclose(y.cpu().numpy(), g["y"], rtol=1e-12, atol=1e-6)
    with torch.no_grad():
        np.testing.assert_allclose(m(s).cpu().numpy(), g["q_on_s"], rtol=1e-12, atol=1e-6)
        np.testing.assert_allclose(tg(s2).cpu().numpy(), g["q_tgt_s2"], rtol=1e-12, atol=1e-6)

    # full train_step (intended order) -> params after one Adam step
    opt = torch.optim.Adam(m.parameters(), lr=float(g["lr"]))
    l2 = dqn_lib.train_step(len(idx), float(g["gamma"]), m, tg, rb, None, opt, DEV,
                            extract_samples_function=ext, idx=idx)
    assert abs(float(l2) - ref) <= 1e-6 + 1e-13 * abs(ref)
    after = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
    if "params_after" in g:
        np.testing.assert_allclose(after, g["params_after"], rtol=1e-10, atol=1e-10)
    else:
        np.testing.assert_allclose(after[g["grad_sel"]], g["params_after_sampled"], rtol=1e-10,
                                   atol=1e-10)


def test_train_step_reference_compat_noop(G, golden_dir):
    from g2048 import dqn_lib
    from g2048.nets import det_init, make_net

    g = fixture(golden_dir, "conv")
    rb = loaded_replay(G, g)
    m = det_init(make_net("conv", torch.float64, DEV), 0.5)
    tg = det_init(make_net("conv", torch.float64, DEV), 0.2)
    before = [p.detach().clone() for p in m.parameters()]
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    loss = dqn_lib.train_step(512, 0.8, m, tg, rb, None, opt, DEV, reference_compat=True,
                              idx=torch.from_numpy(g["idx"]).to(DEV))
    assert abs(float(loss) - float(g["loss_ref"])) <= 1e-6 + 1e-13 * float(g["loss_ref"])
    assert all(torch.equal(p, q) for p, q in zip(m.parameters(), before))


@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_graphed_learner_equals_eager(G, net):
    """hipGraph-captured update == eager update on the same (deterministic) minibatches.
    Gradients of the first update agree to fp64 roundoff; later losses only loosely, because
    Adam's first steps are ~lr*sign(g) and amplify roundoff in near-zero gradients."""
    from g2048.learner import DQNLearner

    n, C = 2048, 16 * 2048
    env = G.VecEnv2048(n, device=DEV, seed=12)
    rb = G.ReplayBuffer(C, device=DEV)
    env.rollout(C // n, replay=rb)
    calls = {"k": 0}

    def sampler(B, replay):  # fixed strided rows, identical for both paths
        return (torch.arange(B, device=DEV) * 13 + 5) % C

    outs = []
    for graph in (True, False):
        L = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=1024, graph=graph, seed=3,
                       target_sync_every=2, sampler=sampler)
        first = [float(L.update())]
        g1 = L.grad_flat.clone()
        first += [float(L.update()) for _ in range(4)]
        outs.append((first, g1))
    assert outs[0][0][0] == pytest.approx(outs[1][0][0], rel=1e-12)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-9, atol=1e-9 * float(outs[1][1].abs().max()))
    np.testing.assert_allclose(outs[0][0], outs[1][0], rtol=1e-3)
    del calls


def test_trainer_runs_and_learns_statistics(G):
    from g2048.learner import DQNLearner, Trainer

    n = 4096
    env = G.VecEnv2048(n, device=DEV, seed=5)
    rb = G.ReplayBuffer(16 * n, device=DEV)
    L = DQNLearner(rb, net="conv", dtype=torch.float32, batch_size=1024, target_sync_every=10)
    T = Trainer(env, rb, L, updates_per_step=1, eps_decay_episodes=5)
    T.prefill(4)
    for _ in range(60):
        T.step()
    torch.cuda.synchronize()
    st = T.episode_stats()
    assert st["episodes"] > 0 and st["merge_score_mean"] > 0
    assert np.isfinite(float(L.last_loss))
    assert len(rb) == 16 * n
    env.check_errors()


def test_play_one_step_mirror(G):
    from g2048 import dqn_lib
    from g2048.nets import make_net

    n = 2048
    env = G.VecEnv2048(n, device=DEV, seed=8)
    rb = G.ReplayBuffer(4 * n, device=DEV)
    m = make_net("conv", torch.float64, DEV)
    env2, a, r, d, mq = dqn_lib.play_one_step(env, 0.0, m, rb, DEV)
    assert env2 is env and a.shape == (n,) and mq.dtype == torch.float64
    # greedy actions must be the compat argmax of the model's Q on the boards before the step
    env3, a3, r3, d3, _ = dqn_lib.play_one_step(G.VecEnv2048(n, device=DEV, seed=8), 1.0, None, rb)
    assert a3.max() <= 3


@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_fused_graphed_learner_equals_eager(G, net):
    """fp32 fused path (targets + train-grad + reduce + FusedAdam): the captured hipGraph update
    reproduces the eager one -- checks the capture warm-up leaves no trace (weights, Adam state,
    device update counter) and that the sampler epoch advances per replay."""
    from g2048.learner import DQNLearner

    n, C = 2048, 16 * 2048
    env = G.VecEnv2048(n, device=DEV, seed=31)
    rb = G.ReplayBuffer(C, device=DEV)
    env.rollout(C // n, replay=rb)
    outs = []
    for graph in (True, False):
        L = DQNLearner(rb, net=net, dtype=torch.float32, batch_size=1024, graph=graph, seed=9,
                       target_sync_every=3)
        assert L.fused
        losses = [float(L.update()) for _ in range(7)]
        outs.append((losses, torch.cat([p.detach().reshape(-1) for p in L.model.parameters()]),
                     int(L.step_dev)))
    assert outs[0][2] == outs[1][2] == 7
    np.testing.assert_allclose(outs[0][0], outs[1][0], rtol=1e-6)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("net", ["dense64", "conv"])
@pytest.mark.parametrize("graph", [True, False])
def test_fused_target_sync_on_device(G, net, graph):
    """The fused Adam syncs the target net when the device update counter hits a multiple of
    target_sync_every (training_loop's `ep % 100 == 0` sync, src/dqn_lib.py:227-228): after
    update 3 the target equals the online net bitwise; after update 4 it still holds the
    update-3 weights."""
    from g2048.learner import DQNLearner

    n, C = 2048, 16 * 2048
    env = G.VecEnv2048(n, device=DEV, seed=13)
    rb = G.ReplayBuffer(C, device=DEV)
    env.rollout(C // n, replay=rb)
    L = DQNLearner(rb, net=net, dtype=torch.float32, batch_size=512, graph=graph, seed=2,
                   target_sync_every=3)
    t0 = [p.detach().clone() for p in L.target.parameters()]
    flat = lambda m: torch.cat([p.detach().reshape(-1) for p in m.parameters()])  # noqa: E731
    for k in range(1, 5):
        L.update()
        torch.cuda.synchronize()
        if k < 3:
            assert all(torch.equal(a, b) for a, b in zip(L.target.parameters(), t0)), k
        if k == 3:
            after3 = flat(L.model).clone()
            assert torch.equal(flat(L.target), after3)
    assert torch.equal(flat(L.target), after3) and not torch.equal(flat(L.model), after3)
    assert int(L.step_dev) == 4 == L.updates


@pytest.mark.parametrize("net", ["dense64", "conv", "conv-gemm"])
def test_fused_f64_matches_reference(G, golden_dir, net, monkeypatch):
    """The fused float64 updates (g2048_dense64_update_f64 / g2048_convnet_update_f64,
    DQNLearner(dtype=float64)) against the reference train_step fixture: loss within 1e-6
    absolute, y, the gradient and the parameters after one Adam step (src/dqn_lib.py:119-164,
    intended order) to 1e-10 relative (gradient: 1e-10 of its largest element).  conv-gemm: the
    conv update with its conv2 / fc1 weight gradients as K = B GEMMs (G2048_CONV64_WGRAD=gemm)."""
    from g2048.learner import DQNLearner
    from g2048.nets import det_init, make_net

    if net == "conv-gemm":
        monkeypatch.setenv("G2048_CONV64_WGRAD", "gemm")
        net = "conv"
    else:
        monkeypatch.delenv("G2048_CONV64_WGRAD", raising=False)

    g = fixture(golden_dir, net)
    rb = loaded_replay(G, g)
    idx = torch.from_numpy(g["idx"]).to(DEV)
    m = det_init(make_net(net, torch.float64, DEV), 0.5)
    L = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=len(idx),
                   lr=float(g["lr"]), target_sync_every=0, model=m, sampler=lambda B, r: idx)
    assert L.fused and L.f64 and L.kind == net
    det_init(L.target, 0.2)
    L.update()
    torch.cuda.synchronize()
    ref = float(g["loss_ref"])
    assert abs(float(L.last_loss) - ref) <= 1e-6 + 1e-13 * abs(ref), (float(L.last_loss), ref)
    assert torch.equal(L._idx, idx)
    np.testing.assert_allclose(L._y.cpu().numpy(), g["y"], rtol=1e-12, atol=1e-9)
    gref = g["grads"]
    np.testing.assert_allclose(L.grad_flat.cpu().numpy(), gref, rtol=1e-10,
                               atol=1e-10 * max(1.0, float(np.abs(gref).max())))
    after = torch.cat([p.detach().reshape(-1) for p in L.model.parameters()]).cpu().numpy()
    np.testing.assert_allclose(after, g["params_after"], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("batch", [1, 33, 1000, 3000, 4096, 20000, 65536])
@pytest.mark.parametrize("double_dqn", [True, False])
@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_fused_f64_equals_torch_path(G, net, double_dqn, batch):
    """Three fused float64 updates (Philox sampler, Adam, target sync every 2) against the torch
    float64 learner on the same rows: losses and gradients to 1e-9 relative; weights to 1e-6
    absolute (Adam divides by |g| + eps, so a parameter whose summed gradient nearly cancels
    (|g| ~ eps) moves by a step that depends on g's last bits -- the two paths sum the rows in
    different orders).  B = 1 / 33: ragged single tiles (one and three workgroups).  B = 4096
    puts the conv update on 256 workgroups, where train B sums train A's slab terms itself
    (SlabShadow) and the reduce reads them summed; B = 20 000: 1 250 conv tiles over the 256
    workgroups, four or five each (the tile loop and its next-tile prefetch past two); B = 65 536:
    eight times the bench's batch (4 096 conv tiles, 16 per workgroup)."""
    from g2048.learner import DQNLearner

    n = 2048
    env = G.VecEnv2048(n, seed=3, device=DEV)
    rb = G.ReplayBuffer(16 * n, device=DEV)
    env.rollout(16, replay=rb)
    a = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=batch, target_sync_every=2,
                   seed=9, use_double_dqn=double_dqn)
    assert a.fused and a.f64
    rows = torch.zeros(batch, dtype=torch.int64, device=DEV)  # (captured by b's graphs)
    b = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=batch, target_sync_every=2,
                   seed=9, loss_fn=torch.nn.L1Loss(reduction="sum"),  # any torch-path learner
                   use_double_dqn=double_dqn)
    b.loss_fn = None  # ... run with the MSE(sum) loss, fed the fused learner's rows
    b.sampler = lambda B, r: rows
    assert not b.fused
    # change a's weights through torch after construction: the fused conv update must re-pack
    # its operands (ConvUpdate64.ensure_packed, tensor version counters), or its loss differs
    with torch.no_grad():
        for p in a.model.parameters():
            p.mul_(0.9)
        for p in a.target.parameters():
            p.mul_(1.1)
    b.model.load_state_dict(a.model.state_dict())
    b.target.load_state_dict(a.target.state_dict())
    for k in range(3):
        a.update()
        rows.copy_(a._idx)
        b.update()
        torch.cuda.synchronize()
        assert abs(float(a.last_loss) - float(b.last_loss)) <= 1e-9 * abs(float(b.last_loss)), k
        ga, gb = a.grad_flat, b.grad_flat
        assert float((ga - gb).norm()) <= 1e-9 * float(gb.norm()), k
        for p, q in zip(list(a.model.parameters()) + list(a.target.parameters()),
                        list(b.model.parameters()) + list(b.target.parameters())):
            assert torch.allclose(p, q, rtol=0, atol=1e-6), k
        # the next update starts from the same weights on both sides
        with torch.no_grad():
            for p, q in zip(list(b.model.parameters()) + list(b.target.parameters()),
                            list(a.model.parameters()) + list(a.target.parameters())):
                p.copy_(q)


@pytest.mark.parametrize("batch", [700, 4096])
@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_fused_f64_adam_step_equals_folded(G, net, batch):
    """The data-parallel float64 split (fused gradient -> grad_out, then g2048_adam_step_sync_f64)
    moves online and target weights bitwise like the single-process update with Adam folded into
    the reduction, over three updates with a target sync every 2 (B = 4096: the conv update with
    train B's slab sums)."""
    from g2048 import qnet
    from g2048.learner import DQNLearner

    n = 2048
    env = G.VecEnv2048(n, seed=21, device=DEV)
    rb = G.ReplayBuffer(8 * n, device=DEV)
    env.rollout(8, replay=rb)
    a = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=batch, target_sync_every=2,
                   seed=5, graph=False)
    b = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=batch, target_sync_every=2,
                   seed=5, graph=False)
    assert a.f64 and b.f64
    b.model.load_state_dict(a.model.state_dict())
    b.target.load_state_dict(a.target.state_dict())
    b._upd.adam = None  # b: gradient only; Adam64.step applies the update (the DP path)
    assert isinstance(b._adam, qnet.Adam64)
    for _ in range(3):
        a.update()
        b._compute_grads()
        b._adam.step(b.grad_flat, b.step_dev)
        torch.cuda.synchronize()
        assert torch.equal(a.grad_flat, b.grad_flat)
        for p, q in zip(list(a.model.parameters()) + list(a.target.parameters()),
                        list(b.model.parameters()) + list(b.target.parameters())):
            assert torch.equal(p, q)


@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_fused_f32_matches_reference(G, golden_dir, net):
    """The fp32 fast path (the fused kernels the bench times as learner.<net>.fp32) on the
    reference train_step fixture's minibatch and weights: the loss within 2e-5 relative of the
    reference's float64 loss, y within 1e-5, and every gradient tensor within 1e-3 relative
    (L2) of the fixture's float64 gradient (fp32 accumulation over 512 rows)."""
    from g2048.learner import DQNLearner
    from g2048.nets import det_init, make_net

    g = fixture(golden_dir, net)
    rb = loaded_replay(G, g)
    idx = torch.from_numpy(g["idx"]).to(DEV)
    m = det_init(make_net(net, torch.float32, DEV), 0.5)
    L = DQNLearner(rb, net=net, dtype=torch.float32, batch_size=len(idx), lr=float(g["lr"]),
                   target_sync_every=0, model=m, sampler=lambda B, r: idx)
    assert L.fused and not L.f64
    det_init(L.target, 0.2)
    L.update()
    torch.cuda.synchronize()
    ref = float(g["loss_ref"])
    assert abs(float(L.last_loss) - ref) <= 2e-5 * abs(ref), (float(L.last_loss), ref)
    np.testing.assert_allclose(L._y.cpu().numpy(), g["y"], rtol=1e-5, atol=1e-4)
    grad = L.grad_flat.double().cpu().numpy()
    gref = g["grads"]
    off = 0
    for p in L.model.parameters():
        k = p.numel()
        a, b = grad[off:off + k], gref[off:off + k]
        assert np.linalg.norm(a - b) <= 1e-3 * max(np.linalg.norm(b), 1e-12), (off, k)
        off += k


@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_fused_f64_vanilla_matches_reference(G, golden_dir, net):
    """The fused float64 updates on the vanilla-DQN branch (use_double_dqn=False,
    src/dqn_lib.py:133-144: y = r + (1-d)*gamma*max_a Q_tgt(s')) against the reference-run
    fixture learner_<net>_vanilla.npz, whose weights make the branch differ from Double DQN on
    most rows: loss within 1e-6 absolute, y to 1e-12, gradient and one Adam step to 1e-10."""
    from g2048.learner import DQNLearner
    from g2048.nets import det_init

    g = fixture(golden_dir, f"{net}_vanilla")
    assert not bool(g["use_double_dqn"])
    rb = loaded_replay(G, g)
    idx = torch.from_numpy(g["idx"]).to(DEV)
    m, _ = fixture_nets(g, net)
    L = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=len(idx), lr=float(g["lr"]),
                   target_sync_every=0, model=m, sampler=lambda B, r: idx, use_double_dqn=False)
    assert L.fused and L.f64 and L.kind == net
    det_init(L.target, float(g["tgt_phase"]), float(g["init_freq"]))
    L.update()
    torch.cuda.synchronize()
    ref = float(g["loss_ref"])
    assert abs(float(L.last_loss) - ref) <= 1e-6 + 1e-13 * abs(ref), (float(L.last_loss), ref)
    np.testing.assert_allclose(L._y.cpu().numpy(), g["y"], rtol=1e-12, atol=1e-9)
    gref = g["grads"]
    np.testing.assert_allclose(L.grad_flat.cpu().numpy(), gref, rtol=1e-10,
                               atol=1e-10 * max(1.0, float(np.abs(gref).max())))
    after = torch.cat([p.detach().reshape(-1) for p in L.model.parameters()]).cpu().numpy()
    np.testing.assert_allclose(after, g["params_after"], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("name,net,double", [("conv_vanilla", "conv", False),
                                             ("dense64_vanilla", "dense64", False),
                                             ("dense_b5000", "dense", True)])
def test_torch_path_vanilla_and_b5000_match_reference(G, golden_dir, name, net, double):
    """The torch-ROCm float64 learner path (HIP gather + encode, then torch) on the vanilla-DQN
    fixtures and on dense-ref at BASELINE configs[0]'s batch of 5000
    (src/configs/double_dqn_dense.py:17): loss within 1e-6 absolute, y and Q to 1e-12."""
    from g2048 import dqn_lib

    g = fixture(golden_dir, name)
    rb = loaded_replay(G, g)
    m, tg = fixture_nets(g, net)
    idx = torch.from_numpy(g["idx"]).to(DEV)
    ext = dqn_lib.extract_samples_conv if net == "conv" else dqn_lib.extract_samples_dense
    s, a, r, s2, d = dqn_lib.sample_experiences(len(idx), rb, DEV, None, ext, idx=idx)
    loss, q, y = dqn_lib.dqn_loss(m, tg, s, a, r, s2, d, float(g["gamma"]), use_double_dqn=double)
    ref = float(g["loss_ref"])
    assert abs(float(loss.detach()) - ref) <= 1e-6 + 1e-13 * abs(ref), (float(loss.detach()), ref)
    np.testing.assert_allclose(q.detach().cpu().numpy(), g["q"], rtol=1e-12, atol=1e-6)
    np.testing.assert_allclose(y.cpu().numpy(), g["y"], rtol=1e-12, atol=1e-6)
    opt = torch.optim.Adam(m.parameters(), lr=float(g["lr"]))
    l2 = dqn_lib.train_step(len(idx), float(g["gamma"]), m, tg, rb, None, opt, DEV,
                            use_double_dqn=double, extract_samples_function=ext, idx=idx)
    assert abs(float(l2) - ref) <= 1e-6 + 1e-13 * abs(ref)
    after = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
    if "params_after" in g:
        np.testing.assert_allclose(after, g["params_after"], rtol=1e-10, atol=1e-10)
    else:
        np.testing.assert_allclose(after[g["grad_sel"]], g["params_after_sampled"], rtol=1e-10,
                                   atol=1e-10)


@pytest.mark.parametrize("double_dqn", [True, False])
def test_dense_ref_f64_hip_targets(G, double_dqn):
    """The torch-path learner of the reference dense net in float64 forms the Bellman target's
    two no-grad forwards with the HIP dense forward (DQNLearner._dfwd_tg): loss and gradient of
    three updates against torch autograd through dqn_lib.dqn_loss on the same rows and the same
    pre-update weights, to 1e-9 relative."""
    import copy

    from g2048 import dqn_lib
    from g2048.learner import DQNLearner

    n = 2048
    env = G.VecEnv2048(n, seed=13, device=DEV)
    rb = G.ReplayBuffer(8 * n, device=DEV)
    env.rollout(8, replay=rb)
    rows = torch.zeros(2000, dtype=torch.int64, device=DEV)
    L = DQNLearner(rb, net="dense", dtype=torch.float64, batch_size=2000, target_sync_every=2,
                   seed=4, use_double_dqn=double_dqn,
                   loss_fn=torch.nn.L1Loss(reduction="sum"))  # the torch path ...
    L.loss_fn = None  # ... with the MSE(sum) loss
    assert not L.fused and L._dfwd_tg is not None
    L.sampler = lambda B, r: rows
    gen = torch.Generator(device=DEV).manual_seed(1)
    for k in range(3):
        rows.copy_(torch.randint(0, 8 * n, (2000,), device=DEV, generator=gen))
        m0, t0 = copy.deepcopy(L.model), copy.deepcopy(L.target)
        L.update()
        s, a, r, s2, d = dqn_lib.sample_experiences(2000, rb, DEV, None,
                                                    dqn_lib.extract_samples_dense,
                                                    dtype=torch.float64, idx=rows)
        loss, _, _ = dqn_lib.dqn_loss(m0, t0, s, a, r, s2, d, L.gamma, double_dqn, None)
        loss.backward()
        torch.cuda.synchronize()
        assert abs(float(L.last_loss) - float(loss)) <= 1e-9 * abs(float(loss)), k
        gref = torch.cat([p.grad.reshape(-1) for p in m0.parameters()])
        assert float((L.grad_flat - gref).norm()) <= 1e-9 * float(gref.norm()), k


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("net", ["dense", "conv"])
def test_torch_path_graph_replays_match_eager(G, net, dtype):
    """Back-to-back replays of the torch-path learner's captured update against the same learner
    run eagerly on the same rows and weights, at B = 8192: every parameter's gradient to 1e-9
    relative on every update.  (torch's dim-0 sum for the bias gradients gave stale results in
    replays of the captured update -- the weights' gradients stayed right -- so nets.Linear
    forms them as a GEMM.)"""
    from g2048.learner import DQNLearner

    n, B = 4096, 8192
    env = G.VecEnv2048(n, seed=17, device=DEV)
    rb = G.ReplayBuffer(8 * n, device=DEV)
    env.rollout(8, replay=rb)
    rows = torch.zeros(B, dtype=torch.int64, device=DEV)
    kw = dict(net=net, dtype=dtype, batch_size=B, target_sync_every=2, seed=7,
              loss_fn=torch.nn.L1Loss(reduction="sum"),  # any torch-path learner ...
              sampler=lambda b, r: rows)
    a = DQNLearner(rb, graph=True, **kw)
    b = DQNLearner(rb, graph=False, **kw)
    assert not a.fused and not b.fused
    a.loss_fn = b.loss_fn = None  # ... run with the MSE(sum) loss
    b.model.load_state_dict(a.model.state_dict())
    b.target.load_state_dict(a.target.state_dict())
    gen = torch.Generator(device=DEV).manual_seed(3)
    sizes = [p.numel() for p in a.model.parameters()]
    tol = 1e-9 if dtype == torch.float64 else 1e-4
    for k in range(4):
        rows.copy_(torch.randint(0, 8 * n, (B,), device=DEV, generator=gen))
        a.update()
        b.update()
        torch.cuda.synchronize()
        off = 0
        for i, sz in enumerate(sizes):
            ga, gb = a.grad_flat[off:off + sz], b.grad_flat[off:off + sz]
            assert float((ga - gb).norm()) <= tol * float(gb.norm()), (k, i)
            off += sz
        with torch.no_grad():  # the next update starts from the same weights on both sides
            for p, q in zip(list(a.model.parameters()) + list(a.target.parameters()),
                            list(b.model.parameters()) + list(b.target.parameters())):
                p.copy_(q)


@pytest.mark.parametrize("double_dqn", [True, False])
@pytest.mark.parametrize("batch", [700, 4096, 8192])
def test_conv64_train_a8_equals_four_wave(G, batch, double_dqn):
    """The eight-wave train A (k_conv64_train_a8, two waves per SIMD) keeps every sum of the
    four-wave k_conv64_train_a in the same order: three float64 conv updates with each (the
    eight-wave one selected by G2048_CONV64_TRAIN_A=8) agree bit for bit -- y, loss, the summed
    gradient (the reduce writes it beside the folded Adam) and both nets' weights.  Both in the
    slab form of the weight gradients (G2048_CONV64_WGRAD=slab), the only one with an eight-wave
    train A."""
    from g2048.learner import DQNLearner

    n = 2048
    env = G.VecEnv2048(n, seed=31, device=DEV)
    rb = G.ReplayBuffer(16 * n, device=DEV)
    env.rollout(16, replay=rb)
    outs = []
    os.environ["G2048_CONV64_WGRAD"] = "slab"
    for eight in (False, True):
        if eight:
            os.environ["G2048_CONV64_TRAIN_A"] = "8"
        try:
            L = DQNLearner(rb, net="conv", dtype=torch.float64, batch_size=batch, seed=6,
                           target_sync_every=2, graph=False, use_double_dqn=double_dqn)
            assert L.fused and L.f64
            res = []
            for _ in range(3):
                L.update()
                torch.cuda.synchronize()
                res += [L._y.clone(), L.last_loss.reshape(1).clone(), L.grad_flat.clone()]
            res += [p.detach().reshape(-1).clone() for p in
                    list(L.model.parameters()) + list(L.target.parameters())]
            outs.append(torch.cat(res))
        finally:
            os.environ.pop("G2048_CONV64_TRAIN_A", None)
    os.environ.pop("G2048_CONV64_WGRAD", None)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("double_dqn", [True, False])
@pytest.mark.parametrize("batch", [1, 33, 700, 4096, 8192, 20000])
def test_conv64_wgrad_gemm_equals_slabs(G, batch, double_dqn, monkeypatch):
    """The float64 conv update's two forms of the conv2 / fc1 weight gradients -- K = B GEMMs
    over stored operands (k_conv64_wgrad, direct form per conv2 tap; G2048_CONV64_WGRAD=gemm)
    and the per-workgroup slabs (the default) -- from the same state (weights, Adam
    moments, update counter copied before every update): y bitwise, the loss to 1e-14 relative
    (the slab form may run the eight-wave train A, whose loss sums in another order), every
    gradient tensor to 1e-12 relative (float64 summation order), three updates; the GEMM form
    run to run bitwise."""
    from g2048.learner import DQNLearner

    n = 2048
    env = G.VecEnv2048(n, seed=37, device=DEV)
    rb = G.ReplayBuffer(16 * n, device=DEV)
    env.rollout(16, replay=rb)
    Ls = [DQNLearner(rb, net="conv", dtype=torch.float64, batch_size=batch, seed=6,
                     target_sync_every=2, graph=False, use_double_dqn=double_dqn,
                     data_parallel=True)  # gradient-only updates: grad_flat is the summed gradient
          for _ in range(3)]
    modes = ("gemm", "slab", "gemm")

    def state(L):
        return (list(L.model.parameters()) + list(L.target.parameters())
                + [L._adam.exp_avg, L._adam.exp_avg_sq, L.step_dev])

    for it in range(3):
        with torch.no_grad():
            for L in (Ls[0], Ls[2]):
                for x, y in zip(state(L), state(Ls[1])):
                    x.copy_(y)
        got = []
        for L, mode in zip(Ls, modes):
            if mode == "gemm":
                monkeypatch.setenv("G2048_CONV64_WGRAD", "gemm")
            else:
                monkeypatch.delenv("G2048_CONV64_WGRAD", raising=False)
            L.update()
            torch.cuda.synchronize()
            got.append((L._y.clone(), L.last_loss.clone(), L.grad_flat.clone()))
        (ya, la, ga), (yb, lb, gb), (yc, lc, gc) = got
        assert torch.equal(ya, yb), it
        assert abs(float(la) - float(lb)) <= 1e-14 * abs(float(lb)), (it, float(la), float(lb))
        assert torch.equal(ga, gc) and torch.equal(la, lc), it  # run to run
        off = 0
        for i, p in enumerate(Ls[0].model.parameters()):
            sz = p.numel()
            x, y = ga[off:off + sz], gb[off:off + sz]
            assert float((x - y).norm()) <= 1e-12 * float(y.norm()) + 1e-300, (it, i, batch)
            off += sz
