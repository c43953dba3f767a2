"""Fused conv Q-net forward (HIP, f32 MFMA) vs the torch forward of the same weights."""
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


@pytest.mark.parametrize("n", [1, 31, 32, 1000, 16383, 20001, 65536])
def test_conv_forward_matches_torch(G, n):
    from g2048.nets import det_init, make_net
    from g2048.qnet import conv_forward

    env = G.VecEnv2048(n, device=DEV, seed=n)
    env.rollout(40)
    m = make_net("conv", torch.float32, DEV)
    det_init(m, 0.3)
    q = conv_forward(m, env.board)
    with torch.no_grad():
        ref = m(env.board.to(torch.float32).view(n, 1, 4, 4))
        ref64 = make_net("conv", torch.float64, DEV)
        ref64.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
        r64 = ref64(env.board.to(torch.float64).view(n, 1, 4, 4))
    torch.testing.assert_close(q, ref, rtol=2e-5, atol=2e-5 * float(ref.abs().max()))
    torch.testing.assert_close(q.double(), r64, rtol=2e-5, atol=2e-5 * float(r64.abs().max()))


def test_conv_forward_gather_and_random_weights(G):
    from g2048.nets import make_net
    from g2048.qnet import conv_forward

    torch.manual_seed(0)
    m = make_net("conv", torch.float32, DEV)  # default (kaiming-uniform) init
    rows = torch.randint(0, 14, (5000, 16), dtype=torch.uint8, device=DEV)
    idx = torch.randint(0, 5000, (777,), device=DEV)
    q = conv_forward(m, rows, idx)
    with torch.no_grad():
        ref = m(rows[idx].to(torch.float32).view(-1, 1, 4, 4))
    torch.testing.assert_close(q, ref, rtol=2e-5, atol=2e-5 * float(ref.abs().max()))
    assert q.shape == (777, 4)


def test_fused_learner_matches_unfused(G):
    """The conv learner with the fused target forwards computes the same first loss and gradient
    as the all-torch path on the same minibatch (fp32 tolerance)."""
    from g2048.learner import DQNLearner

    n, C = 2048, 8 * 2048
    env = G.VecEnv2048(n, device=DEV, seed=21)
    rb = G.ReplayBuffer(C, device=DEV)
    env.rollout(C // n, replay=rb)

    def sampler(B, replay):
        return (torch.arange(B, device=DEV) * 7 + 3) % C

    res = []
    for fused in (True, False):
        L = DQNLearner(rb, net="conv", dtype=torch.float32, batch_size=2048, graph=False, seed=4,
                       sampler=sampler)
        L.fused = fused
        loss = float(L.update())
        res.append((loss, L.grad_flat.clone()))
    assert res[0][0] == pytest.approx(res[1][0], rel=1e-4)
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-3, atol=1e-3 * float(res[1][1].abs().max()))


@pytest.mark.parametrize("B", [1, 17, 32, 1000, 3000, 9000, 20000, 65536])
def test_conv_train_grad_matches_autograd(G, B):
    """Fused graded half of train_step vs torch autograd in float64 on the same minibatch.
    B = 1 / 17: one ragged tile on one workgroup; B = 1000: 63 workgroups, the reduce sums every slab term; 3000: 188 (train bwd sums train
    fwd's terms, k_reduce_pre over a partial round of slabs); 20000: 313 (two rounds); 65536: eight
    times the bench's batch."""
    from g2048.nets import make_net
    from g2048.qnet import ConvTrainGrad

    C = 16384
    env = G.VecEnv2048(4096, device=DEV, seed=B)
    rb = G.ReplayBuffer(C, device=DEV)
    env.rollout(C // 4096, replay=rb)
    torch.manual_seed(B)
    m = make_net("conv", torch.float32, DEV)
    idx = torch.randint(0, C, (B,), device=DEV)
    y = (torch.randn(B, device=DEV) * 20 + 30).float()
    grad = torch.full((33476,), float("nan"), device=DEV)
    loss = torch.zeros((), device=DEV)
    ConvTrainGrad(m, B)(rb.s, rb.a, idx, y, grad, loss)

    m64 = make_net("conv", torch.float64, DEV)
    m64.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
    s = rb.s[idx].double().view(B, 1, 4, 4)
    a = rb.a[idx].long()
    ref_loss = ((m64(s).gather(1, a[:, None])[:, 0] - y.double()) ** 2).sum()
    ref_loss.backward()
    ref = torch.cat([p.grad.reshape(-1) for p in m64.parameters()])
    assert torch.isfinite(grad).all()
    assert float(loss) == pytest.approx(float(ref_loss), rel=1e-5)
    rel = float((grad.double() - ref).norm() / ref.norm())
    assert rel < 1e-4, rel
    # per-parameter-tensor check (catches a layout error in one block)
    off = 0
    for p in m64.parameters():
        g, r = grad[off:off + p.numel()].double(), ref[off:off + p.numel()]
        assert float((g - r).norm()) <= 1e-3 * float(r.norm()) + 1e-6, p.shape
        off += p.numel()


def _filled_ring(G, seed, C=16384, n=4096):
    env = G.VecEnv2048(n, device=DEV, seed=seed)
    rb = G.ReplayBuffer(C, device=DEV)
    env.rollout(C // n, replay=rb)
    return rb


@pytest.mark.parametrize("double_dqn", [True, False])
def test_conv_targets_match_torch(G, double_dqn):
    from g2048 import dqn_lib
    from g2048.nets import make_net
    from g2048.qnet import conv_forward, conv_params, conv_targets

    rb = _filled_ring(G, 3)
    torch.manual_seed(1)
    on, tg = make_net("conv", torch.float32, DEV), make_net("conv", torch.float32, DEV)
    B = 3000
    idx = torch.randint(0, rb.capacity, (B,), device=DEV)
    io = torch.empty(B, dtype=torch.int64, device=DEV)
    y = torch.empty(B, dtype=torch.float32, device=DEV)
    conv_targets(conv_params(on), conv_params(tg), rb, B, io, y, 0.8, double_dqn, idx_in=idx)
    assert torch.equal(io, idx)
    ref = dqn_lib.targets_from_q(conv_forward(on, rb.s2, idx), conv_forward(tg, rb.s2, idx),
                                 rb.r[idx], rb.d[idx], 0.8, double_dqn)
    torch.testing.assert_close(y, ref, rtol=1e-6, atol=1e-5)


def test_conv_targets_sampler_matches_ring_sampler(G):
    """In-kernel indices == g2048_replay_sample_encode's Philox draw for the same (seed, epoch)."""
    from g2048.nets import make_net
    from g2048.qnet import conv_params, conv_targets

    rb = _filled_ring(G, 4)
    m = make_net("conv", torch.float32, DEV)
    B = 2048
    epoch = torch.tensor([5], dtype=torch.int64, device=DEV)
    io = torch.empty(B, dtype=torch.int64, device=DEV)
    y = torch.empty(B, dtype=torch.float32, device=DEV)
    conv_targets(conv_params(m), conv_params(m), rb, B, io, y, 0.8, True, seed=77, epoch=epoch)
    ref_idx = rb.sample_encode(B, torch.float32, seed=77, epoch=5)[5]
    assert torch.equal(io, ref_idx)
    assert int(io.min()) >= 0 and int(io.max()) < rb.capacity


def test_fused_adam_matches_torch_adam(G):
    from g2048.nets import make_net
    from g2048.optim import FusedAdam

    torch.manual_seed(2)
    m1 = make_net("conv", torch.float32, DEV)
    m2 = make_net("conv", torch.float32, DEV)
    m2.load_state_dict(m1.state_dict())
    ref = torch.optim.Adam(m2.parameters(), lr=1e-2)
    fa = FusedAdam(list(m1.parameters()), lr=1e-2)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    for it in range(5):
        grads = [torch.randn_like(p) * (10.0 ** (it - 2)) for p in m1.parameters()]
        for p, g in zip(m2.parameters(), grads):
            p.grad = g.clone()
        ref.step()
        step += 1
        fa.step(torch.cat([g.reshape(-1) for g in grads]), step)
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p1, p2, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B", [2048, 4096])
@pytest.mark.parametrize("sync_every", [0, 2])
def test_conv_train_adam_equals_grad_then_adam(G, sync_every, B):
    """g2048_convnet_train_adam (Adam + target sync folded into the gradient reduction) is
    bitwise train_grad followed by g2048_adam_step_sync, over 3 updates.  B = 4096 runs on 256
    workgroups, where train bwd sums train fwd's slab terms itself (SlabShadow)."""
    from g2048.nets import make_net
    from g2048.optim import FusedAdam
    from g2048.qnet import ConvTrainGrad

    C = 16384
    env = G.VecEnv2048(4096, device=DEV, seed=5)
    rb = G.ReplayBuffer(C, device=DEV)
    env.rollout(C // 4096, replay=rb)
    torch.manual_seed(5)
    nets = [make_net("conv", torch.float32, DEV) for _ in range(4)]
    for m in nets[1:]:
        m.load_state_dict(nets[0].state_dict())
    (m1, t1), (m2, t2) = (nets[0], nets[1]), (nets[2], nets[3])
    a1, a2 = FusedAdam(list(m1.parameters()), lr=1e-2), FusedAdam(list(m2.parameters()), lr=1e-2)
    if sync_every:
        a1.attach_target(list(t1.parameters()), sync_every)
        a2.attach_target(list(t2.parameters()), sync_every)
    tg1, tg2 = ConvTrainGrad(m1, B), ConvTrainGrad(m2, B, adam=a2)
    s1 = torch.zeros(1, dtype=torch.int64, device=DEV)
    s2 = torch.zeros(1, dtype=torch.int64, device=DEV)
    g1 = torch.zeros(33476, device=DEV)
    g2 = torch.zeros(33476, device=DEV)
    l1, l2 = torch.zeros((), device=DEV), torch.zeros((), device=DEV)
    for it in range(3):
        idx = torch.randint(0, C, (B,), device=DEV)
        y = (torch.randn(B, device=DEV) * 20 + 30).float()
        tg1(rb.s, rb.a, idx, y, g1, l1, s1)
        a1.step(g1, s1)
        tg2(rb.s, rb.a, idx, y, g2, l2, s2)
        assert torch.equal(g1, g2) and torch.equal(l1, l2)
    assert int(s1) == int(s2) == 3
    for p1, p2 in zip(list(m1.parameters()) + list(t1.parameters()),
                      list(m2.parameters()) + list(t2.parameters())):
        assert torch.equal(p1, p2)
    assert torch.equal(a1.exp_avg, a2.exp_avg) and torch.equal(a1.exp_avg_sq, a2.exp_avg_sq)
    if sync_every:  # synced at t = 2, then the online net moved on at t = 3
        assert not all(torch.equal(p, q) for p, q in zip(m2.parameters(), t2.parameters()))
        assert not all(torch.equal(p, q) for p, q in zip(t2.parameters(), nets[0].parameters()))


@pytest.mark.parametrize("B,double_dqn,sampled,adam,sync_every",
                         [(8192, True, True, True, 2), (2048, True, False, True, 0),
                          (1000, False, True, True, 3), (8192, True, True, False, 0),
                          (33, True, True, True, 0)])
def test_conv_update_equals_targets_then_train(G, B, double_dqn, sampled, adam, sync_every):
    """g2048_convnet_update (Double DQN: the targets launch split into an online half and a
    target half, y formed in the train launch) is bitwise conv_targets followed by
    ConvTrainGrad (+ Adam folded in, + target sync) over 3 updates: indices, y, loss, gradient
    (adam=False), online / target weights and Adam state."""
    from g2048 import qnet
    from g2048.nets import make_net
    from g2048.optim import FusedAdam

    C = 16384
    rb = _filled_ring(G, 17, C=C)
    torch.manual_seed(B)
    nets = [make_net("conv", torch.float32, DEV) for _ in range(4)]
    with torch.no_grad():  # online pair 0 / 2, target pair 1 / 3 (differs from the online net)
        nets[2].load_state_dict(nets[0].state_dict())
        for p, q in zip(nets[1].parameters(), nets[0].parameters()):
            p.copy_(q * 0.9)
        nets[3].load_state_dict(nets[1].state_dict())
    (m1, t1), (m2, t2) = (nets[0], nets[1]), (nets[2], nets[3])
    a1, a2 = FusedAdam(list(m1.parameters()), lr=1e-2), FusedAdam(list(m2.parameters()), lr=1e-2)
    if sync_every:
        a1.attach_target(list(t1.parameters()), sync_every)
        a2.attach_target(list(t2.parameters()), sync_every)
    tr1 = qnet.ConvTrainGrad(m1, B, adam=a1 if adam else None)
    upd = qnet.ConvUpdate(m2, t2, B, adam=a2 if adam else None)
    p1on, p1tg = qnet.net_params(m1), qnet.net_params(t1)
    kw = dict(device=DEV)
    s1, s2 = torch.zeros(1, dtype=torch.int64, **kw), torch.zeros(1, dtype=torch.int64, **kw)
    i1, i2 = torch.zeros(B, dtype=torch.int64, **kw), torch.zeros(B, dtype=torch.int64, **kw)
    y1, y2 = torch.zeros(B, **kw), torch.zeros(B, **kw)
    g1, g2 = torch.zeros(33476, **kw), torch.zeros(33476, **kw)
    l1, l2 = torch.zeros((), **kw), torch.zeros((), **kw)
    for it in range(3):
        idx_in = None if sampled else torch.randint(0, C, (B,), **kw)
        qnet.conv_targets(p1on, p1tg, rb, B, i1, y1, 0.8, double_dqn, seed=7, epoch=s1,
                          idx_in=idx_in)
        tr1(rb.s, rb.a, i1, y1, g1, l1, s1)
        if not adam:
            a1.step(g1, s1)
        upd(rb, i2, y2, s2, 0.8, double_dqn, seed=7, idx_in=idx_in,
            grad_out=None if adam else g2, loss_out=l2)
        if not adam:
            a2.step(g2, s2)
            assert torch.equal(g1, g2), it
        assert torch.equal(i1, i2) and torch.equal(y1, y2) and torch.equal(l1, l2), it
    assert int(s1) == int(s2) == 3
    for p1, p2 in zip(list(m1.parameters()) + list(t1.parameters()),
                      list(m2.parameters()) + list(t2.parameters())):
        assert torch.equal(p1, p2)
    assert torch.equal(a1.exp_avg, a2.exp_avg) and torch.equal(a1.exp_avg_sq, a2.exp_avg_sq)


# ------------------------------------------------------------------ dense 16-64-4 (configs[2])
def test_dense64_forward_and_targets(G):
    from g2048 import dqn_lib
    from g2048.nets import make_net
    from g2048.qnet import forward, net_params, targets

    rb = _filled_ring(G, 9)
    torch.manual_seed(3)
    on, tg = make_net("dense64", torch.float32, DEV), make_net("dense64", torch.float32, DEV)
    idx = torch.randint(0, rb.capacity, (5000,), device=DEV)
    q = forward(on, rb.s2, idx)
    with torch.no_grad():
        ref = on(rb.s2[idx].float())
    torch.testing.assert_close(q, ref, rtol=2e-5, atol=2e-5 * float(ref.abs().max()))
    io = torch.empty(5000, dtype=torch.int64, device=DEV)
    y = torch.empty(5000, dtype=torch.float32, device=DEV)
    targets("dense64", net_params(on), net_params(tg), rb, 5000, io, y, 0.8, True, idx_in=idx)
    ref_y = dqn_lib.targets_from_q(forward(on, rb.s2, idx), forward(tg, rb.s2, idx), rb.r[idx],
                                   rb.d[idx], 0.8, True)
    torch.testing.assert_close(y, ref_y, rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("B", [64, 1000, 20000])
def test_dense64_train_grad_matches_autograd(G, B):
    from g2048.nets import make_net
    from g2048.qnet import TrainGrad

    rb = _filled_ring(G, B)
    torch.manual_seed(B)
    m = make_net("dense64", torch.float32, DEV)
    idx = torch.randint(0, rb.capacity, (B,), device=DEV)
    y = (torch.randn(B, device=DEV) * 20 + 30).float()
    grad = torch.full((1348,), float("nan"), device=DEV)
    loss = torch.zeros((), device=DEV)
    TrainGrad(m, B)(rb.s, rb.a, idx, y, grad, loss)
    m64 = make_net("dense64", torch.float64, DEV)
    m64.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
    ref_loss = ((m64(rb.s[idx].double()).gather(1, rb.a[idx].long()[:, None])[:, 0]
                 - y.double()) ** 2).sum()
    ref_loss.backward()
    ref = torch.cat([p.grad.reshape(-1) for p in m64.parameters()])
    assert torch.isfinite(grad).all()
    assert float(loss) == pytest.approx(float(ref_loss.detach()), rel=1e-5)
    off = 0
    for p in m64.parameters():
        g, r = grad[off:off + p.numel()].double(), ref[off:off + p.numel()]
        assert float((g - r).norm()) <= 1e-4 * float(r.norm()) + 1e-6, p.shape
        off += p.numel()


@pytest.mark.parametrize("B,double_dqn,sampled", [(8192, True, True), (1000, False, True),
                                                   (45, True, False), (20000, True, False)])
def test_dense64_update_matches_pieces(G, B, double_dqn, sampled):
    """g2048_dense64_update (sampler + targets + gradient in one launch, Adam in the reduction)
    against targets -> train_grad -> FusedAdam: identical rows and targets (bitwise), the
    gradient within fp32 summation-order tolerance (32- vs 64-row slabs), the same update
    counter; and its grad-only mode + FusedAdam.step is bitwise its Adam-in-reduction mode."""
    import copy

    from g2048.nets import make_net
    from g2048.optim import FusedAdam
    from g2048.qnet import Dense64Update, TrainGrad, net_params, targets

    rb = _filled_ring(G, B % 97)
    torch.manual_seed(B)
    on = make_net("dense64", torch.float32, DEV)
    tg = make_net("dense64", torch.float32, DEV)
    idx_in = None if sampled else torch.randint(0, rb.capacity, (B,), device=DEV)
    seed = 0xABCDEF12345
    nets = [copy.deepcopy(on) for _ in range(3)]
    steps = [torch.full((1,), 11, dtype=torch.int64, device=DEV) for _ in range(3)]
    outs = []
    # (0) pieces: targets -> train_grad (bumps the counter) -> FusedAdam
    io, y = torch.empty(B, dtype=torch.int64, device=DEV), torch.empty(B, device=DEV)
    g0, l0 = torch.empty(1348, device=DEV), torch.zeros((), device=DEV)
    targets("dense64", net_params(nets[0]), net_params(tg), rb, B, io, y, 0.8, double_dqn, seed,
            steps[0], idx_in)
    TrainGrad(nets[0], B)(rb.s, rb.a, io, y, g0, l0, steps[0])
    FusedAdam(list(nets[0].parameters()), lr=1e-2).step(g0, steps[0])
    outs.append((io, y, g0, l0))
    # (1) fused update with Adam in the reduction; (2) fused, gradient only, then FusedAdam
    for k, with_adam in ((1, True), (2, False)):
        adam = FusedAdam(list(nets[k].parameters()), lr=1e-2)
        io_k, y_k = torch.empty(B, dtype=torch.int64, device=DEV), torch.empty(B, device=DEV)
        g_k, l_k = torch.full((1348,), float("nan"), device=DEV), torch.zeros((), device=DEV)
        Dense64Update(nets[k], tg, B, adam=adam if with_adam else None)(
            rb, io_k, y_k, steps[k], 0.8, double_dqn, seed, idx_in, grad_out=g_k, loss_out=l_k)
        if not with_adam:
            adam.step(g_k, steps[k])
        outs.append((io_k, y_k, g_k, l_k))
    torch.cuda.synchronize()
    for k in (1, 2):
        assert int(steps[k]) == 12 == int(steps[0])
        assert torch.equal(outs[k][0], outs[0][0])
        assert torch.equal(outs[k][1], outs[0][1])
        torch.testing.assert_close(outs[k][2], outs[0][2], rtol=1e-4,
                                   atol=1e-5 * float(outs[0][2].abs().max()))
        assert float(outs[k][3]) == pytest.approx(float(outs[0][3]), rel=1e-5)
    assert torch.equal(outs[1][2], outs[2][2]) and torch.equal(outs[1][3], outs[2][3])
    for p1, p2, p0 in zip(nets[1].parameters(), nets[2].parameters(), nets[0].parameters()):
        assert torch.equal(p1, p2)
        torch.testing.assert_close(p1, p0, rtol=1e-4, atol=1e-5)  # ~lr*sign(g) first steps
    if sampled:
        assert int(outs[1][0].min()) >= 0 and int(outs[1][0].max()) < int(rb.count)


@pytest.mark.parametrize("B", [32, 1000, 8192])
def test_fused_learner_kernels_are_deterministic(G, B):
    """Bitwise-identical results across repeated launches on the same inputs: the conv / dense64
    forward, targets and train-gradient kernels (the gradient reduction is fixed-order; a race
    shows up here even when it stays inside the parity tolerances)."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    rb = _filled_ring(G, 5 + B)
    torch.manual_seed(B)
    idx = torch.randint(0, rb.capacity, (B,), device=DEV)
    y = (torch.randn(B, device=DEV) * 20 + 30).float()
    epoch = torch.tensor([3], dtype=torch.int64, device=DEV)
    for kind in ("conv", "dense64"):
        m = det_init(make_net(kind, torch.float32, DEV), 0.4)
        tgt = det_init(make_net(kind, torch.float32, DEV), 0.9)
        po, pt = qnet.net_params(m), qnet.net_params(tgt)
        tg = qnet.TrainGrad(m, B)
        outs = []
        for _ in range(6):
            grad = torch.full((tg.n_params,), float("nan"), device=DEV)
            loss = torch.zeros((), device=DEV)
            tg(rb.s, rb.a, idx, y, grad, loss)
            q = qnet.forward(m, rb.s, idx)
            io = torch.empty(B, dtype=torch.int64, device=DEV)
            yo = torch.empty(B, dtype=torch.float32, device=DEV)
            qnet.targets(kind, po, pt, rb, B, io, yo, seed=7, epoch=epoch)
            outs.append((grad, loss, q, io, yo))
        torch.cuda.synchronize()
        assert torch.isfinite(outs[0][0]).all()
        for o in outs[1:]:
            for a, b in zip(o, outs[0]):
                assert torch.equal(a, b), kind
    # the fused dense64 update (gradient-only mode, counter reset per launch)
    m = det_init(make_net("dense64", torch.float32, DEV), 0.4)
    tgt = det_init(make_net("dense64", torch.float32, DEV), 0.9)
    upd = qnet.Dense64Update(m, tgt, B)
    outs = []
    for _ in range(6):
        st = torch.tensor([3], dtype=torch.int64, device=DEV)
        io = torch.empty(B, dtype=torch.int64, device=DEV)
        yo = torch.empty(B, dtype=torch.float32, device=DEV)
        grad = torch.full((1348,), float("nan"), device=DEV)
        loss = torch.zeros((), device=DEV)
        upd(rb, io, yo, st, seed=7, grad_out=grad, loss_out=loss)
        outs.append((grad, loss, io, yo, st))
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0][0]).all() and int(outs[0][4]) == 4
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            assert torch.equal(a, b), "dense64 update"


def _greedy_mask(env, eps):
    """Boards whose next eps-greedy step takes the greedy branch: the step's Philox block
    (counter = step t, global board id; key = seed) from the oracle, u.y / 2^32 >= eps_b."""
    from oracle import oracle as O

    clock = env.clock.cpu().numpy().view(np.uint64)
    seed = env.seed & ((1 << 64) - 1)
    key = [seed & 0xFFFFFFFF, seed >> 32]
    out = np.zeros(env.n, bool)
    for i in range(env.n):
        gid = env.board_offset + i
        t = int(clock[i // 64])
        u = O.philox([t & 0xFFFFFFFF, t >> 32, gid & 0xFFFFFFFF, gid >> 32], key)
        out[i] = not (float(u[1]) * (1.0 / 4294967296.0) < eps[i])
    return torch.from_numpy(out).to(DEV)


@pytest.mark.parametrize("n,form", [(1, 0.0), (17, 1.0), (1000, 0.5), (20001, "tensor"),
                                    (65536 + 37, "schedule"), (300001, 0.5)])
def test_conv_forward_greedy_rows(G, n, form):
    """g2048_convnet_forward_greedy writes Q only for the boards whose next step is greedy --
    bitwise forward()'s rows -- and leaves the explorers' rows alone; stepping on it gives the
    same actions, rewards and boards as stepping on the full forward.  n = 300001 gives every
    workgroup 1172 boards: two selection windows, with a partial tile carried between them."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    envs = []
    ep0 = torch.randint(0, 8, (n,), generator=torch.Generator().manual_seed(n), dtype=torch.int32)
    for _ in range(2):
        e = G.VecEnv2048(n, device=DEV, seed=11 + n, board_offset=5 * n)
        e.rollout(25)
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
    m = det_init(make_net("conv", torch.float32, DEV), 0.3)
    full = qnet.forward(m, envs[0].board)
    out = torch.full((n, 4), float("nan"), device=DEV)
    qnet.forward_greedy(m, envs[0], out=out, **kw)
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


def test_conv_forward_greedy_rejects_dense(G):
    from g2048 import qnet
    from g2048.nets import make_net

    env = G.VecEnv2048(64, device=DEV)
    with pytest.raises(ValueError):
        qnet.forward_greedy(make_net("dense64", torch.float32, DEV), env, 0.5)


@pytest.mark.parametrize("n", [1, 777, 65536])
def test_conv_forward_f64_matches_torch(G, n):
    """g2048_convnet_forward_f64 (f64 MFMA) against the float64 torch net (the reference's
    Sequential arithmetic, src/configs/double_dqn_conv.py:19-28) on the same boards, directly and
    through an index vector: 1e-12 relative (the sums run in another order)."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    env = G.VecEnv2048(n, device=DEV, seed=40 + n)
    env.rollout(30)
    m = det_init(make_net("conv", torch.float64, DEV), 0.4)
    F = qnet.ConvForward64(m)
    q = F(env.board)
    with torch.no_grad():
        ref = m(env.encode(torch.float64, conv=True)).reshape(n, 4)
    torch.testing.assert_close(q, ref, rtol=1e-12, atol=1e-12 * float(ref.abs().max()))
    idx = torch.randint(0, n, (333,), device=DEV)
    torch.testing.assert_close(F(env.board, idx), q[idx], rtol=0, atol=0)


@pytest.mark.parametrize("n,form", [(4096, 0.5), (300001, "schedule")])
def test_conv_forward_greedy_f64_rows(G, n, form):
    """g2048_convnet_forward_greedy_f64 writes Q only for the boards whose next step is greedy --
    bitwise the full f64 forward's rows -- and stepping on it equals stepping on the full Q."""
    from g2048 import qnet
    from g2048.nets import det_init, make_net

    envs = []
    ep0 = torch.randint(0, 8, (n,), generator=torch.Generator().manual_seed(n), dtype=torch.int32)
    for _ in range(2):
        e = G.VecEnv2048(n, device=DEV, seed=11 + n, board_offset=5 * n)
        e.rollout(25)
        e.ep[:, 0] = ep0.to(DEV)
        envs.append(e)
    if form == "schedule":
        kw = dict(eps_schedule=(6.0, 0.1))
        eps = np.maximum((6.0 - ep0.numpy().astype(np.float64)) / 6.0, 0.1)
    else:
        kw = dict(epsilon=form)
        eps = np.full(n, float(form))
    m = det_init(make_net("conv", torch.float64, DEV), 0.3)
    F = qnet.ConvForward64(m)
    full = F(envs[0].board)
    out = torch.full((n, 4), float("nan"), dtype=torch.float64, device=DEV)
    F.greedy(envs[0], out=out, **kw)
    g = _greedy_mask(envs[0], eps)
    assert 0 < int(g.sum()) < n
    assert torch.equal(out[g], full[g])
    assert bool(out[~g].isnan().all())
    eps_arg = kw.get("epsilon", 0.0)
    sched = kw.get("eps_schedule")
    a0, r0, d0 = envs[0].step_egreedy(out, eps_arg, eps_schedule=sched)
    a1, r1, d1 = envs[1].step_egreedy(full, eps_arg, eps_schedule=sched)
    assert torch.equal(a0, a1) and torch.equal(r0, r1) and torch.equal(d0, d1)
    assert torch.equal(envs[0].board, envs[1].board)


@pytest.mark.parametrize("net", ["conv", "dense64"])
def test_f64_trainer_graphed_equals_eager(G, net):
    """The float64 training loops (conv: fused greedy forward + eps-greedy step; dense-64: Q in
    the step kernel; both + the fused f64 update) replayed from one hipGraph per iteration equal
    the eager loops bitwise."""
    from g2048.learner import DQNLearner, Trainer

    outs = []
    for graph in (True, False):
        n = 2048
        env = G.VecEnv2048(n, device=DEV, seed=77)
        rb = G.ReplayBuffer(8 * n, device=DEV)
        L = DQNLearner(rb, net=net, dtype=torch.float64, batch_size=512, seed=4,
                       target_sync_every=3)
        T = Trainer(env, rb, L, updates_per_step=1, min_fill=0, eps_decay_episodes=3,
                    graph=graph)
        T.prefill(2)
        for _ in range(12):
            T.step()
        torch.cuda.synchronize()
        outs.append((env.board.clone(), float(L.last_loss),
                     torch.cat([p.detach().reshape(-1) for p in L.model.parameters()])))
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
    assert torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("B", [45, 1000, 8192, 20000])
@pytest.mark.parametrize("with_adam", [True, False])
def test_dense64_one_launch_equals_two_launches(G, B, with_adam, monkeypatch):
    """g2048_dense64_update as ONE launch (G2048_DENSE64_ONE_LAUNCH=1: the last
    workgroups to finish their tiles reduce the slabs, k_mlp_update1) against the two-launch form
    (k_mlp_update ->
    k_mlp_reduce, the default): bitwise the same rows, targets, gradient, loss,
    parameters, Adam moments, target sync and update counter over 5 updates, at grids of 2 (each
    reducer takes several 64-position chunks), 32, 256 and 256 x 3 tiles.  The arrival counters
    are back at zero after every launch and no reducer's wait was capped."""
    import copy

    from g2048.nets import det_init, make_net
    from g2048.optim import FusedAdam
    from g2048.qnet import Dense64Update

    rb = _filled_ring(G, 3 + B % 13)
    on = det_init(make_net("dense64", torch.float32, DEV), 0.4)
    tg0 = det_init(make_net("dense64", torch.float32, DEV), 0.9)
    runs = []
    for two in (False, True):
        if two:
            monkeypatch.delenv("G2048_DENSE64_ONE_LAUNCH", raising=False)
        else:
            monkeypatch.setenv("G2048_DENSE64_ONE_LAUNCH", "1")
        m, tg = copy.deepcopy(on), copy.deepcopy(tg0)
        adam = FusedAdam(list(m.parameters()), lr=1e-2)
        adam.attach_target(list(tg.parameters()), 2)
        upd = Dense64Update(m, tg, B, adam=adam if with_adam else None)
        step = torch.full((1,), 5, dtype=torch.int64, device=DEV)
        got = []
        for _ in range(5):
            io = torch.empty(B, dtype=torch.int64, device=DEV)
            y = torch.empty(B, device=DEV)
            g = torch.full((1348,), float("nan"), device=DEV)
            loss = torch.zeros((), device=DEV)
            upd(rb, io, y, step, 0.8, True, 0x1234, None, grad_out=g, loss_out=loss)
            if not with_adam:
                adam.step(g, step)
            got += [io, y, g, loss]
        torch.cuda.synchronize()
        tail = upd.workspace[upd._grid * 1352 + 2:].view(torch.int32)[:3].cpu()
        assert upd.sync_errors() == 0
        assert tail.tolist() == [0, 0, 0], tail
        got += [torch.cat([p.reshape(-1) for p in m.parameters()]),
                torch.cat([p.reshape(-1) for p in tg.parameters()]),
                adam.exp_avg.clone(), adam.exp_avg_sq.clone(), step.clone()]
        runs.append(got)
    assert int(runs[0][-1]) == 10
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [45, 1000, 8192, 20000])
def test_dense64_f64_one_launch_equals_two_launches(G, B, monkeypatch):
    """The float64 dense-64 update in one launch (G2048_DENSE64_ONE_LAUNCH=1,
    k_dense64_update1_f64) against its two launches: bitwise over 5 Adam-folded updates with target syncs, grids of 1 .. 256 x 2 tiles."""
    import copy

    from g2048.nets import det_init, make_net
    from g2048.qnet import Adam64, Dense64Update64

    rb = _filled_ring(G, 7 + B % 11)
    on = det_init(make_net("dense64", torch.float64, DEV), 0.4)
    tg0 = det_init(make_net("dense64", torch.float64, DEV), 0.9)
    runs = []
    for two in (False, True):
        if two:
            monkeypatch.delenv("G2048_DENSE64_ONE_LAUNCH", raising=False)
        else:
            monkeypatch.setenv("G2048_DENSE64_ONE_LAUNCH", "1")
        m, tg = copy.deepcopy(on), copy.deepcopy(tg0)
        adam = Adam64(list(m.parameters()), lr=1e-2)
        adam.attach_target(list(tg.parameters()), 2)
        upd = Dense64Update64(m, tg, B, adam=adam)
        step = torch.full((1,), 5, dtype=torch.int64, device=DEV)
        got = []
        for _ in range(5):
            io = torch.empty(B, dtype=torch.int64, device=DEV)
            y = torch.empty(B, dtype=torch.float64, device=DEV)
            loss = torch.zeros((), dtype=torch.float64, device=DEV)
            upd(rb, io, y, step, 0.8, True, 0x1234, None, loss_out=loss)
            got += [io, y, loss]
        torch.cuda.synchronize()
        assert upd.sync_errors() == 0
        assert upd.workspace[upd._grid * 1352 + 1:].view(torch.int32)[:3].tolist() == [0, 0, 0]
        got += [torch.cat([p.reshape(-1) for p in m.parameters()]),
                torch.cat([p.reshape(-1) for p in tg.parameters()]),
                adam.exp_avg.clone(), adam.exp_avg_sq.clone(), step.clone()]
        runs.append(got)
    assert int(runs[0][-1]) == 10
    for a, b in zip(*runs):
        assert torch.equal(a, b)
