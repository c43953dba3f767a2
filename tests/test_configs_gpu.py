"""BASELINE configs[2] and [3] as the stated workloads: 65 536 boards, a 2^20-transition ring,
B = 8192, Double DQN with the dense 16-64-4 and the conv net (src/configs/double_dqn_conv.py),
through the same Trainer the bench times.  The first update's loss and gradient are checked
against float64 autograd of the reference train_step (src/dqn_lib.py:119-164) on the rows the
fused sampler drew; the graphed loop against the eager one; the episode log against the env's
own counters."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N, RING, B = 65536, 1 << 20, 8192


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    from g2048 import train
    return train


def _trainer(G, net, loop_graph=None, dtype=torch.float32):
    return G.build_trainer(n_boards=N, net=net, dtype=dtype, batch_size=B,
                           replay_buffer_length=RING, min_fill=0, target_sync_every=100, seed=1,
                           device=DEV, track_boards=0, episode_log_slots=8, loop_graph=loop_graph)


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_first_update_matches_fp64_autograd(G, net, dtype):
    """fp32: the fast path within fp32 tolerance (loss 1e-4, per-tensor gradient 1e-3); fp64
    (the reference's precision, the fused float64 kernels): loss and gradient to 1e-9."""
    from g2048 import dqn_lib
    from g2048.nets import make_net

    f64 = dtype == "fp64"
    tr = _trainer(G, net, dtype=torch.float64 if f64 else torch.float32)
    L = tr.learner
    assert L.fused and tr.graph and L.f64 == f64
    tr.prefill(RING // N)
    assert len(tr.replay) == RING
    before = {k: v.detach().clone() for k, v in L.model.state_dict().items()}
    tgt = {k: v.detach().clone() for k, v in L.target.state_dict().items()}
    tr.step()  # the fused eps-greedy step + the first update (one graph replay)
    torch.cuda.synchronize()
    idx = L._idx.clone()
    assert int(idx.min()) >= 0 and int(idx.max()) < RING

    on64, tg64 = make_net(net, torch.float64, DEV), make_net(net, torch.float64, DEV)
    on64.load_state_dict({k: v.double() for k, v in before.items()})
    tg64.load_state_dict({k: v.double() for k, v in tgt.items()})
    rb = tr.replay
    s = rb.s[idx].double()
    s2 = rb.s2[idx].double()
    if net == "conv":
        s, s2 = s.view(B, 1, 4, 4), s2.view(B, 1, 4, 4)
    a, r, d = rb.a[idx].long(), rb.r[idx].double(), rb.d[idx].double()
    loss, _, _ = dqn_lib.dqn_loss(on64, tg64, s, a, r, s2, d, 0.8, True)
    loss.backward()
    ref_g = torch.cat([p.grad.reshape(-1) for p in on64.parameters()])
    got_g = L.grad_flat.double()
    tol_l, tol_g = (1e-9, 1e-9) if f64 else (1e-4, 1e-3)
    assert abs(float(L.last_loss) - float(loss.detach())) <= tol_l * abs(float(loss.detach()))
    off = 0
    for p in on64.parameters():
        k = p.numel()
        gr, gg = ref_g[off:off + k], got_g[off:off + k]
        rel = float((gg - gr).norm() / gr.norm().clamp_min(1e-30))
        assert rel < tol_g, (net, tuple(p.shape), rel)
        off += k


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("net", ["dense64", "conv"])
def test_full_size_graphed_loop_equals_eager(G, net, dtype):
    outs = []
    for graph in (True, False):
        tr = _trainer(G, net, loop_graph=graph,
                      dtype=torch.float64 if dtype == "fp64" else torch.float32)
        tr.env.rollout(100)  # random play first, so that episodes end inside the window
        tr.prefill(RING // N)
        for _ in range(5):
            tr.step()
        torch.cuda.synchronize()
        L = tr.learner
        outs.append({"board": tr.env.board.clone(), "meta": tr.env.meta.clone(),
                     "clock": tr.env.clock.clone(), "ep": tr.env.ep.clone(),
                     "s": tr.replay.s.clone(), "r": tr.replay.r.clone(),
                     "count": tr.replay.count.clone(), "loss": L.last_loss.clone(),
                     "params": torch.cat([p.detach().reshape(-1) for p in L.model.parameters()])})
        assert L.updates == 5 and len(tr.replay) == RING
        # every finished episode is in the log, with the env's own last-episode fields
        ep0 = tr.log.ep0.clone()
        rec = tr.log.read()
        done = tr.env.ep[:, 0].long() - ep0
        assert rec["step"].numel() == int(done.sum()) > 0
        one = (done == 1).nonzero()[:, 0].cpu()
        boards = rec["board"].long()
        pos = {int(b): i for i, b in enumerate(boards.tolist())}
        ep = tr.env.ep.cpu().long()
        for b in one[:200].tolist():
            i = pos[b]
            assert int(rec["score"][i]) == int(ep[b, 1]) and int(rec["moves"][i]) == int(ep[b, 2])
            assert int(rec["max_exp"][i]) == int(ep[b, 3])
    a, b = outs
    for k in a:
        assert torch.equal(a[k], b[k]), (net, k)
