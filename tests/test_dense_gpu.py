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
    """The reference dense net on the torch path: the Trainer replays ONE captured graph per
    iteration (HIP greedy-branch forward + fused eps-greedy step + the torch update), and 25
    iterations are bitwise those of the same loop computing every board's Q (the boards start at
    mixed episode counts, so eps spans 1 .. min_epsilon)."""
    from g2048 import train
    from test_train_gpu import _fingerprint, _small

    outs = []
    for greedy in (True, False):
        tr = _small(train, "dense", min_fill=3 * 1024, target_sync_every=3, track_boards=0,
                    dtype=getattr(torch, dtype))
        assert tr.graph and tr.learner._dfwd is not None and not tr.learner.fused
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
