"""Learner parity against the reference's train_step (tests/golden/learner_<net>.npz).

The fixtures hold the reference's own loss for one B=512 minibatch (dqn_lib.train_step,
src/dqn_lib.py:119-164) with deterministic weights, plus Q-values, Bellman targets, correct-order
gradients and one Adam step.  Tolerance (north star): 1e-6 absolute on loss and Q-values in
float64.  These CPU tests run the learner's torch code on CPU tensors; the GPU versions in
test_learner_gpu.py run the same math after the HIP replay gather."""
import os

import numpy as np
import pytest
import torch

from g2048 import dqn_lib
from g2048.nets import det_init, make_net

NETS = ["conv", "dense", "dense64"]
ATOL = 1e-6


def load(golden_dir, net):
    return np.load(os.path.join(golden_dir, f"learner_{net}.npz"))


def batch(g, device="cpu", dtype=torch.float64):
    idx = g["idx"]
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(device)
    s = t(g["buf_s"][idx]).to(dtype)
    s2 = t(g["buf_s2"][idx]).to(dtype)
    return s, t(g["buf_a"][idx]), t(g["buf_r"][idx]).to(dtype), s2, t(g["buf_d"][idx]).to(dtype)


def nets(net, device="cpu", g=None):
    """The fixture's weights: online phase 0.5, target phase 0.2 (or the fixture's tgt_phase),
    frequency 1.3 (or its init_freq)."""
    freq = float(g["init_freq"]) if g is not None and "init_freq" in g else 1.3
    tph = float(g["tgt_phase"]) if g is not None and "tgt_phase" in g else 0.2
    m = det_init(make_net(net, torch.float64, device), 0.5, freq)
    tg = det_init(make_net(net, torch.float64, device), tph, freq)
    return m, tg


# round 3: the vanilla-DQN branch (src/dqn_lib.py:133-144: y = r + (1-d)*gamma*max_a Q_tgt(s')) on
# weights where it differs from Double DQN on most rows, and dense-ref at BASELINE configs[0]'s
# batch of 5000 (src/configs/double_dqn_dense.py:17)
EXTRA = [("conv_vanilla", "conv", False), ("dense64_vanilla", "dense64", False),
         ("dense_b5000", "dense", True)]


@pytest.mark.parametrize("name,net,double", EXTRA)
def test_vanilla_and_b5000_match_reference(golden_dir, name, net, double):
    g = load(golden_dir, name)
    assert bool(g["use_double_dqn"]) == double if "use_double_dqn" in g else double
    m, tg = nets(net, g=g)
    s, a, r, s2, d = batch(g)
    if net == "conv":
        s, s2 = dqn_lib.extract_samples_conv(s), dqn_lib.extract_samples_conv(s2)
    loss, q, y = dqn_lib.dqn_loss(m, tg, s, a, r, s2, d, float(g["gamma"]), use_double_dqn=double)
    assert abs(float(loss) - float(g["loss_ref"])) <= ATOL + 1e-14 * abs(float(g["loss_ref"]))
    np.testing.assert_allclose(q.detach().numpy(), g["q"], rtol=1e-12, atol=ATOL)
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=1e-12, atol=ATOL)
    if not double:  # the fixture really exercises the vanilla branch
        _, _, y_dbl = dqn_lib.dqn_loss(m, tg, s, a, r, s2, d, float(g["gamma"]), use_double_dqn=True)
        assert (y_dbl.numpy() != g["y"]).mean() > 0.9
    opt = torch.optim.Adam(m.parameters(), lr=float(g["lr"]))
    opt.zero_grad()
    loss.backward()
    grads = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).numpy()
    opt.step()
    after = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()
    if "grads" in g:
        np.testing.assert_allclose(grads, g["grads"], rtol=1e-9, atol=1e-9 * np.abs(g["grads"]).max())
        np.testing.assert_allclose(after, g["params_after"], rtol=1e-12, atol=1e-12)
    else:
        sel = g["grad_sel"]
        np.testing.assert_allclose(grads[sel], g["grads_sampled"], rtol=1e-9,
                                   atol=1e-9 * np.abs(g["grads_sampled"]).max())
        np.testing.assert_allclose(grads.sum(), g["grad_sum"], rtol=1e-9)
        np.testing.assert_allclose(after[sel], g["params_after_sampled"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("net", NETS)
def test_loss_and_q_values_match_reference(golden_dir, net):
    g = load(golden_dir, net)
    m, tg = nets(net)
    s, a, r, s2, d = batch(g)
    if net == "conv":
        s, s2 = dqn_lib.extract_samples_conv(s), dqn_lib.extract_samples_conv(s2)
    loss, q, y = dqn_lib.dqn_loss(m, tg, s, a, r, s2, d, float(g["gamma"]))
    assert abs(float(loss) - float(g["loss_ref"])) <= ATOL + 1e-14 * abs(float(g["loss_ref"]))
    np.testing.assert_allclose(q.detach().numpy(), g["q"], rtol=1e-12, atol=ATOL)
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=1e-12, atol=ATOL)
    with torch.no_grad():
        np.testing.assert_allclose(m(s).numpy(), g["q_on_s"], rtol=1e-12, atol=ATOL)
        np.testing.assert_allclose(m(s2).numpy(), g["q_on_s2"], rtol=1e-12, atol=ATOL)
        np.testing.assert_allclose(tg(s2).numpy(), g["q_tgt_s2"], rtol=1e-12, atol=ATOL)
        assert np.array_equal(torch.argmax(m(s2), 1).numpy(), g["a_star"])


@pytest.mark.parametrize("net", NETS)
def test_gradients_and_adam_step(golden_dir, net):
    g = load(golden_dir, net)
    m, tg = nets(net)
    s, a, r, s2, d = batch(g)
    if net == "conv":
        s, s2 = dqn_lib.extract_samples_conv(s), dqn_lib.extract_samples_conv(s2)
    opt = torch.optim.Adam(m.parameters(), lr=float(g["lr"]))
    opt.zero_grad()
    loss, _, _ = dqn_lib.dqn_loss(m, tg, s, a, r, s2, d, float(g["gamma"]))
    loss.backward()
    grads = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).numpy()
    opt.step()
    after = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()
    if "grads" in g:
        np.testing.assert_allclose(grads, g["grads"], rtol=1e-9, atol=1e-9 * np.abs(g["grads"]).max())
        np.testing.assert_allclose(after, g["params_after"], rtol=1e-12, atol=1e-12)
    else:
        sel = g["grad_sel"]
        np.testing.assert_allclose(grads[sel], g["grads_sampled"], rtol=1e-9,
                                   atol=1e-9 * np.abs(g["grads_sampled"]).max())
        np.testing.assert_allclose(grads.sum(), g["grad_sum"], rtol=1e-9)
        np.testing.assert_allclose((grads * grads).sum(), g["grad_sumsq"], rtol=1e-9)
        np.testing.assert_allclose(after[sel], g["params_after_sampled"], rtol=1e-12, atol=1e-12)


def test_reference_compat_order_is_a_noop(golden_dir):
    """F1: backward -> zero_grad -> step leaves the weights exactly unchanged."""
    g = load(golden_dir, "dense64")
    m, tg = nets("dense64")
    before = [p.detach().clone() for p in m.parameters()]
    s, a, r, s2, d = batch(g)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    loss, _, _ = dqn_lib.dqn_loss(m, tg, s, a, r, s2, d, 0.8)
    loss.backward()
    opt.zero_grad()
    opt.step()
    assert all(torch.equal(p, q) for p, q in zip(m.parameters(), before))


def test_one_hot_matches_reference_semantics():
    t = torch.tensor([0, 3, 1, 1])
    oh = dqn_lib.one_hot(t, 4, "cpu")
    assert oh.dtype == torch.float32 and oh.tolist() == [[1, 0, 0, 0], [0, 0, 0, 1], [0, 1, 0, 0],
                                                         [0, 1, 0, 0]]
    with pytest.raises(AssertionError):
        dqn_lib.one_hot(torch.tensor([4]), 4, "cpu")
    with pytest.raises(AssertionError):
        dqn_lib.one_hot(torch.zeros(2, 2, dtype=torch.int64), 4, "cpu")


def test_conv_net_state_dict_matches_reference_layout():
    from torch import nn
    m = make_net("conv", torch.float64)
    ref = nn.Sequential(nn.Conv2d(1, 64, 2), nn.ReLU(), nn.Conv2d(64, 64, 2), nn.ReLU(),
                        nn.Flatten(), nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 4)).double()
    assert [(k, v.shape) for k, v in m.state_dict().items()] == \
           [(k, v.shape) for k, v in ref.state_dict().items()]
    ref.load_state_dict(m.state_dict())
    x = torch.randint(0, 15, (300, 1, 4, 4)).double()
    np.testing.assert_allclose(m(x).detach().numpy(), ref(x).detach().numpy(), rtol=1e-13, atol=1e-12)
    assert sum(p.numel() for p in m.parameters()) == 33476
    assert sum(p.numel() for p in make_net("dense").parameters()) == 403716
    assert sum(p.numel() for p in make_net("dense64").parameters()) == 1348


def test_fused_f64_routing_on_cpu():
    """Which nets the float64 fused kernels take (qnet.kind64_of), and the wrappers' argument
    checks, which fail before any device call: fp32 nets and the dense-ref net are refused."""
    from g2048 import qnet

    conv64, dense64 = make_net("conv", torch.float64, "cpu"), make_net("dense64", torch.float64, "cpu")
    assert qnet.kind64_of(conv64) == "conv" and qnet.kind64_of(dense64) == "dense64"
    assert qnet.kind64_of(make_net("dense", torch.float64, "cpu")) is None
    assert qnet.kind64_of(make_net("conv", torch.float32, "cpu")) is None
    conv32 = make_net("conv", torch.float32, "cpu")
    with pytest.raises(TypeError):
        qnet.ConvUpdate64(conv32, conv32, 512)
    with pytest.raises(TypeError):
        qnet.ConvForward64(conv32)
    with pytest.raises(TypeError):
        qnet.Dense64Update64(conv64, conv64, 512)
    with pytest.raises(ValueError):  # float64 on the CPU: the fused kernels need CUDA tensors
        qnet.ConvUpdate64(conv64, conv64, 512)


def test_trainer_state_version_inference():
    """States written before the version key existed: round 1 (meta [N, 4]) and round 2
    (meta [N, 2] + clock) are told apart by the meta shape."""
    from g2048.learner import _state_version, TRAINER_STATE_VERSION
    assert _state_version({"trainer_state_version": 4}) == TRAINER_STATE_VERSION == 4
    assert _state_version({"trainer_state_version": 3}) == 3
    assert _state_version({"env": {"meta": torch.zeros((5, 4))}}) == 1
    assert _state_version({"env": {"meta": torch.zeros((5, 2))}}) == 2


def test_meta_from_score_moves():
    """A version-3 env meta ({score, moves} per board) as the ABI-v5 rows {score, start}:
    start = group clock - moves (mod 2^32), so clock - start gives the moves back -- also
    across a clock past 2^32 and moves past the clock's low word."""
    from g2048.learner import meta_from_score_moves
    n = 130
    g = torch.Generator().manual_seed(5)
    score = torch.randint(0, 1 << 20, (n,), generator=g, dtype=torch.int64)
    moves = torch.randint(0, 1 << 31, (n,), generator=g, dtype=torch.int64)
    moves[:3] = torch.tensor([0, 1, (1 << 31) + 5])  # a u32 count held in int32
    clock = torch.tensor([7, (1 << 32) + 3, 1 << 40], dtype=torch.int64)
    sm = torch.stack([score, moves], 1)
    sm = torch.where(sm >= 1 << 31, sm - (1 << 32), sm).to(torch.int32)
    m = meta_from_score_moves(sm, clock)
    assert m.shape == (2, n) and m.dtype == torch.int32
    assert torch.equal(m[0], sm[:, 0])
    lo = clock.repeat_interleave(64)[:n] & 0xFFFFFFFF
    back = (lo - (m[1].to(torch.int64) & 0xFFFFFFFF)) & 0xFFFFFFFF
    assert torch.equal(back, sm[:, 1].to(torch.int64) & 0xFFFFFFFF)


def test_board_batch_accessors():
    """BoardBatch answers the Board2048 accessors a reward_function uses (src/board.py:204-231)
    for every board: state (tile values), log_scale().state (exponents), simple_score,
    number_of_empty_cells, merge_score (carried scores; a clear TypeError without them)."""
    b = torch.zeros((3, 16), dtype=torch.uint8)
    b[0, :3] = torch.tensor([1, 2, 17])
    b[2, 15] = 31
    bb = dqn_lib.BoardBatch(b, score=torch.tensor([4, 0, 8]))
    st = bb.state
    assert st.dtype == torch.int64 and st.shape == (3, 4, 4)
    assert st[0, 0, :3].tolist() == [2, 4, 131072] and int(st[2, 3, 3]) == 2 ** 31
    assert torch.equal(bb.log_scale().state.reshape(3, 16), b.long())
    assert bb.simple_score().tolist() == [2 + 4 + 131072, 0, 2 ** 31]
    # Board2048.log_scale().simple_score() sums the exponents (src/board.py:204-205,224-231)
    assert bb.log_scale().simple_score().tolist() == [1 + 2 + 17, 0, 31]
    assert bb.number_of_empty_cells().tolist() == [13, 16, 15]
    assert bb.merge_score().tolist() == [4, 0, 8]
    with pytest.raises(TypeError):
        dqn_lib.BoardBatch(b).merge_score()


def test_split_k_linear_without_bias():
    """nets.Linear(bias=False) (the split-K weight-gradient layer) backpropagates: no gradient
    is returned for the absent bias, and dW / dX match F.linear's."""
    from g2048.nets import Linear

    torch.manual_seed(0)
    lin = Linear(16, 8, bias=False).double()
    x = torch.randn(4096, 16, dtype=torch.float64, requires_grad=True)  # 4096 rows: split-K path
    lin(x).square().sum().backward()
    w2 = lin.weight.detach().clone().requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    torch.nn.functional.linear(x2, w2).square().sum().backward()
    torch.testing.assert_close(lin.weight.grad, w2.grad, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-12, atol=1e-12)
