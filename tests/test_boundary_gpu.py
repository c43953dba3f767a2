"""The reference's injected plug points on the GPU path (src/dqn_lib.py:91-97,119,158,167):
a caller's reward_function, board_to_tensor_function and loss_fn are honoured, not ignored."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def g2048():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    return g2048


def test_custom_reward_function(g2048):
    """play_one_step(reward_function=f) calls f(board, next_board, action, done) as the
    reference does (src/dqn_lib.py:104) and stores its rewards in the ring rows."""
    from g2048 import dqn_lib

    n = 3000
    env = g2048.VecEnv2048(n, seed=5, device=DEV)
    rb = g2048.ReplayBuffer(4 * n, device=DEV)

    def empties_after(board, next_board, action, done):  # a shaping reward on the batch
        return (next_board.board == 0).sum(1) - (board.board == 0).sum(1) + 100 * done.long()

    for t in range(6):
        row0 = t % 4 * n
        _, a, r, d, _ = dqn_lib.play_one_step(env, 1.0, None, rb, reward_function=empties_after)
        s, s2 = rb.s[row0:row0 + n], rb.s2[row0:row0 + n]
        want = (s2 == 0).sum(1) - (s == 0).sum(1) + 100 * rb.d[row0:row0 + n].long()
        assert torch.equal(rb.r[row0:row0 + n].long(), want), t
        assert torch.equal(r.long(), want) and torch.equal(rb.a[row0:row0 + n], a)
    with pytest.raises(ValueError):
        dqn_lib.play_one_step(env, 1.0, None, None, reward_function=empties_after)

    # the reference's own reward shape (src/dqn_lib.py:87-88) on the batch: merge scores after -
    # before == the kernel's merge-score reward, and the Board2048 accessors answer per board
    def ref_style(board, next_board, action, done):
        assert board.state.shape == (board.n, 4, 4) and board.log_scale().state.max() < 32
        return next_board.merge_score() - board.merge_score()

    for t in range(5):
        row0 = (6 + t) % 4 * n
        before = env.score.clone().long()
        _, a, r, d, _ = dqn_lib.play_one_step(env, 1.0, None, rb, reward_function=ref_style)
        gain = rb.r[row0:row0 + n].long()
        assert torch.equal(r.long(), gain) and int(gain.sum()) > 0, t
        live = d == 0  # the env re-deals terminal boards (score 0), the ring keeps the transition
        assert torch.equal((before + gain)[live], env.score.long()[live]), t

    def halves(board, next_board, action, done):
        return torch.full((board.n,), 0.5, device=board.device)

    with pytest.raises(TypeError):
        dqn_lib.play_one_step(env, 1.0, None, rb, reward_function=halves)


def test_custom_board_to_tensor_function(g2048):
    """sample_experiences applies a caller's encoder to the sampled boards (src/dqn_lib.py:71-80)
    instead of the fused log2 encode."""
    from g2048 import dqn_lib

    n = 2048
    env = g2048.VecEnv2048(n, seed=6, device=DEV)
    rb = g2048.ReplayBuffer(8 * n, device=DEV)
    env.rollout(8, replay=rb)
    idx = torch.randint(0, 8 * n, (500,), device=DEV)

    def real_values(boards, device, dtype):  # the tile values, not their log2
        e = boards.board.to(torch.int64)
        return torch.where(e > 0, torch.ones_like(e) << e, 0).to(dtype)

    s, a, r, s2, d = dqn_lib.sample_experiences(500, rb, DEV, real_values,
                                                dqn_lib.extract_samples_dense, idx=idx)
    e = rb.s[idx].long()
    assert torch.equal(s, torch.where(e > 0, torch.ones_like(e) << e, 0).double())
    s_ref, *_ = dqn_lib.sample_experiences(500, rb, DEV, dqn_lib.board_as_flattened_tensor,
                                           dqn_lib.extract_samples_dense, idx=idx)
    assert torch.equal(s_ref, rb.s[idx].double())
    assert torch.equal(a, rb.a[idx].long()) and torch.equal(d, rb.d[idx].double())

    def one_hot_tiles(boards, device, dtype):  # an encoding of another shape passes through
        return torch.nn.functional.one_hot(boards.board.long(), 18).to(dtype)

    s, *_ = dqn_lib.sample_experiences(500, rb, DEV, one_hot_tiles,
                                       dqn_lib.extract_samples_dense, idx=idx)
    assert s.shape == (500, 16, 18)


def test_custom_loss_fn(g2048):
    """DQNLearner(loss_fn=...) computes loss_fn(q, y) (src/dqn_lib.py:158); MSELoss(sum) keeps
    the fused kernels, any other loss runs the torch path."""
    from g2048 import dqn_lib
    from g2048.learner import DQNLearner

    n = 1024
    env = g2048.VecEnv2048(n, seed=7, device=DEV)
    rb = g2048.ReplayBuffer(8 * n, device=DEV)
    env.rollout(8, replay=rb)
    fixed = torch.randint(0, 8 * n, (256,), device=DEV)
    assert DQNLearner(rb, net="conv", batch_size=256,
                      loss_fn=torch.nn.MSELoss(reduction="sum")).fused
    huber = torch.nn.SmoothL1Loss(reduction="sum")
    L = DQNLearner(rb, net="conv", batch_size=256, loss_fn=huber, graph=False,
                   sampler=lambda B, replay: fixed)
    assert not L.fused
    sd = {k: v.detach().clone() for k, v in L.model.state_dict().items()}
    L.update()
    s, a, r, s2, d = dqn_lib.sample_experiences(256, rb, DEV, None, dqn_lib.extract_samples_conv,
                                                dtype=torch.float32, idx=fixed)
    from g2048.nets import make_net
    m = make_net("conv", torch.float32, DEV)
    m.load_state_dict(sd)
    want, _, _ = dqn_lib.dqn_loss(m, L.target, s, a, r, s2, d, 0.8, True, huber)
    assert torch.allclose(L.last_loss, want.detach(), rtol=1e-5)
    mse, _, _ = dqn_lib.dqn_loss(m, L.target, s, a, r, s2, d, 0.8, True)
    assert not torch.allclose(want, mse)
