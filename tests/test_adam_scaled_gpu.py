"""g2048_adam_step_scaled[_f64]: the Adam step of the data-parallel update under RCCL, where the
gradient bucket holds the SUM over ranks (the all-reduce captured in the update's graph) and Adam
reads it times 1 / world.  ADVICE r5: nothing executed the scaled kernels with a scale != 1 (the
world-1 RCCL test has grad_scale 1).  Here: the scaled step equals the unscaled step
(g2048_adam_step_sync[_f64]) on the gradient pre-scaled by torch, bit for bit, for power-of-two
scales (the worlds 2 / 4 / 8 of the driver's run) and for 1/3, 1/6 (no exact scaling), with the
target sync on and off.  Reference semantics: torch.optim.Adam.step after dividing the averaged
gradient (src/configs/double_dqn_conv.py:39)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    from g2048 import qnet
    from g2048.optim import FusedAdam
    return FusedAdam, qnet.Adam64


def _params(dtype, seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 1, 2, 2), (64,), (64, 64, 2, 2), (64,), (64, 256), (64,), (4, 64), (4,)]
    return [torch.randn(s, generator=g, dtype=torch.float64).to(dtype).to(DEV) for s in shapes]


@pytest.mark.parametrize("sync", [0, 2])
@pytest.mark.parametrize("scale", [1 / 2, 1 / 4, 1 / 8, 1 / 3, 1 / 6])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_scaled_step_equals_unscaled_on_prescaled_grad(mods, dtype, scale, sync):
    FusedAdam, Adam64 = mods
    make = FusedAdam if dtype == torch.float32 else Adam64
    runs = []
    for scaled in (True, False):
        ps = _params(dtype, 1)
        tg = [torch.zeros_like(p) for p in ps]
        opt = make(ps, lr=1e-2)
        if sync:
            opt.attach_target(tg, sync)
        step = torch.zeros(1, dtype=torch.int64, device=DEV)
        gen = torch.Generator(device=DEV).manual_seed(7)
        n = sum(p.numel() for p in ps)
        for _ in range(5):
            g_sum = torch.randn(n, dtype=dtype, device=DEV, generator=gen) * 3.0
            step.add_(1)
            if scaled:
                opt.step(g_sum, step, scale)
            else:  # the mean form: divide by world, then the plain step
                opt.step(g_sum * torch.tensor(scale, dtype=dtype, device=DEV), step)
        torch.cuda.synchronize()
        runs.append((torch.cat([p.reshape(-1) for p in ps]), torch.cat([t.reshape(-1) for t in tg]),
                     opt.exp_avg.clone(), opt.exp_avg_sq.clone()))
    (p0, t0, m0, v0), (p1, t1, m1, v1) = runs
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    assert torch.equal(t0, t1)
    if sync:
        assert torch.count_nonzero(t0) > 0  # t = 2, 4 synced the target


def test_scaled_step_rejects_bad_scale(mods):
    FusedAdam, _ = mods
    from g2048._native import NativeError
    ps = _params(torch.float32, 2)
    opt = FusedAdam(ps)
    step = torch.ones(1, dtype=torch.int64, device=DEV)
    g = torch.zeros(sum(p.numel() for p in ps), device=DEV)
    with pytest.raises(NativeError, match="grad_scale"):
        opt.step(g, step, -0.5)
