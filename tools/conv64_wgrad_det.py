# Run-to-run determinism of the float64 conv update gradients: two GEMM-form learners (G2048_CONV64_WGRAD=gemm)
# from the same state, with a slab-form (or GEMM-form) learner updating in between; prints the differing
# gradient elements per tensor.  Usage: conv64_wgrad_det.py [batch] [slab|gemm]
import os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "reinforcement-learning-2048_amd"))
import g2048 as G
from g2048.learner import DQNLearner
DEV = torch.device("cuda:0")
n = 2048
env = G.VecEnv2048(n, seed=37, device=DEV)
rb = G.ReplayBuffer(16 * n, device=DEV)
env.rollout(16, replay=rb)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 700
inter = sys.argv[2] if len(sys.argv) > 2 else "slab"
Ls = [DQNLearner(rb, net="conv", dtype=torch.float64, batch_size=B, seed=6, target_sync_every=2,
                 graph=False, use_double_dqn=True, data_parallel=True) for _ in range(3)]
def state(L):
    return list(L.model.parameters()) + list(L.target.parameters()) + [L._adam.exp_avg, L._adam.exp_avg_sq, L.step_dev]
bounds = [0, 256, 320, 16704, 16768, 33152, 33216, 33472, 33476]
names = ["w1", "b1", "w2", "b2", "f1", "fb1", "f2", "fb2"]
for it in range(4):
    with torch.no_grad():
        for L in (Ls[0], Ls[2]):
            for x, y in zip(state(L), state(Ls[1])):
                x.copy_(y)
    got = []
    for k, L in enumerate(Ls):
        os.environ["G2048_CONV64_WGRAD"] = "gemm" if k != 1 or inter == "gemm" else "slab"
        L.update()
        torch.cuda.synchronize()
        got.append(L.grad_flat.clone())
    d = (got[0] != got[2]).nonzero().flatten().cpu()
    print("it", it, "diff elements", d.numel(), flush=True)
    for a, b, nm in zip(bounds[:-1], bounds[1:], names):
        m = ((d >= a) & (d < b)).sum().item()
        if m:
            dd = d[(d >= a) & (d < b)]
            print("  ", nm, m, "first", (dd[:8] - a).tolist(), "maxabs", float((got[0][dd] - got[2][dd]).abs().max()))
