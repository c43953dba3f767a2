"""Device-resident Double-DQN learner and vectorised training loop.

DQNLearner.update() is one reference train_step (src/dqn_lib.py:119-164) at batch B:
sample (torch RNG on device) -> g2048 gather+encode kernel -> online(s'), target(s') -> Bellman
target -> online(s) -> MSE(sum) -> backward -> [RCCL all_reduce of ONE flat gradient bucket when
world > 1] -> Adam.  Everything except the collective is captured into hipGraphs, so an update
costs one (single GPU) or two graph replays plus one all_reduce.

Trainer is the vectorised training_loop (src/dqn_lib.py:167-244): every iteration steps all N
boards once with the fused epsilon-greedy kernel (Q from the same online net) and runs
`updates_per_step` learner updates; the epsilon schedule, target sync and episode statistics
stay on the device.
"""
from __future__ import annotations

import copy

import torch

from . import dqn_lib
from .dist import FlatGradBucket, broadcast_params, world_size
from .env import ReplayBuffer, VecEnv2048
from .nets import NETS, make_net
from . import qnet
from .optim import FusedAdam


class DQNLearner:
    def __init__(self, replay: ReplayBuffer, net: str = "conv", dtype=torch.float32,
                 batch_size: int = 8192, discount_factor: float = 0.8, lr: float = 1e-2,
                 use_double_dqn: bool = True, target_sync_every: int = 100, graph: bool = True,
                 seed: int = 0, model: torch.nn.Module | None = None,
                 process_group=None, sampler=None):
        self.replay = replay
        self.device = replay.device
        self.dtype = dtype
        self.B = int(batch_size)
        self.gamma = float(discount_factor)
        self.use_double_dqn = use_double_dqn
        self.conv_input = NETS[net][1]
        self.target_sync_every = int(target_sync_every)
        self.pg = process_group
        # sampler(B, replay) -> int64 indices on the device; None = uniform with replacement over
        # the filled rows (src/dqn_lib.py:68), drawn by torch's graph-safe device RNG
        self.sampler = sampler
        self.world = world_size(process_group)
        if model is None:
            torch.manual_seed(seed)
            model = make_net(net, dtype=dtype, device=self.device)
        self.model = model
        broadcast_params(self.model, 0, process_group)  # identical init on every rank
        self.target = copy.deepcopy(self.model).requires_grad_(False)
        # one flat gradient bucket; p.grad are views, so the all-reduce is a single collective
        self.bucket = FlatGradBucket(self.model)
        self.grad_flat = self.bucket.flat
        self.n_params = self.bucket.numel
        params = self.bucket.params
        self.opt = torch.optim.Adam(params, lr=lr, capturable=graph, foreach=True)
        self.updates = 0
        self.last_loss = torch.zeros((), dtype=dtype, device=self.device)
        self._graphs = None
        self.graph = graph
        # fused HIP kernels (csrc/g2048_qnet.hip, g2048_qtrain.hip, g2048_mlp.hip) for the fp32
        # conv and dense 16-64-4 nets; other nets / fp64 run the torch path
        self.kind = qnet.kind_of(self.model)
        self.fused = self.kind is not None
        if self.fused:
            self._p_on = qnet.net_params(self.model)
            self._p_tgt = qnet.net_params(self.target)
            # graded half (forward + MSE + backward) as one HIP launch + a slab reduction that
            # writes the flat gradient bucket directly (csrc/g2048_qtrain.hip); targets (sampler,
            # both target-side forwards, Bellman) as one launch; Adam as one launch.  The device
            # update counter is the sampler epoch and Adam's t (bumped by the train launch).
            self._train_grad = qnet.TrainGrad(self.model, self.B)
            self.step_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._idx = torch.zeros(self.B, dtype=torch.int64, device=self.device)
            self._y = torch.zeros(self.B, dtype=torch.float32, device=self.device)
            self._adam = FusedAdam(params, lr=lr)
            rank = torch.distributed.get_rank(process_group) if self.world > 1 else 0
            self.sample_seed = (int(seed) * 0x9E3779B9 + 0x2048 + (rank << 40)) & ((1 << 64) - 1)

    # -------------------------------------------------------------- one train_step, in pieces
    def _layout(self, s):
        return dqn_lib.extract_samples_conv(s) if self.conv_input else dqn_lib.extract_samples_dense(s)

    def _sample_idx(self):
        if self.sampler is not None:
            return self.sampler(self.B, self.replay)
        return (torch.rand(self.B, dtype=torch.float64, device=self.device)
                * self.replay.count.to(torch.float64)).to(torch.int64)

    def _compute_grads(self):
        if not self.fused:
            self.grad_flat.zero_()
        idx = None if self.fused else self._sample_idx()
        if self.fused:
            idx_in = self.sampler(self.B, self.replay) if self.sampler is not None else None
            qnet.targets(self.kind, self._p_on, self._p_tgt, self.replay, self.B, self._idx,
                         self._y, self.gamma, self.use_double_dqn, self.sample_seed, self.step_dev,
                         idx_in)
            self._train_grad(self.replay.s, self.replay.a, self._idx, self._y, self.grad_flat,
                             self.last_loss, self.step_dev)
            return
        else:
            s, a, r, s2, d = dqn_lib.sample_experiences(self.B, self.replay, self.device, None,
                                                        self._layout, dtype=self.dtype, idx=idx)
            loss, _, _ = dqn_lib.dqn_loss(self.model, self.target, s, a, r, s2, d, self.gamma,
                                          self.use_double_dqn)
        loss.backward()
        self.last_loss.copy_(loss.detach())

    def _allreduce(self):
        self.bucket.allreduce_mean_(self.pg)

    def _apply(self):
        if self.fused:
            self._adam.step(self.grad_flat, self.step_dev)
        else:
            self.opt.step()

    def _capture(self):
        # the warm-up below runs real updates; snapshot weights so capture leaves no trace
        params = list(self.model.parameters())
        snap = [p.detach().clone() for p in params]
        step0 = self.step_dev.clone() if self.fused else None
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):  # warm-up (allocates Adam state, autograd buffers)
            for _ in range(2):
                self._compute_grads()
                self._allreduce()
                self._apply()
        torch.cuda.current_stream(self.device).wait_stream(side)
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            self._compute_grads()
            if self.world == 1:
                self._apply()
        g2 = None
        if self.world > 1:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._apply()
        self._graphs = (g1, g2)
        with torch.no_grad():  # restore in place (the graphs hold these addresses)
            for p, s in zip(params, snap):
                p.copy_(s)
            for st in self.opt.state.values():
                for v in st.values():
                    if torch.is_tensor(v):
                        v.zero_()
            self.grad_flat.zero_()
            self.last_loss.zero_()
            if self.fused:
                self._adam.reset_state()
                self.step_dev.copy_(step0)

    def update(self) -> torch.Tensor:
        """One Double-DQN update (intended order zero_grad -> backward -> step). Returns the loss
        tensor of this update (device, no sync)."""
        if self.graph:
            if self._graphs is None:
                self._capture()
            g1, g2 = self._graphs
            g1.replay()
            if g2 is not None:
                self._allreduce()
                g2.replay()
        else:
            self._compute_grads()
            self._allreduce()
            self._apply()
        self.updates += 1
        if self.target_sync_every and self.updates % self.target_sync_every == 0:
            dqn_lib.sync_target(self.model, self.target)
        return self.last_loss

    @torch.no_grad()
    def q_values(self, env: VecEnv2048) -> torch.Tensor:
        if self.fused:
            return qnet.forward(self.model, env.board, params=self._p_on)
        x = env.encode(self.dtype, conv=self.conv_input)
        return self.model(x).reshape(env.n, 4).contiguous()


class Trainer:
    """Vectorised training_loop (src/dqn_lib.py:167-244).

    Per iteration: Q = online(boards) -> fused epsilon-greedy step of all N boards with replay
    append -> `updates_per_step` learner updates once the ring holds `min_fill` transitions.
    epsilon_b = max((eps_decay_episodes - e_b) / eps_decay_episodes, min_epsilon) with e_b the
    number of episodes board b has finished -- the reference's per-episode schedule (:184-188)
    applied per board inside the fused step kernel."""

    def __init__(self, env: VecEnv2048, replay: ReplayBuffer, learner: DQNLearner,
                 updates_per_step: int = 1, min_fill: int | None = None,
                 eps_decay_episodes: float = 1000.0, min_epsilon: float = 0.01):
        self.env, self.replay, self.learner = env, replay, learner
        self.updates_per_step = int(updates_per_step)
        self.min_fill = int(min_fill if min_fill is not None else learner.B)
        self.eps_decay = float(eps_decay_episodes)
        self.min_eps = float(min_epsilon)
        self.steps = 0

    def prefill(self, steps: int) -> None:
        """Random-policy steps (eps = 1) in one rollout launch, appended to the ring."""
        self.env.rollout(steps, replay=self.replay)
        self.steps += steps

    def step(self) -> None:
        q = self.learner.q_values(self.env)
        self.env.step_egreedy(q, None, replay=self.replay,
                              eps_schedule=(self.eps_decay, self.min_eps))
        self.steps += 1
        if self.steps * self.env.n >= self.min_fill:
            for _ in range(self.updates_per_step):
                self.learner.update()

    def episode_stats(self) -> dict:
        """Experiment.add_episode fields (src/experiments.py:112-122) over the last finished
        episode of every board (host sync)."""
        ep = self.env.ep.to(torch.int64)
        fin = ep[:, 0] > 0
        if not bool(fin.any()):
            return {"episodes": 0}
        sel = ep[fin]
        return {"episodes": int(ep[:, 0].sum()),
                "merge_score_mean": float(sel[:, 1].double().mean()),
                "number_moves_mean": float(sel[:, 2].double().mean()),
                "max_tile_max": int(2 ** int(sel[:, 3].max())),
                "max_tile_hist": {int(2 ** int(k)): int(v) for k, v in
                                  zip(*torch.unique(sel[:, 3], return_counts=True))},
                "epsilon_mean": float(self.current_epsilon().mean())}

    def current_epsilon(self) -> torch.Tensor:
        e = self.env.ep[:, 0].to(torch.float64)
        return torch.clamp((self.eps_decay - e) / self.eps_decay, min=self.min_eps)


def flops_per_update(net: str, batch: int) -> float:
    """Algorithmic FLOPs of one update: 3 forwards (online s', target s', online s) + backward of
    the online forward (2x), i.e. 5 forward-equivalents, 2 FLOP per MAC."""
    mac = {"conv": 84480, "dense": 402432, "dense64": 1280}[net]
    return 5.0 * 2.0 * mac * batch

