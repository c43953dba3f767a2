"""Device-resident Double-DQN learner and vectorised training loop.

DQNLearner.update() is one reference train_step (src/dqn_lib.py:119-164) at batch B:
sample (torch RNG on device) -> g2048 gather+encode kernel -> online(s'), target(s') -> Bellman
target -> online(s) -> MSE(sum) -> backward -> [RCCL all_reduce of ONE flat gradient bucket when
data-parallel] -> Adam.  The whole update is one hipGraph replay: under RCCL the SUM all-reduce is
captured with it (Adam reads the gradient times 1 / world, no divide launch); over gloo, which runs
on the host, the collective sits between two replays.

Trainer is the vectorised training_loop (src/dqn_lib.py:167-244): every iteration steps all N
boards once with the fused epsilon-greedy kernel (Q from the same online net) and runs
`updates_per_step` learner updates; the epsilon schedule, target sync and episode statistics
stay on the device.
"""
from __future__ import annotations

import copy

import torch

from . import dqn_lib
from .dist import (FlatGradBucket, broadcast_params, captures_collectives, graph_capture,
                   quiesce_for_capture, world_size)
from .env import ReplayBuffer, VecEnv2048
from .nets import NETS, make_net
from . import qnet
from .optim import FusedAdam

# Trainer.state_dict layout (experiment.py wraps it in its own file format tag).  Versions:
#   1 (round 1): env meta [N, 4], no clock;
#   2 (round 2): meta [N, 2] + a per-wave clock, ABI-v2 random-policy draws (no version key was
#                written then; load_state_dict infers 1 / 2 from the meta shape);
#   3: the layout of 2 with the ABI-v3 random policy (include/g2048.h), whose draws differ;
#   4 (ABI v5): env meta [2, N] = {score row, episode-start clock row}; a version-3 state is read
#     by converting its {score, moves} pairs (start = clock - moves).
TRAINER_STATE_VERSION = 4
_STATE_LAYOUTS = {1: "env meta [N, 4], no step clock", 2: "env meta [N, 2] + per-wave clock, ABI-v2 "
                  "random-policy draws", 3: "env meta [N, 2] + per-wave clock, ABI-v3 random-policy "
                  "draws", 4: "env meta [2, N] {score, episode start} + per-wave clock, ABI-v3 "
                  "random-policy draws"}
_READABLE = (3, 4)


def meta_from_score_moves(sm: torch.Tensor, clock: torch.Tensor) -> torch.Tensor:
    """A version-3 env meta ([N, 2] {score, moves}, int32) as the v4 rows [2, N] {score, start}:
    start = (the board's group clock - moves) mod 2^32, stored as int32."""
    n = sm.shape[0]
    lo = clock.to(torch.int64).repeat_interleave(64)[:n] & 0xFFFFFFFF
    start = (lo - (sm[:, 1].to(torch.int64) & 0xFFFFFFFF)) & 0xFFFFFFFF
    start = torch.where(start >= 1 << 31, start - (1 << 32), start).to(torch.int32)
    return torch.stack([sm[:, 0].to(torch.int32), start])


def _state_version(st: dict) -> int:
    if "trainer_state_version" in st:
        return int(st["trainer_state_version"])
    meta = st.get("env", {}).get("meta")
    return 1 if meta is not None and meta.shape[-1] == 4 else 2


class DQNLearner:
    def __init__(self, replay: ReplayBuffer, net: str = "conv", dtype=torch.float32,
                 batch_size: int = 8192, discount_factor: float = 0.8, lr: float = 1e-2,
                 use_double_dqn: bool = True, target_sync_every: int = 100, graph: bool = True,
                 seed: int = 0, model: torch.nn.Module | None = None,
                 process_group=None, sampler=None, loss_fn=None,
                 data_parallel: bool | None = None):
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
        # loss_fn(q, y) of train_step (src/dqn_lib.py:158): None / MSELoss(sum) -- the configs'
        # loss, which the fused kernels implement; any other loss runs the torch path
        self.loss_fn = None if dqn_lib.is_mse_sum(loss_fn) else loss_fn
        self.world = world_size(process_group)
        # data-parallel: gradient-only updates, the bucket all-reduced, then Adam.  Default: world
        # > 1; data_parallel=True forces it at world 1 (the captured collective is tested on one
        # GPU with a world-1 RCCL group)
        self.dp = self.world > 1 if data_parallel is None else bool(data_parallel)
        # RCCL: the SUM all-reduce captured into the update's graph, 1 / world folded into Adam
        self.capture_collective = self.dp and captures_collectives(process_group)
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
        if self.capture_collective:
            # RCCL sets a communicator up on its first collective, which must not happen inside
            # a graph capture: one eager all-reduce of the (zero) bucket now
            self.bucket.allreduce_sum_(process_group)
        params = self.bucket.params
        self.updates = 0
        # Adam on the device: torch's Adam update in ONE HIP launch over the flat gradient bucket
        # (FusedAdam fp32 / Adam64 fp64, csrc/g2048_adam.hip), t and the target sync on the device
        # update counter -- on the fused paths and on the torch path alike (torch's foreach Adam
        # is ~8 multi_tensor_apply launches per step: 40-70 us of the dense-ref update).  torch
        # Adam remains only for models the one-launch kernel cannot take (> 16 tensors, mixed
        # dtypes, not on a GPU).
        self.opt = None
        self._adam = None
        self.step_dev = None
        if self.device.type == "cuda" and len(params) <= 16 and all(
                p.dtype == dtype and p.is_contiguous() for p in params) and dtype in (
                torch.float32, torch.float64):
            self.step_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._adam = (qnet.Adam64(params, lr=lr) if dtype == torch.float64
                          else FusedAdam(params, lr=lr))
            if self.target_sync_every:
                self._adam.attach_target(list(self.target.parameters()), self.target_sync_every)
        else:
            self.opt = torch.optim.Adam(params, lr=lr, capturable=graph, foreach=True)
        self.last_loss = torch.zeros((), dtype=dtype, device=self.device)
        self._graphs = None
        self.graph = graph
        # fused HIP kernels (csrc/g2048_qnet.hip, g2048_qtrain.hip, g2048_mlp.hip) for the fp32
        # conv and dense 16-64-4 nets; other nets / fp64 run the torch path
        # float64 (the reference's precision): the dense 16-64-4 and conv nets have fused
        # updates too (g2048_dense64_update_f64, g2048_convnet_update_f64), and the reference
        # dense net one in both dtypes (g2048_densenet_update); with world > 1 the gradient is
        # all-reduced and the one-launch Adam follows
        self.kind = qnet.update_kind(self.model) if self.loss_fn is None else None
        self.f64 = self.kind is not None and next(self.model.parameters()).dtype == torch.float64
        self.fused = self.kind is not None
        self._upd = None
        # float64 conv: the rollout's Q through the fused forward as well
        self._fwd64 = qnet.ConvForward64(self.model) if self.f64 and self.kind == "conv" else None
        # the reference dense net on the torch path: the rollout's Q through one HIP launch
        # (g2048_densenet_forward[_greedy]) instead of torch's four GEMMs over every board
        self._dfwd = (qnet.DenseForward(self.model)
                      if self.kind in (None, "dense") and self.device.type == "cuda"
                      and qnet.is_dense_ref(self.model) else None)
        # ... and, in float64, the update's two no-grad forwards (Q_online(s'), Q_target(s') of
        # the Bellman target, src/dqn_lib.py:125-144) as the same HIP launch on the sampled s'
        # rows: only Q_online(s) goes through torch autograd (B = 8192: 1.44 -> 1.18 ms per
        # update).  Not in float32: its 64-row tiles put B = 8192 rows on 128 of the 256 CUs,
        # slower than torch's two GEMM forwards (0.74 -> 0.80 ms).
        self._dfwd_tg = (qnet.DenseForward(self.target)
                         if self._dfwd is not None and not self.fused
                         and self.dtype == torch.float64 else None)
        if self.fused:
            small = not self.f64 and self.kind in ("conv", "dense64")
            self._p_on = qnet.net_params(self.model) if small else None
            self._p_tgt = qnet.net_params(self.target) if small else None
            # targets (sampler, both target-side forwards, Bellman), the graded half (forward +
            # MSE + backward) and a fixed-order slab reduction that writes the flat gradient
            # bucket or applies Adam (csrc/g2048_qnet.hip, g2048_qtrain.hip, g2048_mlp.hip).  The
            # device update counter is the sampler epoch and Adam's t (bumped by the train launch);
            # the target sync (every target_sync_every updates) is done by the Adam launch on it:
            # no host decision between graph replays
            assert self._adam is not None
            self._idx = torch.zeros(self.B, dtype=torch.int64, device=self.device)
            self._y = torch.zeros(self.B, dtype=torch.float64 if self.f64 else torch.float32,
                                  device=self.device)
            # one whole update per call; single process: Adam (+ target sync) folded into the
            # gradient reduction.  conv: targets (two half-grids, one net each), train forward,
            # train backward, reduce+Adam = 4 launches; dense64: sampler + targets + gradient in
            # ONE launch + reduce+Adam = 2 launches
            if self.kind == "dense":  # the reference dense net, float32 or float64
                upd = qnet.DenseRefUpdate
            elif self.f64:
                upd = qnet.Dense64Update64 if self.kind == "dense64" else qnet.ConvUpdate64
            else:
                upd = qnet.Dense64Update if self.kind == "dense64" else qnet.ConvUpdate
            self._upd = upd(self.model, self.target, self.B,
                            adam=self._adam if not self.dp else None)
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
            self._upd(self.replay, self._idx, self._y, self.step_dev, self.gamma,
                      self.use_double_dqn, self.sample_seed, idx_in,
                      grad_out=self.grad_flat, loss_out=self.last_loss)
            return
        elif self._dfwd_tg is not None:
            s, a, r, _, d, _ = self.replay.sample_encode(self.B, self.dtype, idx=idx, want_s2=False)
            y = dqn_lib.targets_from_q(self._dfwd(self.replay.s2, idx),
                                       self._dfwd_tg(self.replay.s2, idx), r, d, self.gamma,
                                       self.use_double_dqn)
            q = self.model(self._layout(s)).gather(1, a[:, None])[:, 0]
            loss = ((q - y) ** 2).sum() if self.loss_fn is None else self.loss_fn(q, y)
        else:
            s, a, r, s2, d = dqn_lib.sample_experiences(self.B, self.replay, self.device, None,
                                                        self._layout, dtype=self.dtype, idx=idx)
            loss, _, _ = dqn_lib.dqn_loss(self.model, self.target, s, a, r, s2, d, self.gamma,
                                          self.use_double_dqn, self.loss_fn)
        loss.backward()
        self.last_loss.copy_(loss.detach())

    def _allreduce(self):
        if not self.dp:
            return
        if self.capture_collective:  # SUM; Adam applies 1 / world (grad_scale)
            self.bucket.allreduce_sum_(self.pg)
        else:
            self.bucket.allreduce_mean_(self.pg)

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world if self.capture_collective else 1.0

    def _apply(self):
        if self._upd is not None and self._upd.adam is not None:
            return  # applied inside the update's gradient reduction
        if self._adam is not None:
            if not self.fused:  # the fused train launches bump t themselves
                self.step_dev.add_(1)
            self._adam.step(self.grad_flat, self.step_dev, self.grad_scale)
        else:
            if self.grad_scale != 1.0:  # torch's Adam takes no scale: divide (not captured)
                self.grad_flat.mul_(self.grad_scale)
            self.opt.step()

    def _capture(self):
        # the warm-up below runs real updates; snapshot weights so capture leaves no trace
        params = list(self.model.parameters())
        snap = [p.detach().clone() for p in params]
        tparams = list(self.target.parameters())  # the fused Adam may sync the target
        tsnap = [p.detach().clone() for p in tparams]
        dev_adam = self._adam is not None
        step0 = self.step_dev.clone() if dev_adam else None
        loss0 = self.last_loss.clone()
        rng0 = torch.cuda.get_rng_state(self.device)  # the warm-up draws must not shift the stream
        # optimizer moments too (a resumed learner captures with non-zero Adam state)
        if dev_adam:
            adam0 = (self._adam.exp_avg.clone(), self._adam.exp_avg_sq.clone())
        else:
            adam0 = {p: {k: v.clone() for k, v in st.items() if torch.is_tensor(v)}
                     for p, st in self.opt.state.items()}
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):  # warm-up (allocates Adam state, autograd buffers)
            for _ in range(2):
                self._compute_grads()
                self._allreduce()
                self._apply()
        torch.cuda.current_stream(self.device).wait_stream(side)
        quiesce_for_capture(self.pg)  # the side-stream warm-up (and its collectives) done first
        g1 = torch.cuda.CUDAGraph()
        with graph_capture(g1, self.pg):
            self._compute_grads()
            if not self.dp or self.capture_collective:  # the whole update in one graph
                self._allreduce()
                self._apply()
        g2 = None
        if self.dp and not self.capture_collective:  # gloo: the collective between two replays
            g2 = torch.cuda.CUDAGraph()
            with graph_capture(g2, self.pg):
                self._apply()
        self._graphs = (g1, g2)
        with torch.no_grad():  # restore in place (the graphs hold these addresses)
            for p, s in zip(params, snap):
                p.copy_(s)
            for p, s in zip(tparams, tsnap):
                p.copy_(s)
            for p, st in (self.opt.state.items() if self.opt is not None else ()):
                prev = adam0.get(p, {})
                for k, v in st.items():
                    if torch.is_tensor(v):
                        v.copy_(prev[k]) if k in prev else v.zero_()
            self.grad_flat.zero_()
            self.last_loss.copy_(loss0)
        torch.cuda.set_rng_state(rng0, self.device)
        with torch.no_grad():
            if dev_adam:
                self._adam.exp_avg.copy_(adam0[0])
                self._adam.exp_avg_sq.copy_(adam0[1])
                self.step_dev.copy_(step0)

    def before_replay(self) -> None:
        """Host-side checks a captured update relies on: the float64 conv update's packed weight
        operands must match the weights (re-packed when torch modified a parameter)."""
        if self._upd is not None and hasattr(self._upd, "ensure_packed"):
            self._upd.ensure_packed()

    def update(self) -> torch.Tensor:
        """One Double-DQN update (intended order zero_grad -> backward -> step). Returns the loss
        tensor of this update (device, no sync)."""
        if self.graph:
            if self._graphs is None:
                self._capture()
            self.before_replay()
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
        self.host_target_sync()
        return self.last_loss

    def host_target_sync(self) -> None:
        """The target sync every target_sync_every updates (src/dqn_lib.py:227-228) of a learner
        on torch's Adam, after self.updates was counted; the device Adam (every fused path and the
        torch path on a GPU) syncs on the device update counter instead."""
        if (self._adam is None and self.target_sync_every
                and self.updates % self.target_sync_every == 0):
            dqn_lib.sync_target(self.model, self.target)

    @torch.no_grad()
    def q_values(self, env: VecEnv2048) -> torch.Tensor:
        if self._dfwd is not None:
            return self._dfwd(env.board)
        if self.fused and not self.f64:
            return qnet.forward(self.model, env.board, params=self._p_on)
        if self._fwd64 is not None:
            return self._fwd64(env.board)
        x = env.encode(self.dtype, conv=self.conv_input)
        return self.model(x).reshape(env.n, 4).contiguous()

    # -------------------------------------------------------------- checkpoint / resume
    def state_dict(self) -> dict:
        """Everything an update depends on (tensors cloned to the host)."""
        cpu = lambda t: t.detach().cpu().clone()  # noqa: E731
        st = {"fused": self.fused, "kind": self.kind or "", "dtype": str(self.dtype),
              "batch_size": self.B, "gamma": self.gamma, "double_dqn": self.use_double_dqn,
              "target_sync_every": self.target_sync_every, "updates": self.updates, "last_loss": cpu(self.last_loss),
              "model": {k: cpu(v) for k, v in self.model.state_dict().items()},
              "target": {k: cpu(v) for k, v in self.target.state_dict().items()},
              "cuda_rng": torch.cuda.get_rng_state(self.device)}
        if self._adam is not None:
            st.update(adam_exp_avg=cpu(self._adam.exp_avg), adam_exp_avg_sq=cpu(self._adam.exp_avg_sq),
                      step_dev=cpu(self.step_dev))
            if self.fused:
                st["sample_seed"] = self.sample_seed
        else:
            params = self.bucket.params
            st["adam"] = [{k: cpu(v) for k, v in self.opt.state[p].items() if torch.is_tensor(v)}
                          if p in self.opt.state else {} for p in params]
        return st

    @torch.no_grad()
    def load_state_dict(self, st: dict) -> None:
        """Restore in place: parameter, optimizer and counter tensors keep their addresses, so
        already-captured graphs stay valid."""
        # the reference dense net trained on the torch path up to round 4 (fused False, kind ''):
        # the same parameters and Adam (torch's per-parameter state, converted below), so its
        # checkpoints resume on the fused update; they hold no sampler seed (the torch path drew
        # minibatches with torch's RNG), so this learner's own seed is kept
        torch_path_dense = (not bool(st["fused"]) and st["kind"] == "" and self.kind == "dense"
                            and self.fused)
        if not torch_path_dense and (bool(st["fused"]) != self.fused
                                     or st["kind"] != (self.kind or "")):
            raise ValueError("checkpoint was written by a learner of another net / path")
        for k, v in (("batch_size", self.B), ("gamma", self.gamma), ("double_dqn", self.use_double_dqn),
                     ("dtype", str(self.dtype))):
            if st[k] != v:
                raise ValueError(f"checkpoint {k}={st[k]!r} != this learner's {v!r}")
        for mod, key in ((self.model, "model"), (self.target, "target")):
            cur = mod.state_dict()
            if set(cur) != set(st[key]):
                raise ValueError(f"{key}: parameter names differ from the checkpoint")
            for k, v in cur.items():
                v.copy_(st[key][k])
        self.updates = int(st["updates"])
        self.last_loss.copy_(st["last_loss"])
        torch.cuda.set_rng_state(st["cuda_rng"], self.device)
        if self._adam is not None:
            if "adam_exp_avg" not in st:
                st = dict(st, **_flat_adam_state(st.get("adam", []), self.bucket.params))
            self._adam.exp_avg.copy_(st["adam_exp_avg"])
            self._adam.exp_avg_sq.copy_(st["adam_exp_avg_sq"])
            self.step_dev.copy_(st["step_dev"])
            if self.fused and not torch_path_dense:
                self.sample_seed = int(st["sample_seed"])
        else:
            for p, saved in zip(self.bucket.params, st["adam"]):
                if not saved:
                    continue
                cur = self.opt.state[p]
                for k, v in saved.items():
                    if k in cur and torch.is_tensor(cur[k]):
                        cur[k].copy_(v)
                    else:
                        cur[k] = v.to(p.device) if (k != "step" or self.graph) else v


class Trainer:
    """Vectorised training_loop (src/dqn_lib.py:167-244).

    Per iteration: Q = online(boards) -> fused epsilon-greedy step of all N boards with replay
    append (for the fp32 dense 16-64-4 net, Q is computed inside the step kernel itself; the fused
    conv net evaluates only the boards whose step takes the greedy branch, as
    epsilon_greedy_policy does, src/dqn_lib.py:20-24) ->
    `updates_per_step` learner updates once the ring holds `min_fill` transitions.
    epsilon_b = max((eps_decay_episodes - e_b) / eps_decay_episodes, min_epsilon) with e_b the
    number of episodes board b has finished -- the reference's per-episode schedule (:184-188)
    applied per board inside the fused step kernel.  Every finished episode is appended to the
    env's device episode log by the step kernel itself (add_episode fields, :206-207); the
    first `track_boards` boards also keep a device ring of their last `history_len`
    transitions, from which complete games are cut for snapshot_game (:208-209)."""

    def __init__(self, env: VecEnv2048, replay: ReplayBuffer, learner: DQNLearner,
                 updates_per_step: int = 1, min_fill: int | None = None,
                 eps_decay_episodes: float = 1000.0, min_epsilon: float = 0.01,
                 episode_log_slots: int = 8, track_boards: int = 0,
                 history_len: int = 4096, graph: bool | None = None):
        self.env, self.replay, self.learner = env, replay, learner
        # graph: replay one captured hipGraph per iteration (step + updates) once the learner is
        # updating; default on for the fused learners and for the reference dense net on the
        # torch path (its rollout forward is the HIP g2048_densenet_forward_greedy)
        capturable = learner.fused or (learner._dfwd is not None and learner.sampler is None)
        self.graph = (capturable and learner.graph) if graph is None else bool(graph)
        if self.graph and not capturable:
            raise ValueError("the graphed loop needs a fused learner or the reference dense net")
        if self.graph and not learner.fused and not learner.graph:
            # the torch path's Adam was built capturable=learner.graph: capturing its step would
            # fail at capture time, far from the cause
            raise ValueError("graph=True with a torch-path learner needs DQNLearner(graph=True) "
                             "(its optimizer must be capturable)")
        # Q of the greedy-branch boards only (False: every board; tests compare the two)
        self.greedy_forward = True
        self._loop_graph = None
        self.updates_per_step = int(updates_per_step)
        self.min_fill = int(min_fill if min_fill is not None else learner.B)
        self.eps_decay = float(eps_decay_episodes)
        self.min_eps = float(min_epsilon)
        self.steps = 0
        self.log = env.attach_episode_log(episode_log_slots) if episode_log_slots else None
        self.track = int(min(track_boards, env.n))
        self.history_len = int(history_len)
        if self.track:
            kw = dict(device=env.device)
            self.h_s = torch.zeros((self.history_len, self.track, 16), dtype=torch.uint8, **kw)
            self.h_a = torch.zeros((self.history_len, self.track), dtype=torch.uint8, **kw)
            self.h_r = torch.zeros((self.history_len, self.track), dtype=torch.int32, **kw)
            self.h_d = torch.zeros((self.history_len, self.track), dtype=torch.uint8, **kw)
            self.h_t0 = self.steps  # first trainer step the ring holds
            # per tracked board: its running episode starts inside the window (no moves yet)
            self._clean = (env.moves[:self.track] == 0).cpu().numpy()
        self._action = torch.empty(env.n, dtype=torch.uint8, device=env.device)
        self._reward = torch.empty(env.n, dtype=torch.int32, device=env.device)
        self._done = torch.empty(env.n, dtype=torch.uint8, device=env.device)
        # fused conv learner: Q of the greedy-branch boards only (rows of explorers unused)
        self._q = None
        if learner.fused and learner.kind == "conv":
            self._q = torch.zeros((env.n, 4), dtype=torch.float64 if learner.f64 else torch.float32,
                                  device=env.device)
        elif learner._dfwd is not None:
            self._q = torch.zeros((env.n, 4), dtype=learner._dfwd.dtype, device=env.device)
        self._numbers = {}  # (board, board_episode) -> Experiment episode number

    def prefill(self, steps: int) -> None:
        """Random-policy steps (eps = 1) in one rollout launch, appended to the ring."""
        if self.track:
            raise RuntimeError("prefill before enabling board tracking (histories need every step)")
        self.env.rollout(steps, replay=self.replay)
        self.steps += steps

    def _rollout_step(self) -> None:
        """Device work of play_one_step for all boards (stream-ordered, capturable)."""
        sched = (self.eps_decay, self.min_eps)
        L = self.learner
        if L.kind == "dense64":  # Q inside the step kernel (fp32 or float64)
            self.env.step_egreedy_dense64(L._upd.on if L.f64 else L._p_on, replay=self.replay,
                                          reward=self._reward, done=self._done,
                                          action=self._action, eps_schedule=sched, f64=L.f64)
        else:
            if self._q is not None and L._dfwd is not None:  # reference dense net, HIP forward
                q = (L._dfwd.greedy(self.env, eps_schedule=sched, out=self._q)
                     if self.greedy_forward else L._dfwd(self.env.board, out=self._q))
            elif self._q is not None and self.learner._fwd64 is not None:  # greedy branch only
                q = self.learner._fwd64.greedy(self.env, eps_schedule=sched, out=self._q)
            elif self._q is not None:  # the model runs on the greedy branch only (src/dqn_lib.py:20-24)
                q = qnet.forward_greedy(self.learner.model, self.env, eps_schedule=sched,
                                        out=self._q, params=self.learner._p_on)
            else:
                q = self.learner.q_values(self.env)
            self.env.step_egreedy(q, None, replay=self.replay, reward=self._reward,
                                  done=self._done, action=self._action, eps_schedule=sched)

    def _graphed_iteration(self) -> None:
        """One iteration (step + updates_per_step updates, target syncs included: the fused
        Adam performs them on the device update counter) as ONE hipGraph replay.  Capture
        records without executing, and every kernel of the fused path reads its varying state
        (boards, ring position, update counter) from device memory, so replay k equals eager
        iteration k bit for bit."""
        L = self.learner
        if L.dp and not L.capture_collective:
            return self._graphed_iteration_dp()
        # a learner on torch's Adam syncs its target on the host between updates: one update in
        # the graph, the others through the learner's own graphed update
        ups = self.updates_per_step if L._adam is not None else 1
        if self._loop_graph is None:
            if not L.fused and L._graphs is None:
                L._capture()  # autograd warm-up on a side stream (leaves no trace)
            quiesce_for_capture(L.pg)
            g = torch.cuda.CUDAGraph()
            with graph_capture(g, L.pg):
                self._rollout_step()
                for _ in range(ups):
                    L._compute_grads()
                    L._allreduce()  # data-parallel under RCCL: the SUM all-reduce, captured
                    L._apply()
            self._loop_graph = g
        L.before_replay()
        self._loop_graph.replay()
        for _ in range(ups):
            L.updates += 1
            L.host_target_sync()
        for _ in range(self.updates_per_step - ups):
            L.update()

    def _graphed_iteration_dp(self) -> None:
        """Data-parallel form over a host-side collective (gloo): graph A = the rollout step + the
        first update's gradient, the flat-bucket all-reduce between replays, graph B = Adam (+
        target sync); further updates of the iteration run the learner's own two-graph update.
        (Under RCCL the iteration is ONE graph with the all-reduce captured in it,
        _graphed_iteration.)"""
        L = self.learner
        if self._loop_graph is None:
            if not L.fused and L._graphs is None:
                L._capture()  # autograd warm-up on a side stream (leaves no trace)
            quiesce_for_capture(L.pg)
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with graph_capture(ga, L.pg):
                self._rollout_step()
                L._compute_grads()
            with graph_capture(gb, L.pg):
                L._apply()
            self._loop_graph = (ga, gb)
        ga, gb = self._loop_graph
        L.before_replay()
        ga.replay()
        L._allreduce()
        gb.replay()
        L.updates += 1
        L.host_target_sync()
        for _ in range(self.updates_per_step - 1):
            L.update()

    def step(self) -> None:
        if self.track:
            row = self.steps % self.history_len
            self.h_s[row].copy_(self.env.board[:self.track])
        updating = (self.steps + 1) * self.env.n >= self.min_fill
        if self.graph and updating and self.updates_per_step > 0:
            self._graphed_iteration()
        else:
            self._rollout_step()
        if self.track:
            self.h_a[row].copy_(self._action[:self.track])
            self.h_r[row].copy_(self._reward[:self.track])
            self.h_d[row].copy_(self._done[:self.track])
        self.steps += 1
        if not self.graph and self.steps * self.env.n >= self.min_fill:
            for _ in range(self.updates_per_step):
                self.learner.update()

    # ------------------------------------------------------------------ statistics
    def collect_episodes(self, experiment=None) -> dict:
        """Drain the device episode log (host sync).  With an Experiment, append one reference
        add_episode dict per finished episode (src/experiments.py:112-122)."""
        rec = self.log.read()
        if experiment is not None and rec["step"].numel():
            base = len(experiment.episodes)
            experiment.add_episodes_from_log(rec, self.eps_decay, self.min_eps)
            for j, (b, e) in enumerate(zip(rec["board"].tolist(), rec["episode"].tolist())):
                self._numbers[(b, e)] = base + j
        return rec

    def game_histories(self) -> list:
        """Complete games of the tracked boards still inside the history ring, as
        (board, board_episode, [(state int64[4,4], 'u'|'d'|'l'|'r', reward), ...]) --
        the board_history of src/dqn_lib.py:196-199."""
        from .experiment import ACTION_LETTERS, real_state
        if not self.track:
            return []
        T = self.history_len
        lo = max(self.h_t0, self.steps - T)
        rows = [t % T for t in range(lo, self.steps)]
        s = self.h_s[rows].cpu().numpy()
        a = self.h_a[rows].cpu().numpy()
        r = self.h_r[rows].cpu().numpy()
        d = self.h_d[rows].cpu().numpy()
        ep = self.env.ep[:self.track, 0].cpu().numpy()
        games = []
        for j in range(self.track):
            ends = [k for k in range(len(rows)) if d[k, j]]
            n_done_after = len(ends)
            # episode index of the first game ending in the window
            first_ep = int(ep[j]) - n_done_after
            start = 0 if (lo == self.h_t0 and self._clean[j]) else None
            for g, k in enumerate(ends):
                if start is not None:
                    hist = [(real_state(s[t, j]), ACTION_LETTERS[int(a[t, j])], int(r[t, j]))
                            for t in range(start, k + 1)]
                    games.append((self.env.board_offset + j, first_ep + g, hist))
                start = k + 1
        return games

    def snapshot_games(self, experiment) -> int:
        """snapshot_game (src/experiments.py:124) of every complete tracked game, named by its
        episode number in the experiment (collect_episodes first)."""
        n = 0
        for b, e, hist in self.game_histories():
            num = self._numbers.get((b, e))
            if num is not None:
                experiment.snapshot_game(hist, num)
                n += 1
        return n

    def episode_stats(self) -> dict:
        """Summary of the last finished episode of every board (host sync)."""
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

    # ------------------------------------------------------------------ checkpoint / resume
    def state_dict(self) -> dict:
        cpu = lambda t: t.detach().cpu().clone()  # noqa: E731
        env, rb = self.env, self.replay
        st = {"trainer_state_version": TRAINER_STATE_VERSION,
              "trainer": {"steps": self.steps, "updates_per_step": self.updates_per_step,
                          "min_fill": self.min_fill, "eps_decay": self.eps_decay,
                          "min_eps": self.min_eps},
              "env": {"n": env.n, "seed": env.seed, "board_offset": env.board_offset,
                      "flags": env.flags, "epoch": env.epoch, "board": cpu(env.board),
                      "meta": cpu(env.meta), "ep": cpu(env.ep), "clock": cpu(env.clock)},
              "replay": {"capacity": rb.capacity, "s": cpu(rb.s), "s2": cpu(rb.s2), "a": cpu(rb.a),
                         "r": cpu(rb.r), "d": cpu(rb.d), "count": cpu(rb.count)},
              "learner": self.learner.state_dict()}
        if self.log is not None:
            st["episode_log"] = {"slots": self.log.slots, "raw": cpu(self.log.raw),
                                 "qsum": cpu(self.log.qsum), "read_ep": cpu(self.log.read_ep),
                                 "ep0": cpu(self.log.ep0)}
        return st

    @torch.no_grad()
    def load_state_dict(self, st: dict) -> None:
        self._loop_graph = None  # host-side env state (the reset epoch) is baked into a capture
        fmt = _state_version(st)
        if fmt not in _READABLE:
            raise ValueError(
                f"trainer state version {fmt} ({_STATE_LAYOUTS.get(fmt, 'unknown layout')}) is not "
                f"readable by this build (version {TRAINER_STATE_VERSION}: "
                f"{_STATE_LAYOUTS[TRAINER_STATE_VERSION]}); resume it with the build that wrote it")
        env, rb = self.env, self.replay
        e = st["env"]
        for k in ("n", "seed", "board_offset", "flags"):
            if e[k] != getattr(env, k):
                raise ValueError(f"checkpoint env {k}={e[k]} != this env's {getattr(env, k)}")
        if st["replay"]["capacity"] != rb.capacity:
            raise ValueError("checkpoint replay capacity differs")
        env.board.copy_(e["board"])
        env.meta.copy_(e["meta"] if fmt == TRAINER_STATE_VERSION
                       else meta_from_score_moves(e["meta"], e["clock"]))
        env.ep.copy_(e["ep"])
        env.clock.copy_(e["clock"])
        env.epoch = e["epoch"]
        for k in ("s", "s2", "a", "r", "d", "count"):
            getattr(rb, k).copy_(st["replay"][k])
        if self.log is not None and "episode_log" in st:
            lg = st["episode_log"]
            if lg["slots"] != self.log.slots:
                raise ValueError("checkpoint episode-log slots differ")
            self.log.raw.copy_(lg["raw"])
            self.log.qsum.copy_(lg["qsum"])
            self.log.read_ep.copy_(lg["read_ep"])
            self.log.ep0.copy_(lg["ep0"])
        t = st["trainer"]
        self.steps = int(t["steps"])
        self.updates_per_step, self.min_fill = int(t["updates_per_step"]), int(t["min_fill"])
        self.eps_decay, self.min_eps = float(t["eps_decay"]), float(t["min_eps"])
        self.learner.load_state_dict(st["learner"])
        if self.track:
            self.h_t0 = self.steps
            self._clean = (env.moves[:self.track] == 0).cpu().numpy()


def _flat_adam_state(per_param: list, params) -> dict:
    """A torch-Adam checkpoint of the torch path (round 4: one {step, exp_avg, exp_avg_sq} dict per
    parameter, or {} before the first step) as the device Adam's flat state."""
    if not any(per_param):
        z = torch.zeros(sum(p.numel() for p in params), dtype=params[0].dtype)
        return {"adam_exp_avg": z, "adam_exp_avg_sq": z.clone(),
                "step_dev": torch.zeros(1, dtype=torch.int64)}
    cat = lambda k: torch.cat([d[k].reshape(-1).cpu() for d in per_param])  # noqa: E731
    step = int(float(per_param[0]["step"]))
    return {"adam_exp_avg": cat("exp_avg"), "adam_exp_avg_sq": cat("exp_avg_sq"),
            "step_dev": torch.tensor([step], dtype=torch.int64)}


def flops_per_update(net: str, batch: int) -> float:
    """Algorithmic FLOPs of one update: 3 forwards (online s', target s', online s) + backward of
    the online forward (2x), i.e. 5 forward-equivalents, 2 FLOP per MAC."""
    mac = {"conv": 84480, "dense": 402432, "dense64": 1280}[net]
    return 5.0 * 2.0 * mac * batch

