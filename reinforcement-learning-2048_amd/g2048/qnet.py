"""Fused Q-network kernels behind the C ABI (csrc/g2048_qnet.hip, g2048_qtrain.hip,
g2048_mlp.hip), for the two fp32 fast-path nets:

  conv     src/configs/double_dqn_conv.py:19-28   (g2048.nets.Conv2048)
  dense64  BASELINE.json configs[2]: 16 -> 64 -> 4 (nn.Sequential(Linear, ReLU, Linear))

forward(model, rows, idx)   == model(board_as_*_tensor(rows[idx]))        one launch
targets(...)                == sampler + Q_online(s') + Q_target(s') + Bellman target, one launch
TrainGrad(model, B)(...)    == d/dtheta sum_b (Q(s_b)[a_b] - y_b)^2 into a flat bucket, 2 launches
Dense64Update(...)()        == a whole dense64 train_step (sampler, targets, gradient, Adam), 2 launches
"""
from __future__ import annotations

import ctypes as C

import torch
from torch import nn

from . import _native as N
from .nets import Conv2048

_CONV_ORDER = ("0.weight", "0.bias", "2.weight", "2.bias", "5.weight", "5.bias", "7.weight",
               "7.bias")
_DENSE_ORDER = ("0.weight", "0.bias", "2.weight", "2.bias")


_DENSE_REF_ORDER = ("0.weight", "0.bias", "2.weight", "2.bias", "4.weight", "4.bias", "6.weight",
                    "6.bias")


def is_dense_ref(model) -> bool:
    """The reference dense net, src/configs/double_dqn_dense.py:7-15: 16-512-512-256-4, ReLUs."""
    dims = [(16, 512), (512, 512), (512, 256), (256, 4)]
    return (isinstance(model, nn.Sequential) and len(model) == 7
            and all(isinstance(model[2 * i], nn.Linear)
                    and (model[2 * i].in_features, model[2 * i].out_features) == d
                    for i, d in enumerate(dims))
            and all(isinstance(model[2 * i + 1], nn.ReLU) for i in range(3)))


class DenseForward:
    """The reference dense net's forward as one HIP launch (g2048_densenet_forward / _greedy):
    Q [n, 4] in the net's dtype (float32 or float64) of board rows, or only of the env boards
    whose next eps-greedy step takes the greedy branch (the rows epsilon_greedy_policy evaluates
    the model on, src/dqn_lib.py:20-24).  Parameter pointers are read at construction."""

    def __init__(self, model):
        if not is_dense_ref(model):
            raise TypeError("DenseForward needs the reference dense net (16-512-512-256-4)")
        dt = next(model.parameters()).dtype
        if dt not in (torch.float32, torch.float64):
            raise TypeError("DenseForward runs float32 or float64 nets")
        self.dtype = dt
        self.code = N.F32 if dt == torch.float32 else N.F64
        self._params = _tensors(model, _DENSE_REF_ORDER, dt)
        self.p = N.DenseNetParams(*[t.data_ptr() for t in self._params])

    def _out(self, n, device, out):
        if out is None:
            return torch.empty((n, 4), dtype=self.dtype, device=device)
        if out.shape != (n, 4) or out.dtype != self.dtype or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous {self.dtype} [{n}, 4] tensor")
        return out

    def __call__(self, rows: torch.Tensor, idx: torch.Tensor | None = None,
                 out: torch.Tensor | None = None) -> torch.Tensor:
        if rows.dtype != torch.uint8 or rows.dim() != 2 or rows.shape[1] != 16 or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous uint8 [*, 16] board tensor")
        if idx is not None and (idx.dtype != torch.int64 or not idx.is_contiguous()):
            raise ValueError("idx must be contiguous int64")
        n = rows.shape[0] if idx is None else idx.numel()
        out = self._out(n, rows.device, out)
        N.check(N.load().g2048_densenet_forward(C.byref(self.p), self.code, N.ptr(rows),
                                                N.ptr(idx), n, N.ptr(out),
                                                N.stream_of(rows.device)),
                "g2048_densenet_forward")
        return out

    def greedy(self, env, epsilon=0.0, eps_schedule=None, out: torch.Tensor | None = None):
        out = self._out(env.n, env.device, out)
        eps_ptr, eps_val, dec, mn = env.eps_args(epsilon, eps_schedule)
        N.check(N.load().g2048_densenet_forward_greedy(
            C.byref(self.p), self.code, env.handle, eps_ptr, eps_val, dec, mn, N.ptr(out),
            N.stream_of(env.device)), "g2048_densenet_forward_greedy")
        return out


def is_dense64(model) -> bool:
    return (isinstance(model, nn.Sequential) and len(model) == 3
            and isinstance(model[0], nn.Linear) and model[0].in_features == 16
            and model[0].out_features == 64 and isinstance(model[1], nn.ReLU)
            and isinstance(model[2], nn.Linear) and model[2].in_features == 64
            and model[2].out_features == 4)


def kind_of(model) -> str | None:
    """'conv' / 'dense64' when a fused fp32 kernel exists for this model, else None."""
    if next(model.parameters()).dtype != torch.float32:
        return None
    if isinstance(model, Conv2048):
        return "conv"
    if is_dense64(model):
        return "dense64"
    return None


def kind64_of(model) -> str | None:
    """'conv' / 'dense64' when a fused float64 update exists for this model, else None."""
    if next(model.parameters()).dtype != torch.float64:
        return None
    if isinstance(model, Conv2048):
        return "conv"
    return "dense64" if is_dense64(model) else None


def update_kind(model) -> str | None:
    """The fused whole-update kernels that take this model: 'conv' / 'dense64' (float32 or
    float64), 'dense' (the reference dense net, g2048_densenet_update, float32 or float64)."""
    k = kind_of(model) or kind64_of(model)
    if k is None and is_dense_ref(model) and next(model.parameters()).dtype in (torch.float32,
                                                                                torch.float64):
        return "dense"
    return k


def _tensors(model, order, dtype=torch.float32):
    sd = dict(model.named_parameters())
    ts = [sd[k] for k in order]
    for t in ts:
        if t.dtype != dtype or not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"fused Q-net kernels run {dtype} contiguous CUDA parameters")
    return ts


def net_params(model):
    """ctypes parameter struct (device pointers) for the model's fused kernels."""
    k = kind_of(model)
    if k == "conv":
        return N.ConvNetParams(*[t.data_ptr() for t in _tensors(model, _CONV_ORDER)])
    if k == "dense64":
        return N.Dense64Params(*[t.data_ptr() for t in _tensors(model, _DENSE_ORDER)])
    raise TypeError("no fused kernel for this model (fp32 Conv2048 or dense 16-64-4 only)")


def _sym(model_or_kind, what):
    k = model_or_kind if isinstance(model_or_kind, str) else kind_of(model_or_kind)
    return getattr(N.load(), f"g2048_{'convnet' if k == 'conv' else 'dense64'}_{what}")


def conv_params(model: Conv2048) -> N.ConvNetParams:
    if not isinstance(model, Conv2048):
        raise TypeError("conv_params needs the reference conv net (g2048.nets.Conv2048)")
    return net_params(model)


def forward(model, rows: torch.Tensor, idx: torch.Tensor | None = None,
            out: torch.Tensor | None = None, params=None):
    """Q-values [n, 4] (fp32) of boards rows[idx] (or rows) -- no autograd."""
    if rows.dtype != torch.uint8 or rows.dim() != 2 or rows.shape[1] != 16 or not rows.is_contiguous():
        raise ValueError("rows must be a contiguous uint8 [*, 16] board tensor")
    n = rows.shape[0] if idx is None else idx.numel()
    if idx is not None and (idx.dtype != torch.int64 or not idx.is_contiguous()):
        raise ValueError("idx must be contiguous int64")
    if out is None:
        out = torch.empty((n, 4), dtype=torch.float32, device=rows.device)
    p = params if params is not None else net_params(model)
    N.check(_sym(model, "forward")(C.byref(p), N.ptr(rows), N.ptr(idx), n, N.ptr(out),
                                   N.stream_of(rows.device)), "fused forward")
    return out


conv_forward = forward


def forward_greedy(model, env, epsilon=0.0, eps_schedule=None, out: torch.Tensor | None = None,
                   params=None):
    """Q-values [n, 4] of env's boards, computed only for the boards whose next eps-greedy step
    (env.step_egreedy with the same epsilon / eps_schedule) takes the greedy branch -- the only
    branch where epsilon_greedy_policy evaluates the model (src/dqn_lib.py:20-24).  Those rows
    are bitwise forward()'s; the other rows of `out` are left as they are.  Conv net only."""
    if kind_of(model) != "conv":
        raise ValueError("forward_greedy: conv net only (the dense-64 step computes Q in-kernel)")
    if out is None:
        out = torch.empty((env.n, 4), dtype=torch.float32, device=env.device)
    if out.shape != (env.n, 4) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous float32 [{env.n}, 4] tensor")
    eps_ptr, eps_val, dec, mn = env.eps_args(epsilon, eps_schedule)
    p = params if params is not None else net_params(model)
    N.check(N.load().g2048_convnet_forward_greedy(C.byref(p), env.handle, eps_ptr, eps_val, dec,
                                                  mn, N.ptr(out), N.stream_of(env.device)),
            "g2048_convnet_forward_greedy")
    return out


CONV64_FWD_WORKSPACE = 53248  # G2048_CONVNET_F64_FWD_WORKSPACE


class ConvForward64:
    """The float64 conv net's forward (g2048_convnet_forward_f64 / _greedy_f64): Q f64 [n, 4]
    of board rows, or only of the env boards whose next eps-greedy step is greedy (the rows
    epsilon_greedy_policy evaluates the model on, src/dqn_lib.py:20-24).  Holds the packed-operand
    workspace; the parameter pointers are read at construction (the tensors keep their storage)."""

    def __init__(self, model):
        if kind64_of(model) != "conv":
            raise TypeError("ConvForward64 needs an fp64 Conv2048")
        self.p = N.ConvNetParams(*[t.data_ptr() for t in
                                   _tensors(model, _CONV_ORDER, torch.float64)])
        self.ws = torch.empty(CONV64_FWD_WORKSPACE, dtype=torch.float64,
                              device=next(model.parameters()).device)

    def __call__(self, rows: torch.Tensor, idx: torch.Tensor | None = None,
                 out: torch.Tensor | None = None) -> torch.Tensor:
        if rows.dtype != torch.uint8 or rows.dim() != 2 or rows.shape[1] != 16 or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous uint8 [*, 16] board tensor")
        if idx is not None and (idx.dtype != torch.int64 or not idx.is_contiguous()):
            raise ValueError("idx must be contiguous int64")
        n = rows.shape[0] if idx is None else idx.numel()
        if out is None:
            out = torch.empty((n, 4), dtype=torch.float64, device=rows.device)
        N.check(N.load().g2048_convnet_forward_f64(C.byref(self.p), N.ptr(rows), N.ptr(idx), n,
                                                   N.ptr(out), N.ptr(self.ws),
                                                   N.stream_of(rows.device)),
                "g2048_convnet_forward_f64")
        return out

    def greedy(self, env, epsilon=0.0, eps_schedule=None, out: torch.Tensor | None = None):
        if out is None:
            out = torch.empty((env.n, 4), dtype=torch.float64, device=env.device)
        if out.shape != (env.n, 4) or out.dtype != torch.float64 or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous float64 [{env.n}, 4] tensor")
        eps_ptr, eps_val, dec, mn = env.eps_args(epsilon, eps_schedule)
        N.check(N.load().g2048_convnet_forward_greedy_f64(
            C.byref(self.p), env.handle, eps_ptr, eps_val, dec, mn, N.ptr(out), N.ptr(self.ws),
            N.stream_of(env.device)), "g2048_convnet_forward_greedy_f64")
        return out


class TrainGrad:
    """Graded half of train_step for a fused net: writes the loss and the gradient of
    sum_b (Q(s_b)[a_b] - y_b)^2 into a flat fp32 buffer laid out like
    torch.cat([p.reshape(-1) for p in model.parameters()]).  For the conv net an `adam`
    (FusedAdam over model.parameters()) folds optimizer.step() -- and its attached target sync --
    into the gradient reduction (g2048_convnet_train_adam; single process only: the gradient is
    final there, with no all-reduce in between)."""

    def __init__(self, model, batch: int, adam=None):
        self.kind = kind_of(model)
        self.params = net_params(model)
        self.batch = int(batch)
        self.n_params = sum(p.numel() for p in model.parameters())
        if adam is not None and self.kind != "conv":
            raise TypeError("the Adam-folded reduction exists for the conv net only")
        self.adam = adam
        self._tparams = None
        if adam is not None and adam.sync_every:
            tps = list(adam._target)  # model.parameters() order == the struct's field order
            if len(tps) != 8:
                raise ValueError("the attached target must be the conv net's 8 tensors")
            self._tparams = N.ConvNetParams(*[t.data_ptr() for t in tps])
        dev = next(model.parameters()).device
        n = _sym(self.kind, "train_workspace")(self.batch)
        self.workspace = torch.empty(n, dtype=torch.float32, device=dev)

    def __call__(self, rows: torch.Tensor, actions: torch.Tensor, idx: torch.Tensor,
                 y: torch.Tensor, grad_out: torch.Tensor | None, loss_out: torch.Tensor | None = None,
                 step: torch.Tensor | None = None):
        if idx.numel() != self.batch or y.numel() != self.batch:
            raise ValueError("idx / y must have `batch` elements")
        if y.dtype != torch.float32 or (grad_out is not None and (
                grad_out.dtype != torch.float32 or grad_out.numel() != self.n_params)):
            raise ValueError(f"y and grad_out must be float32; grad_out has {self.n_params} elements")
        a = self.adam
        if a is None:
            if grad_out is None:
                raise ValueError("without Adam state the gradient needs a grad_out buffer")
            N.check(_sym(self.kind, "train_grad")(
                C.byref(self.params), N.ptr(rows), N.ptr(actions), N.ptr(idx), N.ptr(y), self.batch,
                N.ptr(self.workspace), N.ptr(grad_out), N.ptr(loss_out), N.ptr(step),
                N.stream_of(rows.device)), "fused train_grad")
            return
        if step is None:
            raise ValueError("the Adam-folded update needs the device step counter")
        tp = C.byref(self._tparams) if self._tparams is not None else None
        N.check(N.load().g2048_convnet_train_adam(
            C.byref(self.params), N.ptr(rows), N.ptr(actions), N.ptr(idx), N.ptr(y), self.batch,
            N.ptr(self.workspace), N.ptr(grad_out), N.ptr(loss_out), N.ptr(step),
            N.ptr(a.exp_avg), N.ptr(a.exp_avg_sq), a.lr, a.betas[0], a.betas[1], a.eps, tp,
            int(a.sync_every) if self._tparams is not None else 0, N.stream_of(rows.device)),
            "g2048_convnet_train_adam")


ConvTrainGrad = TrainGrad


class ConvUpdate:
    """One whole Double-DQN update of the fp32 conv net (g2048_convnet_update): targets (sampler,
    both target-side forwards; for Double DQN split over two half-grids that each stage one net)
    and the train launches, then Adam applied in the gradient reduction (adam given) or the
    summed gradient left in grad_out (adam=None).  Same call as Dense64Update."""

    def __init__(self, model, target, batch: int, adam=None):
        if kind_of(model) != "conv" or kind_of(target) != "conv":
            raise TypeError("ConvUpdate needs the conv net for online and target")
        self.on, self.tg = net_params(model), net_params(target)
        self.batch = int(batch)
        self.adam = adam
        dev = next(model.parameters()).device
        n = N.load().g2048_convnet_train_workspace(self.batch)
        self.workspace = torch.empty(n, dtype=torch.float32, device=dev)

    def __call__(self, replay, idx_out, y_out, step_dev, gamma=0.8, double_dqn=True, seed=0,
                 idx_in=None, grad_out=None, loss_out=None):
        if idx_out.numel() != self.batch or y_out.numel() != self.batch:
            raise ValueError("idx_out / y_out must have `batch` elements")
        if self.adam is None and grad_out is None:
            raise ValueError("without Adam state the gradient needs a grad_out buffer")
        a = self.adam
        m, v = (a.exp_avg, a.exp_avg_sq) if a is not None else (None, None)
        lr, b1, b2, eps = (a.lr, a.betas[0], a.betas[1], a.eps) if a is not None else (0, 0, 0, 0)
        N.check(N.load().g2048_convnet_update(
            C.byref(self.on), C.byref(self.tg), replay.handle, N.ptr(idx_in), self.batch,
            int(seed), N.ptr(step_dev), float(gamma), int(bool(double_dqn)), N.ptr(idx_out),
            N.ptr(y_out), N.ptr(self.workspace), N.ptr(grad_out), N.ptr(loss_out), N.ptr(m),
            N.ptr(v), float(lr), float(b1), float(b2), float(eps),
            int(a.sync_every) if a is not None else 0, N.stream_of(y_out.device)),
            "g2048_convnet_update")


class Adam64:
    """Adam state of the fused float64 update (torch Adam semantics, applied inside the
    gradient reduction): flat exp_avg / exp_avg_sq in the parameters' order; attach_target as
    FusedAdam's."""

    def __init__(self, params, lr: float = 1e-2, betas=(0.9, 0.999), eps: float = 1e-8):
        self.params = list(params)
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.exp_avg = torch.zeros(n, dtype=torch.float64, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float64, device=dev)
        self.sync_every = 0

        self._ptrs = (C.c_void_p * len(self.params))(*[p.data_ptr() for p in self.params])
        self._numel = (C.c_int64 * len(self.params))(*[p.numel() for p in self.params])
        self._tptrs = None

    def attach_target(self, target_params, sync_every: int) -> None:
        self._target = list(target_params)
        self._tptrs = (C.c_void_p * len(self._target))(*[t.data_ptr() for t in self._target])
        self.sync_every = int(sync_every)

    def reset_state(self):
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()

    def step(self, grad_flat: torch.Tensor, step_counter: torch.Tensor, grad_scale: float = 1.0):
        """Adam over the flat float64 gradient (the data-parallel path: after the all-reduce);
        step_counter: device u64 holding t; the target sync as attached; the gradient read as
        grad * grad_scale (1 / world after a SUM all-reduce)."""
        lib = N.load()
        args = (self._ptrs, self._numel, len(self.params), N.ptr(grad_flat), N.ptr(self.exp_avg),
                N.ptr(self.exp_avg_sq), N.ptr(step_counter), self.lr, self.betas[0], self.betas[1],
                self.eps, self._tptrs, self.sync_every if self._tptrs is not None else 0)
        if grad_scale == 1.0:
            N.check(lib.g2048_adam_step_sync_f64(*args, N.stream_of(grad_flat.device)),
                    "g2048_adam_step_sync_f64")
        else:
            N.check(lib.g2048_adam_step_scaled_f64(*args, float(grad_scale),
                                                   N.stream_of(grad_flat.device)),
                    "g2048_adam_step_scaled_f64")


class Dense64Update64:
    """One whole Double-DQN update of a float64 dense 16-64-4 net (the reference's precision)
    in two launches (g2048_dense64_update_f64): the same call and step_dev protocol as
    Dense64Update, float64 throughout, Adam (Adam64) applied in the reduction."""

    def __init__(self, model, target, batch: int, adam: Adam64 | None = None):
        if kind64_of(model) != "dense64" or kind64_of(target) != "dense64":
            raise TypeError("Dense64Update64 needs fp64 dense 16-64-4 online and target nets")
        self.on = N.Dense64Params(*[t.data_ptr() for t in
                                    _tensors(model, _DENSE_ORDER, torch.float64)])
        self.tg = N.Dense64Params(*[t.data_ptr() for t in
                                    _tensors(target, _DENSE_ORDER, torch.float64)])
        self.batch = int(batch)
        self.adam = adam
        dev = next(model.parameters()).device
        n = N.load().g2048_dense64_update_f64_workspace(self.batch)
        # zeroed: its tail holds the one-launch update's arrival counters (include/g2048.h)
        self.workspace = torch.zeros(n, dtype=torch.float64, device=dev)
        self._grid = min((self.batch + 63) // 64, 256)

    def sync_errors(self) -> int:
        """As Dense64Update.sync_errors (host sync)."""
        return int(self.workspace[self._grid * 1352 + 1:].view(torch.int32)[2])

    def __call__(self, replay, idx_out, y_out, step_dev, gamma=0.8, double_dqn=True, seed=0,
                 idx_in=None, grad_out=None, loss_out=None):
        if idx_out.numel() != self.batch or y_out.numel() != self.batch:
            raise ValueError("idx_out / y_out must have `batch` elements")
        if y_out.dtype != torch.float64:
            raise TypeError("y_out must be float64")
        if self.adam is None and grad_out is None:
            raise ValueError("without Adam state the gradient needs a grad_out buffer")
        a = self.adam
        m, v = (a.exp_avg, a.exp_avg_sq) if a is not None else (None, None)
        lr, b1, b2, eps = (a.lr, a.betas[0], a.betas[1], a.eps) if a is not None else (0, 0, 0, 0)
        N.check(N.load().g2048_dense64_update_f64(
            C.byref(self.on), C.byref(self.tg), replay.handle, N.ptr(idx_in), self.batch,
            int(seed), N.ptr(step_dev), float(gamma), int(bool(double_dqn)), N.ptr(idx_out),
            N.ptr(y_out), N.ptr(self.workspace), N.ptr(grad_out), N.ptr(loss_out), N.ptr(m),
            N.ptr(v), float(lr), float(b1), float(b2), float(eps),
            int(a.sync_every) if a is not None else 0, N.stream_of(y_out.device)),
            "g2048_dense64_update_f64")


class ConvUpdate64:
    """One whole Double-DQN update of a float64 conv net (the reference's precision) in four
    launches (g2048_convnet_update_f64): targets, two train launches and the reduction with Adam
    (Adam64) applied in place, which also re-packs the weights it writes into the workspace's
    f64-MFMA operand order; the same call and step_dev protocol as Dense64Update64.

    The packed operands must match the weights: they are packed here at construction, and
    ensure_packed() re-packs them when torch changed a parameter of either net since (every
    in-place torch op bumps the tensor's version counter; the fused kernels write through raw
    pointers and keep the packs current themselves).  __call__ runs it outside graph capture;
    graph replays call it first (DQNLearner.update, Trainer)."""

    def __init__(self, model, target, batch: int, adam: Adam64 | None = None):
        if kind64_of(model) != "conv" or kind64_of(target) != "conv":
            raise TypeError("ConvUpdate64 needs fp64 Conv2048 online and target nets")
        self._params = (_tensors(model, _CONV_ORDER, torch.float64)
                        + _tensors(target, _CONV_ORDER, torch.float64))
        self.on = N.ConvNetParams(*[t.data_ptr() for t in self._params[:8]])
        self.tg = N.ConvNetParams(*[t.data_ptr() for t in self._params[8:]])
        self.batch = int(batch)
        self.adam = adam
        dev = next(model.parameters()).device
        n = N.load().g2048_convnet_update_f64_workspace(self.batch)
        self.workspace = torch.empty(n, dtype=torch.float64, device=dev)
        self._packed_at = None
        self.ensure_packed()

    def _versions(self):
        return tuple(t._version for t in self._params)

    def ensure_packed(self, force: bool = False) -> bool:
        """Pack both nets into the workspace if torch modified a parameter since the last pack
        (or force).  Stream-ordered; returns whether it packed.

        Limit: the check keys on tensor version counters, which only torch's in-place ops bump.
        A write that bypasses them -- `p.data.copy_(...)` on a detached alias, a c10d collective
        into parameter storage, another raw-pointer kernel -- leaves the packed operands stale,
        and the update would train on the old conv2 / fc1 weights: call ensure_packed(force=True)
        after any such write.  (The fused kernels of this class keep the packs current
        themselves; the library refuses an Adam update on a workspace never packed, ABI v4.)"""
        v = self._versions()
        if not force and v == self._packed_at:
            return False
        N.check(N.load().g2048_convnet_pack_f64(C.byref(self.on), C.byref(self.tg),
                                                N.ptr(self.workspace),
                                                N.stream_of(self.workspace.device)),
                "g2048_convnet_pack_f64")
        self._packed_at = v
        return True

    def __call__(self, replay, idx_out, y_out, step_dev, gamma=0.8, double_dqn=True, seed=0,
                 idx_in=None, grad_out=None, loss_out=None):
        if idx_out.numel() != self.batch or y_out.numel() != self.batch:
            raise ValueError("idx_out / y_out must have `batch` elements")
        if y_out.dtype != torch.float64:
            raise TypeError("y_out must be float64")
        if self.adam is None and grad_out is None:
            raise ValueError("without Adam state the gradient needs a grad_out buffer")
        if not torch.cuda.is_current_stream_capturing():
            self.ensure_packed()
        a = self.adam
        m, v = (a.exp_avg, a.exp_avg_sq) if a is not None else (None, None)
        lr, b1, b2, eps = (a.lr, a.betas[0], a.betas[1], a.eps) if a is not None else (0, 0, 0, 0)
        N.check(N.load().g2048_convnet_update_f64(
            C.byref(self.on), C.byref(self.tg), replay.handle, N.ptr(idx_in), self.batch,
            int(seed), N.ptr(step_dev), float(gamma), int(bool(double_dqn)), N.ptr(idx_out),
            N.ptr(y_out), N.ptr(self.workspace), N.ptr(grad_out), N.ptr(loss_out), N.ptr(m),
            N.ptr(v), float(lr), float(b1), float(b2), float(eps),
            int(a.sync_every) if a is not None else 0, N.stream_of(y_out.device)),
            "g2048_convnet_update_f64")


class DenseRefUpdate:
    """One whole Double-DQN update of the reference dense net (src/configs/double_dqn_dense.py:
    7-15) in float32 or float64 (g2048_densenet_update): the Philox sampler, the two target-side
    forwards, the row tiles (forward with stored activations, MSE, the input-gradient GEMMs on
    MFMA), the K = B weight-gradient GEMMs and the fixed-order reduction with Adam (FusedAdam /
    Adam64 state; adam=None leaves the summed gradient in grad_out for a data-parallel
    all-reduce).  The same call and step_dev protocol as ConvUpdate64."""

    def __init__(self, model, target, batch: int, adam=None):
        if not (is_dense_ref(model) and is_dense_ref(target)):
            raise TypeError("DenseRefUpdate needs the reference dense net for online and target")
        dt = next(model.parameters()).dtype
        if dt not in (torch.float32, torch.float64):
            raise TypeError("DenseRefUpdate runs float32 or float64 nets")
        self.dtype = dt
        self.code = N.F32 if dt == torch.float32 else N.F64
        self._params = (_tensors(model, _DENSE_REF_ORDER, dt)
                        + _tensors(target, _DENSE_REF_ORDER, dt))
        self.on = N.DenseNetParams(*[t.data_ptr() for t in self._params[:8]])
        self.tg = N.DenseNetParams(*[t.data_ptr() for t in self._params[8:]])
        self.batch = int(batch)
        self.adam = adam
        dev = next(model.parameters()).device
        n = N.load().g2048_densenet_update_workspace(self.batch, self.code)
        self.workspace = torch.empty(n, dtype=dt, device=dev)

    def __call__(self, replay, idx_out, y_out, step_dev, gamma=0.8, double_dqn=True, seed=0,
                 idx_in=None, grad_out=None, loss_out=None):
        if idx_out.numel() != self.batch or y_out.numel() != self.batch:
            raise ValueError("idx_out / y_out must have `batch` elements")
        if y_out.dtype != self.dtype:
            raise TypeError(f"y_out must be {self.dtype}")
        if self.adam is None and grad_out is None:
            raise ValueError("without Adam state the gradient needs a grad_out buffer")
        a = self.adam
        m, v = (a.exp_avg, a.exp_avg_sq) if a is not None else (None, None)
        lr, b1, b2, eps = (a.lr, a.betas[0], a.betas[1], a.eps) if a is not None else (0, 0, 0, 0)
        N.check(N.load().g2048_densenet_update(
            C.byref(self.on), C.byref(self.tg), self.code, replay.handle, N.ptr(idx_in),
            self.batch, int(seed), N.ptr(step_dev), float(gamma), int(bool(double_dqn)),
            N.ptr(idx_out), N.ptr(y_out), N.ptr(self.workspace), N.ptr(grad_out),
            N.ptr(loss_out), N.ptr(m), N.ptr(v), float(lr), float(b1), float(b2), float(eps),
            int(a.sync_every) if a is not None else 0, N.stream_of(y_out.device)),
            "g2048_densenet_update")


class Dense64Update:
    """One whole Double-DQN update of an fp32 dense 16-64-4 net in two launches
    (g2048_dense64_update): sampler + both target-side forwards + Bellman + MSE gradient per
    32-row tile, then the fixed-order gradient reduction with Adam applied in place (adam given)
    or the summed gradient left in grad_out (adam=None, for a data-parallel all-reduce followed by
    FusedAdam.step).  step_dev: device u64 update counter (sampler epoch in, +1 out).  An Adam
    with attach_target(target params, K) also syncs the target net every K-th update."""

    def __init__(self, model, target, batch: int, adam=None):
        if kind_of(model) != "dense64" or kind_of(target) != "dense64":
            raise TypeError("Dense64Update needs fp32 dense 16-64-4 online and target nets")
        self.on, self.tg = net_params(model), net_params(target)
        self.batch = int(batch)
        self.adam = adam
        dev = next(model.parameters()).device
        n = N.load().g2048_dense64_update_workspace(self.batch)
        # zeroed: its tail holds the one-launch update's arrival counters (include/g2048.h)
        self.workspace = torch.zeros(n, dtype=torch.float32, device=dev)
        self._grid = min((self.batch + 31) // 32, 256)

    def sync_errors(self) -> int:
        """Capped waits of the one-launch update's reducers, or launches on a workspace that was
        not zeroed (the tail's error word; host sync).  0 on a healthy device."""
        tail = self.workspace[self._grid * 1352 + 2:].view(torch.int32)
        return int(tail[2])

    def __call__(self, replay, idx_out, y_out, step_dev, gamma=0.8, double_dqn=True, seed=0,
                 idx_in=None, grad_out=None, loss_out=None):
        if idx_out.numel() != self.batch or y_out.numel() != self.batch:
            raise ValueError("idx_out / y_out must have `batch` elements")
        if self.adam is None and grad_out is None:
            raise ValueError("without Adam state the gradient needs a grad_out buffer")
        a = self.adam
        m, v = (a.exp_avg, a.exp_avg_sq) if a is not None else (None, None)
        lr, b1, b2, eps = (a.lr, a.betas[0], a.betas[1], a.eps) if a is not None else (0, 0, 0, 0)
        N.check(N.load().g2048_dense64_update(
            C.byref(self.on), C.byref(self.tg), replay.handle, N.ptr(idx_in), self.batch,
            int(seed), N.ptr(step_dev), float(gamma), int(bool(double_dqn)), N.ptr(idx_out),
            N.ptr(y_out), N.ptr(self.workspace), N.ptr(grad_out), N.ptr(loss_out), N.ptr(m),
            N.ptr(v), float(lr), float(b1), float(b2), float(eps),
            int(a.sync_every) if a is not None else 0, N.stream_of(y_out.device)),
            "g2048_dense64_update")


def targets(kind: str, online, target, replay, batch: int, idx_out: torch.Tensor,
            y_out: torch.Tensor, gamma: float = 0.8, double_dqn: bool = True, seed: int = 0,
            epoch: torch.Tensor | None = None, idx_in: torch.Tensor | None = None):
    """Bellman targets y [B] (fp32) and the sampled ring indices in one launch; epoch is a device
    u64 counter (graph-safe sampler epoch).  online/target: net_params() structs."""
    if idx_in is None and epoch is None:
        raise ValueError("need idx_in or a device epoch counter")
    N.check(_sym(kind, "targets")(
        C.byref(online), C.byref(target), replay.handle, N.ptr(idx_in), int(batch), int(seed),
        N.ptr(epoch), float(gamma), int(bool(double_dqn)), N.ptr(idx_out), N.ptr(y_out),
        N.stream_of(y_out.device)), "fused targets")
    return idx_out, y_out


def conv_targets(online, target, replay, batch, idx_out, y_out, gamma=0.8, double_dqn=True,
                 seed=0, epoch=None, idx_in=None):
    return targets("conv", online, target, replay, batch, idx_out, y_out, gamma, double_dqn,
                   seed, epoch, idx_in)
