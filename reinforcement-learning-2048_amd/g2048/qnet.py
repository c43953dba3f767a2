"""Fused Q-network kernels (csrc/g2048_qnet.hip) behind the C ABI.

conv_forward(model, rows, idx) == model(board_as_4d_tensor(rows[idx])) for the reference conv
net (src/configs/double_dqn_conv.py:19-28) in fp32, as ONE launch that reads the u8 boards
(optionally through replay indices) and writes Q [n, 4]."""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as N
from .nets import Conv2048

_ORDER = ("0.weight", "0.bias", "2.weight", "2.bias", "5.weight", "5.bias", "7.weight", "7.bias")


def conv_params(model: Conv2048) -> N.ConvNetParams:
    if not isinstance(model, Conv2048):
        raise TypeError("conv_forward needs the reference conv net (g2048.nets.Conv2048)")
    sd = dict(model.named_parameters())
    ts = [sd[k] for k in _ORDER]
    for t in ts:
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("fused conv net runs fp32 contiguous CUDA parameters")
    return N.ConvNetParams(*[t.data_ptr() for t in ts])


def conv_forward(model: Conv2048, rows: torch.Tensor, idx: torch.Tensor | None = None,
                 out: torch.Tensor | None = None, params: N.ConvNetParams | None = None):
    """Q-values [n, 4] (fp32) of boards rows[idx] (or rows) -- no autograd."""
    if rows.dtype != torch.uint8 or rows.dim() != 2 or rows.shape[1] != 16 or not rows.is_contiguous():
        raise ValueError("rows must be a contiguous uint8 [*, 16] board tensor")
    n = rows.shape[0] if idx is None else idx.numel()
    if idx is not None and (idx.dtype != torch.int64 or not idx.is_contiguous()):
        raise ValueError("idx must be contiguous int64")
    if out is None:
        out = torch.empty((n, 4), dtype=torch.float32, device=rows.device)
    p = params if params is not None else conv_params(model)
    N.check(N.load().g2048_convnet_forward(C.byref(p), N.ptr(rows), N.ptr(idx), n, N.ptr(out),
                                           N.stream_of(rows.device)), "g2048_convnet_forward")
    return out


class ConvTrainGrad:
    """Fused graded half of train_step for the conv net (csrc/g2048_qtrain.hip): writes the loss
    and the gradient of sum_b (Q(s_b)[a_b] - y_b)^2 into a flat fp32 buffer laid out like
    torch.cat([p.reshape(-1) for p in model.parameters()])."""

    def __init__(self, model: Conv2048, batch: int):
        self.params = conv_params(model)
        self.batch = int(batch)
        dev = next(model.parameters()).device
        n = N.load().g2048_convnet_train_workspace(self.batch)
        self.workspace = torch.empty(n, dtype=torch.float32, device=dev)

    def __call__(self, rows: torch.Tensor, actions: torch.Tensor, idx: torch.Tensor,
                 y: torch.Tensor, grad_out: torch.Tensor, loss_out: torch.Tensor | None = None,
                 step: torch.Tensor | None = None):
        if idx.numel() != self.batch or y.numel() != self.batch:
            raise ValueError("idx / y must have `batch` elements")
        if y.dtype != torch.float32 or grad_out.dtype != torch.float32 or grad_out.numel() != 33476:
            raise ValueError("y and grad_out must be float32; grad_out has 33476 elements")
        N.check(N.load().g2048_convnet_train_grad(
            C.byref(self.params), N.ptr(rows), N.ptr(actions), N.ptr(idx), N.ptr(y), self.batch,
            N.ptr(self.workspace), N.ptr(grad_out), N.ptr(loss_out), N.ptr(step),
            N.stream_of(rows.device)),
            "g2048_convnet_train_grad")


def conv_targets(online: N.ConvNetParams, target: N.ConvNetParams, replay, batch: int,
                 idx_out: torch.Tensor, y_out: torch.Tensor, gamma: float = 0.8,
                 double_dqn: bool = True, seed: int = 0, epoch: torch.Tensor | None = None,
                 idx_in: torch.Tensor | None = None):
    """Bellman targets y [B] (fp32) and the sampled ring indices in one launch
    (g2048_convnet_targets); epoch is a device u64 counter (graph-safe sampler epoch)."""
    if idx_in is None and epoch is None:
        raise ValueError("need idx_in or a device epoch counter")
    N.check(N.load().g2048_convnet_targets(
        C.byref(online), C.byref(target), replay.handle, N.ptr(idx_in), int(batch), int(seed),
        N.ptr(epoch), float(gamma), int(bool(double_dqn)), N.ptr(idx_out), N.ptr(y_out),
        N.stream_of(y_out.device)), "g2048_convnet_targets")
    return idx_out, y_out
