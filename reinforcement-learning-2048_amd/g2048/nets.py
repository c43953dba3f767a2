"""Q-networks of the reference configs, state_dict-compatible with them.

conv    src/configs/double_dqn_conv.py:19-28  Conv2d(1,64,2) ReLU Conv2d(64,64,2) ReLU Flatten
                                              Linear(256,64) ReLU Linear(64,4)      (33 476 params)
dense   src/configs/double_dqn_dense.py:7-15  16-512-512-256-4 ReLU MLP              (403 716 params)
dense64 BASELINE.json configs[2]              16-64-4 ReLU MLP                       (1 348 params)

The conv net keeps nn.Conv2d / nn.Linear parameters under the reference's Sequential indices
("0", "2", "5", "7") but runs its forward as three GEMMs on 2x2 patches of the 4x4 board:
conv1 = [B*9, 4] @ [4, 64], conv2 = [B*4, 256] @ [256, 64] (channels-last activations), then
the two Linears on the (C, H, W)-flattened features -- the same arithmetic as the reference's
Sequential, routed to rocBLAS/hipBLASLt instead of tiny-kernel convolutions.
"""
from __future__ import annotations

import math

import torch
from torch import nn
from torch.nn import functional as F


# ------------------------------------------------------------------ split-K weight gradients
# "gemm": bias gradients through the chunked GEMMs (the product path); "sum": torch's dim-0 sum over
# all m rows, the round-3 form -- only tests/test_graph_hazards_gpu.py sets it, to reproduce the
# captured-update failure that form showed
BIAS_GRAD_FORM = "gemm"


def _splits(m: int) -> int:
    """Row-chunk count for a weight gradient over m rows: ~512 rows per chunk, at most 64 chunks,
    a power of two dividing m (1 = no split)."""
    s = 1
    while s < 64 and m % (2 * s) == 0 and m // (2 * s) >= 512:
        s *= 2
    return s


class _LinearSplitK(torch.autograd.Function):
    """y = x W^T + b whose weight gradient dW = dY^T X sums its m rows in `splits` independent
    chunks (one batched GEMM + a fixed-order sum).  dW is a tall-skinny reduction (K = B x
    positions, up to 32 768 rows, into a 64 x 256 output): rocBLAS runs it as one or two
    workgroups walking the whole K (5.7 ms per fp64 conv2 gradient at B = 8192); chunked, every
    CU takes a slice."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t()) if b is not None else x @ w.t()

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gy @ w if ctx.needs_input_grad[0] else None
        m = x.shape[0]
        s = _splits(m)
        gys = gy.reshape(s, m // s, -1)
        if s > 1:
            gw = torch.bmm(gys.transpose(1, 2), x.reshape(s, m // s, -1)).sum(0)
        else:
            gw = gy.t() @ x
        # the bias gradient through the same chunked GEMMs (dY_chunk^T 1) plus the same small
        # sum over chunks as dW, not torch's dim-0 sum over all m rows: in replays of the captured
        # update that reduction returned stale, deterministic garbage for the conv and fc biases
        # (weights' gradients right, eager runs right) once another learner's work ran between
        # the replays (tests/test_learner_gpu.py test_fused_f64_equals_torch_path at B = 4096).
        # (A [1 x m] x [m x n] GEMM was right too, but a poor rocBLAS shape: +0.9 ms per f64
        # dense-ref update.)
        gb = None
        if ctx.needs_input_grad[2]:
            if BIAS_GRAD_FORM == "sum":  # round 3's form: diagnostics only
                gb = gy.sum(0)
            else:
                gb = torch.bmm(gys.transpose(1, 2), gy.new_ones(s, m // s, 1)).sum(0)[:, 0]
        # b is None for a bias-free layer: autograd takes no gradient for a non-tensor input
        return gx, gw, gb


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None) -> torch.Tensor:
    """F.linear over the last dim, with the split-K weight gradient whenever autograd will need
    dW (the torch learner paths: float64, and float32 nets without a fused kernel)."""
    if not torch.is_grad_enabled() or not w.requires_grad:
        return F.linear(x, w, b)
    shp = x.shape
    y = _LinearSplitK.apply(x.reshape(-1, shp[-1]), w, b)
    return y.reshape(*shp[:-1], w.shape[0])


class Linear(nn.Linear):
    """nn.Linear (same parameters / state_dict) whose backward uses the split-K weight gradient
    of `linear`."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)


class Conv2048(nn.Module):
    def __init__(self):
        super().__init__()
        self.add_module("0", nn.Conv2d(1, 64, kernel_size=2))
        self.add_module("2", nn.Conv2d(64, 64, kernel_size=2))
        self.add_module("5", nn.Linear(2 * 2 * 64, 64))
        self.add_module("7", nn.Linear(64, 4))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        c1, c2, l1, l2 = self._modules["0"], self._modules["2"], self._modules["5"], self._modules["7"]
        B = x.shape[0]
        x = x.reshape(B, 4, 4)
        # conv1: 3x3 output positions, patch (kh, kw) flattened like weight[out, 1, kh, kw]
        p1 = x.unfold(1, 2, 1).unfold(2, 2, 1).reshape(B, 9, 4)
        h1 = F.relu(linear(p1, c1.weight.reshape(64, 4), c1.bias))            # [B, 9, 64] (H,W,C)
        h1 = h1.reshape(B, 3, 3, 64)
        # conv2: 2x2 output positions; patch ordered (in, kh, kw) like weight[out, in, kh, kw]
        p2 = h1.unfold(1, 2, 1).unfold(2, 2, 1)                                # [B, 2, 2, 64, kh, kw]
        h2 = F.relu(linear(p2.reshape(B, 4, 256), c2.weight.reshape(64, 256), c2.bias))  # [B,4,64]
        feat = h2.transpose(1, 2).reshape(B, 256)                              # Flatten: (C, H, W)
        return linear(F.relu(linear(feat, l1.weight, l1.bias)), l2.weight, l2.bias)


def conv_net() -> nn.Module:
    return Conv2048()


def dense_net() -> nn.Module:
    return nn.Sequential(Linear(16, 512), nn.ReLU(), Linear(512, 512), nn.ReLU(),
                         Linear(512, 256), nn.ReLU(), Linear(256, 4))


def dense64_net() -> nn.Module:
    return nn.Sequential(Linear(16, 64), nn.ReLU(), Linear(64, 4))


NETS = {"conv": (conv_net, True), "dense": (dense_net, False), "dense64": (dense64_net, False)}


def make_net(kind: str, dtype=torch.float32, device=None) -> nn.Module:
    """Build a reference-architecture Q-net; `conv_input` of NETS[kind] says whether it eats
    [B, 1, 4, 4] (board_as_4d_tensor) or [B, 16] (board_as_flattened_tensor)."""
    if kind not in NETS:
        raise ValueError(f"unknown net {kind!r}; choose from {sorted(NETS)}")
    return NETS[kind][0]().to(dtype=dtype, device=device)


def det_init(model: nn.Module, phase: float, freq: float = 1.3) -> nn.Module:
    """Deterministic weights p.flat[k] = sin(freq k + phase) / sqrt(fan_in) -- the pattern the
    golden learner fixtures were generated with (tests/golden/gen_goldens.py)."""
    with torch.no_grad():
        for p in model.parameters():
            k = torch.arange(p.numel(), dtype=torch.float64)
            fan_in = int(math.prod(p.shape[1:])) if p.dim() > 1 else 4
            p.copy_((torch.sin(freq * k + phase) / math.sqrt(fan_in)).reshape(p.shape).to(p.dtype))
    return model
