"""FusedAdam: torch.optim.Adam semantics in ONE HIP launch over a flat gradient bucket
(csrc/g2048_adam.hip); the step counter lives on the device, so the update is graph-replay safe."""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as N


class FusedAdam:
    def __init__(self, params, lr: float = 1e-2, betas=(0.9, 0.999), eps: float = 1e-8):
        self.params = [p for p in params]
        if len(self.params) > 16:
            raise ValueError("FusedAdam handles at most 16 parameter tensors")
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                raise ValueError("FusedAdam needs contiguous fp32 CUDA parameters")
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self._ptrs = (C.c_void_p * len(self.params))(*[p.data_ptr() for p in self.params])
        self._numel = (C.c_int64 * len(self.params))(*[p.numel() for p in self.params])
        self._tptrs, self.sync_every = None, 0

    def attach_target(self, target_params, sync_every: int) -> None:
        """Also write the updated parameters into target_params whenever the device step
        counter t is a multiple of sync_every (the target-net sync of training_loop, decided
        on the device, so graph replays need no host decision)."""
        tps = [t for t in target_params]
        if len(tps) != len(self.params) or any(t.shape != p.shape or t.dtype != p.dtype
                                               or not t.is_contiguous()
                                               for t, p in zip(tps, self.params)):
            raise ValueError("target params must match the optimised params")
        self._target = tps
        self._tptrs = (C.c_void_p * len(tps))(*[t.data_ptr() for t in tps])
        self.sync_every = int(sync_every)

    def reset_state(self):
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()

    def step(self, grad_flat: torch.Tensor, step_counter: torch.Tensor, grad_scale: float = 1.0):
        """grad_flat: fp32 gradients of self.params packed in order; step_counter: device u64
        holding t (>= 1) for this step's bias correction; grad_scale: the gradient is read as
        grad * grad_scale (1 / world after a SUM all-reduce captured in the same graph)."""
        lib = N.load()
        args = (self._ptrs, self._numel, len(self.params), N.ptr(grad_flat), N.ptr(self.exp_avg),
                N.ptr(self.exp_avg_sq), N.ptr(step_counter), self.lr, self.betas[0], self.betas[1],
                self.eps, self._tptrs, self.sync_every if self._tptrs is not None else 0)
        if grad_scale == 1.0:
            N.check(lib.g2048_adam_step_sync(*args, N.stream_of(grad_flat.device)),
                    "g2048_adam_step_sync")
        else:
            N.check(lib.g2048_adam_step_scaled(*args, float(grad_scale),
                                               N.stream_of(grad_flat.device)),
                    "g2048_adam_step_scaled")
