"""Optimizers.

``FusedAdam`` updates every parameter of a network with ONE multi-tensor HIP kernel
launch per step (fp32 master weights + fp32 moments, chunked tensor-list metadata):
the reference runs ``torch.optim.Adam`` per tensor (127 update sets per step,
/root/reference/train.py:241-243).  CPU parameters (and the eager baseline) use
``torch.optim.Adam`` with identical semantics (Adam, not AdamW; bias-corrected).
"""
from __future__ import annotations

import torch

from .. import _native


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=2e-4, betas=(0.5, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._meta_cache = {}

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        p2p = _native.ops()
        for gi, group in enumerate(self.param_groups):
            params, grads, m1, m2 = [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                params.append(p)
                grads.append(p.grad)
                m1.append(st["exp_avg"])
                m2.append(st["exp_avg_sq"])
            if not params:
                continue
            step = self.state[params[0]]["step"]
            b1, b2 = group["betas"]
            p2p.adam_multi(params, grads, m1, m2, float(group["lr"]), float(b1), float(b2),
                           float(group["eps"]), float(group["weight_decay"]), int(step))
        return loss


def make_adam(params, lr=2e-4, betas=(0.5, 0.999), eps=1e-8):
    params = [p for p in params]
    on_gpu = bool(params) and params[0].is_cuda
    if on_gpu and _native.get_backend() == "native" and _native.available() and \
            hasattr(_native.ops(), "adam_multi"):
        return FusedAdam(params, lr=lr, betas=betas, eps=eps)
    return torch.optim.Adam(params, lr=lr, betas=betas, eps=eps)
