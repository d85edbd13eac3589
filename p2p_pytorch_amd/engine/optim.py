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
    """Adam whose update is the multi-tensor HIP kernel (``csrc/optim.hip``).

    ``lr`` and the step count live in device tensors, so a step captured into a hipGraph
    keeps following LR schedulers (``param_groups[i]['lr']`` is mirrored into the device
    tensor on every eager ``step`` and by ``sync_lr()``) and bias correction.
    """

    def __init__(self, params, lr=2e-4, betas=(0.5, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        dev = self.param_groups[0]["params"][0].device
        self._lr_t = [torch.tensor([float(g["lr"])], device=dev) for g in self.param_groups]
        self._step_t = [torch.zeros(1, device=dev) for _ in self.param_groups]
        # moments allocated up front (not on first step): the state tensors exist before any
        # warmup, so a graph capture can snapshot and restore them (engine/graph.py); only
        # for trainable parameters (spectral norm's weight_u / weight_v never get a grad)
        for g in self.param_groups:
            for p in g["params"]:
                if p.requires_grad:
                    self._init_state(p)

    def _init_state(self, p):
        st = self.state[p]
        if not st:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        return st

    def sync_lr(self):
        for g, t in zip(self.param_groups, self._lr_t):
            t.fill_(float(g["lr"]))

    @torch.no_grad()
    def step(self, closure=None, skip=None):
        """``skip``: optional device flag (fp32 scalar tensor, non-zero = skip this update,
        e.g. from ``utils.guards.nonfinite``); decided on the device, no host sync."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from ..ops import hip
        capturing = torch.cuda.is_current_stream_capturing()
        for gi, group in enumerate(self.param_groups):
            params, grads, m1, m2 = [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self._init_state(p)
                st["step"] += 1
                params.append(p)
                grads.append(p.grad.contiguous())
                m1.append(st["exp_avg"])
                m2.append(st["exp_avg_sq"])
            if not params:
                continue
            if not capturing:   # lr mirrored into the device tensor (HIP kernel: t = lr)
                hip.P().lincomb_(self._lr_t[gi], None, 0.0, 0.0, float(group["lr"]))
            # step += 1 - skip on the device (HIP kernel)
            hip.P().lincomb_(self._step_t[gi],
                             None if skip is None else skip.reshape(1).float().contiguous(),
                             1.0, -1.0, 1.0)
            b1, b2 = group["betas"]
            hip.adam_(params, grads, m1, m2, self._lr_t[gi], self._step_t[gi], b1, b2,
                      group["eps"], group["weight_decay"],
                      None if skip is None else skip.reshape(1).float().contiguous())
        return loss

    def state_dict(self):
        sd = super().state_dict()
        sd["device_step"] = [float(t.item()) for t in self._step_t]
        return sd

    def load_state_dict(self, sd):
        steps = sd.get("device_step")
        sd = {k: v for k, v in sd.items() if k != "device_step"}
        super().load_state_dict(sd)
        if steps:
            for t, v in zip(self._step_t, steps):
                t.fill_(v)


def guarded_step(opt, reducer, skipped, *losses):
    """Optimizer step behind the NaN/Inf guard: a non-finite loss skips the update on the
    device (FusedAdam: no host sync; agreed across ranks by a 4-byte MAX all-reduce) and is
    added to the ``skipped`` device counter, which is returned (created on first use)."""
    from ..utils.guards import nonfinite
    agree = reducer is not None and reducer.comm and reducer.world > 1
    if skipped is None:
        skipped = torch.zeros((), device=losses[0].device)
    if not agree:
        flag = nonfinite(*losses, counter=skipped)     # flag + count in one launch
    else:
        flag = nonfinite(*losses)
        reducer.all_reduce_max_(flag)
        skipped.add_(flag)
    if isinstance(opt, FusedAdam):
        opt.step(skip=flag)
    elif float(flag) == 0.0:   # stock optimizer: host decision (eager baseline / CPU)
        opt.step()
    return skipped


def make_adam(params, lr=2e-4, betas=(0.5, 0.999), eps=1e-8):
    params = [p for p in params]
    on_gpu = bool(params) and params[0].is_cuda
    if on_gpu and _native.get_backend() == "native":
        _native.ops()  # fail loudly if the extension is missing
        return FusedAdam(params, lr=lr, betas=betas, eps=eps)
    return torch.optim.Adam(params, lr=lr, betas=betas, eps=eps)
