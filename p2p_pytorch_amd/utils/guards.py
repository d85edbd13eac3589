"""NaN / Inf guards (SURVEY.md sections 5.2-5.3).

``nonfinite(*losses)`` returns a device fp32 flag (1.0 when any loss is NaN/Inf) with no
host synchronisation, so it can gate ``FusedAdam.step(skip=flag)`` inside a captured
hipGraph: a poisoned step is skipped on the device and counted, never applied.
``check_finite`` is the debug-mode eager check (one sync per call).
"""
from __future__ import annotations

import torch


def nonfinite(*tensors, counter=None) -> torch.Tensor:
    """fp32 device flag, 1.0 when any of ``tensors`` (loss scalars) is NaN/Inf; with
    ``counter`` (a 0-d fp32 device tensor) also ``counter += flag``.  Native GPU scalars: one
    HIP kernel (csrc/elementwise.hip guard_flag); otherwise torch ops."""
    ts = [t for t in tensors if t is not None]
    if ts and all(t.is_cuda and t.dtype == torch.float32 and t.numel() == 1 for t in ts) \
            and len(ts) <= 8 and (counter is None or counter.dtype == torch.float32):
        from .. import _native
        if _native.get_backend() == "native" and _native.load():
            return _native.ops().guard_flag([t.detach() for t in ts], counter)
    flag = None
    for t in tensors:
        if t is None:
            continue
        bad = (~torch.isfinite(t.detach().float())).any().float()
        flag = bad if flag is None else torch.maximum(flag, bad)
    if counter is not None:
        counter.add_(flag)
    return flag


def check_finite(named: dict, where: str = ""):
    bad = [k for k, v in named.items() if isinstance(v, torch.Tensor) and not torch.isfinite(v).all()]
    if bad:
        raise FloatingPointError(f"non-finite values{(' in ' + where) if where else ''}: {bad}")
