"""NaN / Inf guards (SURVEY.md sections 5.2-5.3).

``nonfinite(*losses)`` returns a device fp32 flag (1.0 when any loss is NaN/Inf) with no
host synchronisation, so it can gate ``FusedAdam.step(skip=flag)`` inside a captured
hipGraph: a poisoned step is skipped on the device and counted, never applied.
``check_finite`` is the debug-mode eager check (one sync per call).
"""
from __future__ import annotations

import torch


def nonfinite(*tensors) -> torch.Tensor:
    flag = None
    for t in tensors:
        if t is None:
            continue
        bad = (~torch.isfinite(t.detach().float())).any().float()
        flag = bad if flag is None else torch.maximum(flag, bad)
    return flag


def check_finite(named: dict, where: str = ""):
    bad = [k for k, v in named.items() if isinstance(v, torch.Tensor) and not torch.isfinite(v).all()]
    if bad:
        raise FloatingPointError(f"non-finite values{(' in ' + where) if where else ''}: {bad}")
