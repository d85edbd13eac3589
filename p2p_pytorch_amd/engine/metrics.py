"""Evaluation metrics on the device (reference train.py:54-65, :477-482).

The reference moves every test image to the host and runs numpy / skimage; here PSNR and
SSIM are batched tensor reductions on the GPU (no D2H copy until the epoch's means).

Reference-compatible semantics (``ref_compat=True``, the default):
  * images go through ``tensor2np`` first: x * 255 clipped to [0, 255] and rounded down to
    uint8 -- on [-1, 1] data the negative half clips to 0 (quirk A11);
  * PSNR = 10 log10(255^2 / MSE) with MSE over all pixels and channels; an infinite PSNR
    is reported as 60 by the trainer (train.py:480-482);
  * SSIM = skimage ``structural_similarity(x, y, multichannel=True)`` on float arrays:
    7x7 uniform window, K1 = 0.01, K2 = 0.03, sample covariance (N / (N - 1)), mean over the
    valid (un-padded) window positions and channels, and -- because the arrays are float
    with no ``data_range`` -- skimage's float dtype range 2.0 (C1 = (0.01 * 2)^2).
``ref_compat=False`` evaluates the [-1, 1] images mapped to [0, 1] and uses data_range 255.

On the GPU with the native backend both metrics come from ONE HIP kernel
(``csrc/metrics.hip``: exact integer 7x7 window moments, double SSIM ratio, fixed-order
reduction); the tensor code below is the CPU path and the test oracle.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _native


def to_uint8_levels(x: torch.Tensor, ref_compat: bool = True) -> torch.Tensor:
    """[N, C, H, W] model-range tensor -> float tensor holding uint8 levels 0..255."""
    x = x.detach().float()
    if not ref_compat:
        x = (x + 1.0) * 0.5
    return torch.floor((x * 255.0).clamp(0.0, 255.0))


def _native_ok(a: torch.Tensor, b: torch.Tensor, win: int) -> bool:
    return (win == 7 and _native.use_native(a) and a.shape == b.shape and a.dim() == 4
            and a.dtype == b.dtype and a.dtype in (torch.float32, torch.bfloat16)
            and a.shape[2] >= 7 and a.shape[3] >= 7)


def image_metrics(pred: torch.Tensor, ground: torch.Tensor, ref_compat: bool = True,
                  data_range: float | None = None):
    """(psnr [N], ssim [N]) in one pass -- the eval loop's call (train.py:477-478)."""
    if data_range is None:
        data_range = 2.0 if ref_compat else 255.0
    if _native_ok(pred, ground, 7):
        out = _native.ops().image_metrics(pred.detach(), ground.detach(), not ref_compat,
                                          float(data_range))
        return out[:, 0].float(), out[:, 1].float()
    return (_psnr_torch(ground, pred, ref_compat),
            _ssim_torch(pred, ground, ref_compat, 7, data_range))


def psnr(ground: torch.Tensor, pred: torch.Tensor, ref_compat: bool = True) -> torch.Tensor:
    """Per-image PSNR [N] in dB (inf where identical)."""
    if _native_ok(pred, ground, 7):
        return image_metrics(pred, ground, ref_compat)[0]
    return _psnr_torch(ground, pred, ref_compat)


def _psnr_torch(ground: torch.Tensor, pred: torch.Tensor, ref_compat: bool = True) -> torch.Tensor:
    g = to_uint8_levels(ground, ref_compat)
    p = to_uint8_levels(pred, ref_compat)
    mse = ((g - p) ** 2).flatten(1).mean(1)
    return 10.0 * torch.log10(255.0 ** 2 / mse)


def ssim(pred: torch.Tensor, ground: torch.Tensor, ref_compat: bool = True, win: int = 7,
         data_range: float | None = None) -> torch.Tensor:
    """Per-image SSIM [N] (skimage structural_similarity, uniform window)."""
    if _native_ok(pred, ground, win):
        return image_metrics(pred, ground, ref_compat, data_range)[1]
    return _ssim_torch(pred, ground, ref_compat, win, data_range)


def _ssim_torch(pred: torch.Tensor, ground: torch.Tensor, ref_compat: bool = True, win: int = 7,
                data_range: float | None = None) -> torch.Tensor:
    x = to_uint8_levels(pred, ref_compat).double()
    y = to_uint8_levels(ground, ref_compat).double()
    if data_range is None:
        data_range = 2.0 if ref_compat else 255.0
    C1 = (0.01 * data_range) ** 2
    C2 = (0.03 * data_range) ** 2
    n = win * win
    cov_norm = n / (n - 1.0)
    C = x.shape[1]
    k = torch.full((C, 1, win, win), 1.0 / n, dtype=x.dtype, device=x.device)

    def filt(t):  # valid windows only == skimage's filtered image cropped by (win-1)//2
        return F.conv2d(t, k, groups=C)

    ux, uy = filt(x), filt(y)
    uxx, uyy, uxy = filt(x * x), filt(y * y), filt(x * y)
    vx = cov_norm * (uxx - ux * ux)
    vy = cov_norm * (uyy - uy * uy)
    vxy = cov_norm * (uxy - ux * uy)
    a1 = 2 * ux * uy + C1
    a2 = 2 * vxy + C2
    b1 = ux * ux + uy * uy + C1
    b2 = vx + vy + C2
    s = (a1 * a2) / (b1 * b2)
    return s.flatten(1).mean(1).float()
