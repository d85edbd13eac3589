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
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def to_uint8_levels(x: torch.Tensor, ref_compat: bool = True) -> torch.Tensor:
    """[N, C, H, W] model-range tensor -> float tensor holding uint8 levels 0..255."""
    x = x.detach().float()
    if not ref_compat:
        x = (x + 1.0) * 0.5
    return torch.floor((x * 255.0).clamp(0.0, 255.0))


def psnr(ground: torch.Tensor, pred: torch.Tensor, ref_compat: bool = True) -> torch.Tensor:
    """Per-image PSNR [N] in dB (inf where identical)."""
    g = to_uint8_levels(ground, ref_compat)
    p = to_uint8_levels(pred, ref_compat)
    mse = ((g - p) ** 2).flatten(1).mean(1)
    return 10.0 * torch.log10(255.0 ** 2 / mse)


def ssim(pred: torch.Tensor, ground: torch.Tensor, ref_compat: bool = True, win: int = 7,
         data_range: float | None = None) -> torch.Tensor:
    """Per-image SSIM [N] (skimage structural_similarity, uniform window)."""
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
