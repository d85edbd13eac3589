"""Losses (reference networks.py:808-894 and train.py:123-126).

All are device-agnostic (reference quirk A7: the original hard-codes
``torch.cuda.FloatTensor``) and never materialise constant target tensors: the
fused kernels compute ``mean((x - c)^2)`` / BCE against a scalar label directly.
"""
from __future__ import annotations

from math import pi

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class GANLoss(nn.Module):
    """GAN objective against a constant real/fake label.

    ``gan_mode``: 'lsgan' (MSE, reference default), 'bce' (BCE on probabilities, the
    reference's ``use_lsgan=False``), 'vanilla' (BCE-with-logits, pix2pix default) or
    'wgangp'.  Accepts a single prediction, a list of D features (uses the last) or a
    multiscale list of lists (sums the last feature of each scale, networks.py:841-847).
    """

    def __init__(self, use_lsgan=True, target_real_label=1.0, target_fake_label=0.0, tensor=None,
                 gan_mode=None):
        super().__init__()
        self.real_label = float(target_real_label)
        self.fake_label = float(target_fake_label)
        self.gan_mode = gan_mode or ("lsgan" if use_lsgan else "bce")
        if self.gan_mode not in ("lsgan", "bce", "vanilla", "wgangp"):
            raise NotImplementedError(f"gan mode {self.gan_mode} not implemented")

    def _one(self, pred, is_real):
        t = self.real_label if is_real else self.fake_label
        if self.gan_mode == "lsgan":
            return ops.mse_const(pred, t)
        if self.gan_mode == "vanilla":
            return ops.bce_logits_const(pred, t)
        if self.gan_mode == "bce":
            return ops.bce_const(pred, t)
        return -pred.float().mean() if is_real else pred.float().mean()

    def forward(self, pred, target_is_real):
        if isinstance(pred, (list, tuple)):
            if isinstance(pred[0], (list, tuple)):
                terms = [self._one(p[-1], target_is_real) for p in pred]
                return ops.lincomb_n(terms, [1.0] * len(terms))
            return self._one(pred[-1], target_is_real)
        return self._one(pred, target_is_real)


def calc_tv_Loss(x):
    return ops.tv(x)


class angular_loss(nn.Module):
    """mean(acos(clamp(cos_sim_c(a, b)))) in degrees (networks.py:870-894)."""

    def forward(self, illum_gt, illum_pred):
        cos = F.cosine_similarity(illum_gt.float(), illum_pred.float(), dim=1)
        cos = torch.clamp(cos, -0.99999, 0.99999)
        return torch.mean(torch.acos(cos)) * 180 / pi


_SOBEL_X = torch.tensor([[1.0, 0.0, -1.0], [2.0, 0.0, -2.0], [1.0, 0.0, -1.0]])


def sobelLayer(img, gpu_id=None):
    """Sobel gradient magnitude of channel 0 (networks.py:852-868), without building
    new modules on every call.  Returns [1, H, W] for a batch-1 input like the reference."""
    x = img[:, :1].float()
    kx = _SOBEL_X.to(x.device).view(1, 1, 3, 3)
    ky = _SOBEL_X.t().contiguous().to(x.device).view(1, 1, 3, 3)
    gx = F.conv2d(x, kx, padding=1)
    gy = F.conv2d(x, ky, padding=1)
    g = torch.sqrt(gx * gx + gy * gy)
    return g[0] if g.shape[0] == 1 else g[:, 0]
