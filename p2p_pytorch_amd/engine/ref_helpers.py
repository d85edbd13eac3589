"""The reference ``train.py``'s module-level helpers, importable under the same names and
signatures (/root/reference/train.py:33-126; SURVEY.md section 1 L4 lists them as the
importable surface).  ``train.py`` re-exports every one, so ``from train import psnr,
load_checkpoint, calc_tv_Loss`` works as it does against the reference.

Behaviour notes:
  * ``tensor2img`` / ``tensor2np`` keep the reference's [0, 1] assumption (quirk A11: on
    [-1, 1] data the negative half clips to 0).
  * ``ssim`` / ``psnr`` return Python floats like the reference's numpy / skimage path; the
    SSIM is the in-repo skimage-compatible one (``engine/metrics.py``: 7x7 uniform window,
    sample covariance, float data range 2) because skimage is not available.
  * ``load_checkpoint`` keeps the reference's argument order and 8-tuple return, reads with
    ``weights_only=True``, and raises ``SystemExit`` where the reference calls ``exit()``.
  * ``extract_features`` applies the ImageNet normalisation the reference gets from
    torchvision ``transforms.Normalize`` (not installed here) by hand.
"""
from __future__ import annotations

import os

import torch

from ..data.image_io import tensor2img, tensor2np  # noqa: F401  (same semantics)
from ..models.losses import calc_tv_Loss  # noqa: F401
from . import metrics as _metrics

_IMAGENET_MEAN = (0.485, 0.456, 0.406)
_IMAGENET_STD = (0.229, 0.224, 0.225)


def _as_batch(t: torch.Tensor) -> torch.Tensor:
    t = t.detach().float().cpu()
    while t.dim() < 4:
        t = t.unsqueeze(0)
    return t


def ssim(image_out, image_ref) -> float:
    """SSIM of two [1, C, H, W] (or [C, H, W]) tensors through ``tensor2img`` levels
    (train.py:54-58)."""
    return float(_metrics.ssim(_as_batch(image_out), _as_batch(image_ref))[0])


def psnr(ground, compressed) -> float:
    """10 log10(255^2 / MSE) on the uint8 levels (train.py:60-65); inf when identical."""
    return float(_metrics.psnr(_as_batch(ground), _as_batch(compressed))[0])


def extract_features(model, x, layers):
    """Run ``model`` (an iterable of layers) on ImageNet-normalised ``x`` and collect the
    outputs of the ``layers`` indices (train.py:67-77)."""
    mean = torch.tensor(_IMAGENET_MEAN, dtype=x.dtype, device=x.device).view(1, -1, 1, 1)
    std = torch.tensor(_IMAGENET_STD, dtype=x.dtype, device=x.device).view(1, -1, 1, 1)
    x = (x - mean) / std
    features = []
    for index, layer in enumerate(model):
        x = layer(x)
        if index in layers:
            features.append(x)
    return features


def gram(x):
    b, c, h, w = x.size()
    f = x.reshape(b, c, h * w)
    return torch.bmm(f, f.transpose(1, 2)).div(h * w)


def calc_Gram_Loss(features, targets, weights=None):
    if weights is None:
        weights = [1 / len(features)] * len(features)
    loss = 0
    for f, t, w in zip(features, targets, weights):
        loss = loss + torch.nn.functional.mse_loss(gram(f), gram(t)) * w
    return loss


def calc_c_loss(features, targets, weights=None):
    if weights is None:
        weights = [1 / len(features)] * len(features)
    loss = 0
    for f, t, w in zip(features, targets, weights):
        loss = loss + torch.nn.functional.mse_loss(f, t) * w
    return loss


def load_checkpoint(net_g, net_d, opt_g, opt_d, sched_g, sched_d, loss_logger,
                    filename="net_epoch_x.pth"):
    """Reference signature and return tuple (train.py:103-121).  Works on the files this
    framework writes (which carry the keys the reference's own files lack)."""
    if not os.path.isfile(filename):
        print("=> No checkpoint found at '{}'".format(filename))
        raise SystemExit(1)
    print("=> Loading checkpoint '{}'".format(filename))
    state = torch.load(filename, map_location="cpu", weights_only=True)
    start_epoch = state["epoch"]
    net_g.load_state_dict(state["state_dict_g"])
    net_d.load_state_dict(state["state_dict_d"])
    opt_g.load_state_dict(state["optimizer_g"])
    opt_d.load_state_dict(state["optimizer_d"])
    sched_g.load_state_dict(state["scheduler_g"])
    sched_d.load_state_dict(state["scheduler_d"])
    loss_logger = state["losslogger"]
    return start_epoch, net_g, net_d, opt_g, opt_d, sched_g, sched_d, loss_logger
