"""Functional op layer used by every model in ``p2p_pytorch_amd.models``.

Each op routes GPU tensors to the HIP/CDNA4 kernels (``ops/hip.py`` -> ``torch.ops.p2p``)
and CPU tensors to the PyTorch oracle (``ops/reference.py``).  See ``_native.use_native``
for the no-silent-fallback policy.
"""
from __future__ import annotations

import torch

from .. import _native
from . import reference as ref

LRELU_SLOPE = ref.LRELU_SLOPE
apply_act = ref.apply_act


def _first(x):
    return x[0] if isinstance(x, (tuple, list)) else x


def _hip():
    from . import hip  # imported lazily: it touches torch.ops.p2p
    return hip


def conv2d(x, weight, bias=None, stride=1, padding=0, pad_mode="zeros", upsample=1,
           act_in=None, act_out=None, stats=False, grad_gate=None, out_gated=False, skip_grad=None):
    """HIP-path fusion hints (ignored by the oracle): ``stats`` -- the output feeds a norm,
    emit its statistics; ``grad_gate`` / ``out_gated`` -- move the producer's activation
    derivative into this conv's dgrad epilogue; ``skip_grad`` -- one gradient write for a
    tensor read by two convs (see ``hip._ConvCfg``)."""
    if _native.use_native(_first(x)):
        return _hip().conv2d(x, weight, bias, stride, padding, pad_mode, upsample, act_in, act_out,
                             stats, grad_gate, out_gated, skip_grad)
    return ref.conv2d(x, weight, bias, stride, padding, pad_mode, upsample, act_in, act_out)


def conv_transpose2d(x, weight, bias=None, stride=2, padding=1, act_in=None, act_out=None,
                     stats=False, grad_gate=None, out_gated=False, skip_grad=None, gate_x2=True):
    """``gate_x2=False`` (HIP path): the second half of a virtual-concat input is already
    ReLU'd by its producer, whose backward applies the same gate -- skip re-reading it."""
    if _native.use_native(_first(x)):
        return _hip().conv_transpose2d(x, weight, bias, stride, padding, act_in, act_out, stats,
                                       grad_gate, out_gated, skip_grad, gate_x2)
    return ref.conv_transpose2d(x, weight, bias, stride, padding, act_in, act_out)


def instance_norm(x, eps=1e-5, act=None, weight=None, bias=None, qkey=None):
    """``qkey`` (HIP path, fp8 precision): stable key of the module's fp8 shadow sites."""
    if _native.use_native(x):
        return _hip().instance_norm(x, eps, act, weight, bias, qkey)
    return ref.instance_norm(x, eps, act, weight, bias)


def batch_norm(x, running_mean, running_var, weight, bias, training, momentum=0.1, eps=1e-5,
               act=None, qkey=None, prelu_weight=None, residual=None, defer_residual=False):
    """``prelu_weight``: a shared-slope PReLU applied to the output (fused into the apply pass
    and, in the backward, into the norm's partial-sum pass -- slope gradient included).
    ``residual``: y = act(BN(x) + residual) in the apply pass (a residual block's join);
    ``defer_residual`` (HIP path): residual's gradient goes to the conv that also reads it."""
    if _native.use_native(x):
        return _hip().batch_norm(x, running_mean, running_var, weight, bias, training, momentum,
                                 eps, act, prelu_weight=prelu_weight, qkey=qkey,
                                 residual=residual, defer_residual=defer_residual)
    if residual is not None:
        y = ref.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
        return ref.apply_act(y + residual, act)
    y = ref.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps, act)
    return y if prelu_weight is None else ref.prelu(y, prelu_weight)


def prelu(x, weight):
    if _native.use_native(x):
        return _hip().prelu(x, weight)
    return ref.prelu(x, weight)


def act(x, name):
    if name is None:
        return x
    if _native.use_native(x):
        return _hip().act(x, name)
    return ref.apply_act(x, name)


def add_act(a, b, name, defer_b=False):
    """act(a + b) -- one fused pass on the native path (residual joins).  ``defer_b`` (HIP
    path): hand b's gradient to the conv that also reads b (its ``skip_grad="take"``)."""
    if name is None:
        return a + b
    if _native.use_native(a):
        return _hip().add_act(a, b, name, defer_b)
    return ref.apply_act(a + b, name)


def fan_out(x, n):
    """``n`` handles of ``x`` for ``n`` consumers.  HIP path: their gradients are summed by HIP
    adds in one backward node, not by autograd's input-buffer accumulation (an aten add per
    extra consumer); elsewhere the same tensor ``n`` times."""
    if x is not None and x.requires_grad and _native.use_native(x):
        return _hip().fan_out(x, n)
    return (x,) * n


def dropout(x, p, training, salt=None):
    """``salt``: per-module constant mixed with the device seed (advanced once per step), so
    a captured graph draws the same masks as the eager step it replays."""
    if not training or p == 0.0:
        return x
    if _native.use_native(x):
        return _hip().dropout(x, p, salt)
    return ref.dropout(x, p, training)


def mse_const(pred, target):
    if _native.use_native(pred):
        return _hip().mse_const(pred, target)
    return ref.mse_const(pred, target)


def bce_logits_const(pred, target):
    if _native.use_native(pred):
        return _hip().bce_logits_const(pred, target)
    return ref.bce_logits_const(pred, target)


def bce_const(prob, target):
    if _native.use_native(prob):
        return _hip().bce_const(prob, target)
    return ref.bce_const(prob, target)


def l1(a, b, gate_a=None, defer=False):
    """``gate_a`` (HIP path): the gradient of ``a`` also carries that activation's derivative
    (its producer is ``out_gated``); the oracle's producers apply their own activation.
    ``defer`` (HIP path): a's gradient goes to the conv reading ``a`` with
    ``skip_grad="take"`` (added in its dgrad epilogue) instead of through autograd."""
    if _native.use_native(a):
        return _hip().l1(a, b, gate_a, defer)
    return ref.l1(a, b)


def mse(a, b):
    if _native.use_native(a):
        return _hip().mse(a, b)
    return ref.mse(a, b)


def tv(x):
    if _native.use_native(x):
        return _hip().tv(x)
    return ref.tv(x)


def quantize(x, bits, unshuffle=0):
    """``unshuffle`` r (HIP path): the same pass also writes the pixel-unshuffled, channel-
    padded copy that ``pixel_unshuffle(y, r, conv_input=True)`` hands to the next conv."""
    if _native.use_native(x):
        return _hip().quantize(x, bits, unshuffle)
    return ref.quantize(x, bits)


def avg_pool3_s2(x):
    if _native.use_native(x):
        return _hip().avg_pool3_s2(x)
    return ref.avg_pool3_s2(x)


def l2_normalize_channels(x, eps=1e-12, residual=None, shuffle=1):
    """x / ||x||_2 over channels, plus ``residual`` (fused into the same pass when native).
    ``shuffle`` r > 1: of ``pixel_shuffle(x, r)`` -- on the native path the shuffle is the
    normalising pass's own addressing (forward and backward), not a pass."""
    if _native.use_native(x):
        return _hip().l2_normalize_channels(x, eps, residual, shuffle)
    if shuffle > 1:
        x = torch.nn.functional.pixel_shuffle(x, shuffle)
    y = ref.l2_normalize_channels(x, eps)
    return y if residual is None else y + residual


def lincomb_n(terms, weights):
    """``sum(w * t)`` of loss scalars: one HIP launch each way for GPU tensors on the native
    backend (python-float terms allowed only on the torch path)."""
    ts = [t for t in terms if isinstance(t, torch.Tensor)]
    if ts and len(ts) == len(terms) and _native.use_native(ts[0]) and all(
            t.dtype == torch.float32 and t.numel() == 1 for t in ts):
        return _hip().lincomb_n(terms, weights)
    out = 0
    for t, w in zip(terms, weights):
        out = out + w * t
    return out


def pixel_shuffle(x, r):
    if _native.use_native(x):
        return _hip().pixel_shuffle(x, r)
    return torch.nn.functional.pixel_shuffle(x, r)


def pixel_unshuffle(x, r, conv_input=False):
    """``conv_input`` (HIP path): the result only feeds a conv -- a copy the producer of ``x``
    already wrote unshuffled and channel-padded (``quantize(..., unshuffle=r)``) is returned
    as is (a packed pad-8 conv input), so no unshuffle / pad pass runs."""
    if _native.use_native(x):
        return _hip().pixel_unshuffle(x, r, conv_input)
    return torch.nn.functional.pixel_unshuffle(x, r)


def max_pool2(x):
    if _native.use_native(x):
        return _hip().max_pool2(x)
    return torch.nn.functional.max_pool2d(x, 2, 2)
