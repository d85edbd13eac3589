"""Building-block modules.  They subclass the stock ``torch.nn`` classes so parameter
names / shapes / ``state_dict`` keys are identical to what the reference saves, but
their ``forward`` goes through ``p2p_pytorch_amd.ops`` (HIP kernels on the GPU) and can
fuse the neighbouring pad / upsample / concat / activation into the conv itself.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .. import _native, ops
from ..ops.fp8 import obj_key as _f8_key


class Conv2d(nn.Conv2d):
    """nn.Conv2d with fused prologue (pad mode, nearest upsample, input activation,
    virtual concat of a tuple input) and fused output activation."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True,
                 pad_mode="zeros", upsample=1, act_in=None, act_out=None):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         bias=bias)
        self.pad_mode = pad_mode
        self.upsample = upsample
        self.act_in = act_in
        self.act_out = act_out
        self.norm_stats = False   # set by link_norm(): a norm consumes the output
        self.grad_gate = None     # set by link_gate(): apply the producer's act' in dgrad
        self.out_gated = False    # set by link_gate(): consumers apply act_out' for us
        self.skip_grad = None     # set by link_skip(): "take" a parked skip gradient in dgrad

    def forward(self, x):  # noqa: D401
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.pad_mode,
                          self.upsample, self.act_in, self.act_out,
                          stats=self.norm_stats and self.training, grad_gate=self.grad_gate,
                          out_gated=self.out_gated, skip_grad=self.skip_grad)


class ConvTranspose2d(nn.ConvTranspose2d):
    """nn.ConvTranspose2d (weight [Cin, Cout, kh, kw]) with fused input activation and
    virtual concat -- the pix2pix decoder ``ReLU -> ConvT`` on ``cat(skip, up)``."""

    def __init__(self, in_channels, out_channels, kernel_size=4, stride=2, padding=1, bias=True,
                 act_in=None, act_out=None):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         bias=bias)
        self.act_in = act_in
        self.act_out = act_out
        self.norm_stats = False
        self.grad_gate = None
        self.out_gated = False
        self.skip_grad = None
        self.gate_x2 = True       # False: the concat's second half arrives already ReLU'd

    def forward(self, x):
        return ops.conv_transpose2d(x, self.weight, self.bias, self.stride[0], self.padding[0],
                                    self.act_in, self.act_out,
                                    stats=self.norm_stats and self.training,
                                    grad_gate=self.grad_gate, out_gated=self.out_gated,
                                    skip_grad=self.skip_grad, gate_x2=self.gate_x2)


def link_norm(conv, norm):
    """Mark ``conv`` as feeding ``norm`` directly: on the HIP path the conv epilogue then
    emits the per-tile (mean, M2) partials and the norm skips its own statistics pass."""
    if isinstance(norm, (InstanceNorm2d, BatchNorm2d)) and hasattr(conv, "norm_stats"):
        conv.norm_stats = True


def link_skip(first, second):
    """``first`` (whose backward runs first: the decoder ConvT reading a U-Net skip as the
    x1 half of its virtual concat) parks its skip gradient; ``second`` (the next encoder
    conv, reading the same tensor as its only input) adds it in its dgrad epilogue -- one
    gradient write per skip instead of two writes plus autograd's accumulate kernel."""
    if os.environ.get("P2P_SKIP_GRAD_FUSE", "1") == "0":   # A/B knob
        return
    if hasattr(first, "skip_grad") and hasattr(second, "skip_grad"):
        first.skip_grad = "defer"
        second.skip_grad = "take"


def link_gate(producer, consumers):
    """Fuse ``producer``'s output-activation derivative (ReLU / LeakyReLU, whose sign test
    reads the same from the stored output as from the input) into the dgrad epilogues of
    its ``consumers`` -- only when EVERY consumer of the output is listed here and either
    gates (``grad_gate``) or already applies an equivalent input ReLU (``act_in``)."""
    act = getattr(producer, "act_out", None)
    if act not in ("relu", "lrelu"):
        return
    for c in consumers:
        if getattr(c, "act_in", None) == "relu":
            continue   # relu'(act(x)) * act'(x) == relu'(act(x)) for relu / lrelu
        if getattr(c, "act_in", None) is not None or not hasattr(c, "grad_gate"):
            return
    for c in consumers:
        if getattr(c, "act_in", None) is None:
            c.grad_gate = act
    producer.out_gated = True


class InstanceNorm2d(nn.Module):
    """InstanceNorm2d(affine=False, track_running_stats=False) + fused activation
    (pix2pix 'instance' norm)."""

    def __init__(self, num_features, eps=1e-5, act=None, affine=False):
        super().__init__()
        self.num_features = num_features
        self.eps = eps
        self.act = act
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)

    def forward(self, x):
        return ops.instance_norm(x, self.eps, self.act, self.weight, self.bias, qkey=_f8_key(self))


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d (same buffers/keys) with a fused output activation."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, act=None):
        super().__init__(num_features, eps=eps, momentum=momentum, affine=affine)
        self.act = act

    def forward(self, x, prelu=None, residual=None, act=None, defer_residual=False):
        """``prelu``: slope Parameter of a following shared-slope PReLU, fused in.
        ``residual`` / ``act``: y = act(BN(x) + residual) in the same apply pass (overrides the
        module's own act); ``defer_residual``: see ``ops.batch_norm``."""
        training = self.training or not self.track_running_stats
        if self.training and self.track_running_stats:
            if self.num_batches_tracked.is_cuda and _native.use_native(x):
                _native.ops().i64_add_(self.num_batches_tracked, 1)   # HIP kernel, not aten
            else:
                self.num_batches_tracked.add_(1)
        return ops.batch_norm(x, self.running_mean if self.track_running_stats else None,
                              self.running_var if self.track_running_stats else None,
                              self.weight, self.bias, training, self.momentum, self.eps,
                              self.act if residual is None else act,
                              qkey=_f8_key(self), prelu_weight=prelu, residual=residual,
                              defer_residual=defer_residual)


class Act(nn.Module):
    def __init__(self, name):
        super().__init__()
        self.name = name

    def forward(self, x):
        return ops.act(x, self.name)


class Dropout(nn.Module):
    _next_salt = 1

    def __init__(self, p=0.5, salt=None):
        super().__init__()
        self.p = p
        # fixed per module: masks vary per step through the device seed only (models pass
        # their own salts so two instances of a network draw identical masks)
        if salt is None:
            salt = Dropout._next_salt
            Dropout._next_salt += 1
        self.salt = int(salt)

    def forward(self, x):
        return ops.dropout(x, self.p, self.training, self.salt)


def norm_layer(kind: str, channels: int, act=None):
    if kind == "instance":
        return InstanceNorm2d(channels, act=act)
    if kind == "batch":
        return BatchNorm2d(channels, act=act)
    if kind in ("none", None):
        return Act(act) if act else nn.Identity()
    raise NotImplementedError(f"normalization layer [{kind}] is not found")
