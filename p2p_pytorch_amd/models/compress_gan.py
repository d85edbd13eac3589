"""Model family R: the reference's learned-compression / bit-depth-expansion GAN.

Parameter / buffer names match the reference exactly so generator checkpoints stay
interchangeable:

  * ``ExpandNetwork``        /root/reference/networks.py:447-523  (169 state-dict keys)
  * ``CompressionNetwork``   networks.py:201-236
  * ``ConvLayer`` / ``UpsampleConvLayer`` / ``ResidualBlock``  networks.py:395-444
  * ``SpectralNorm``         networks.py:525-582 (``weight_u``/``weight_v``/``weight_bar``)
  * ``NLayerDiscriminatorSN`` / ``MultiscaleDiscriminator``  networks.py:716-806

The forward passes are re-expressed on the fused op layer: reflection pad and nearest
upsample are folded into the conv's address generation (no padded / 4x tensor is ever
materialised), LeakyReLU is a conv epilogue, and the spectral-norm 1/sigma is applied to
the bf16 weight copy rather than materialised per call as a new parameter.
Reference quirks that are *observable* are reproduced (single shared PReLU, SN convs
keep PyTorch's default init, full-res input -> ``scale{num_D-1}_*``).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native, ops
from .layers import BatchNorm2d, Conv2d, link_norm


# P2P_FEAT_DEFER=0: D's feature-matching gradients accumulate through autograd (A/B knob)
_FEAT_DEFER = os.environ.get("P2P_FEAT_DEFER", "1") != "0"
# P2P_FAMR_STATS=0: the BNs compute their own statistics (A/B knob for the conv-epilogue stats)
_FUSED_STATS = os.environ.get("P2P_FAMR_STATS", "1") != "0"
# P2P_RES_FUSE=0: the residual join relu(BN(h) + x) as a separate add+act pass (A/B knob)
_RES_FUSE = os.environ.get("P2P_RES_FUSE", "1") != "0"


def ops_hip():
    from ..ops import hip   # imported lazily: it touches torch.ops.p2p
    return hip


class PReLU(nn.PReLU):
    def forward(self, x):
        return ops.prelu(x, self.weight)


class PixelUnshuffle(nn.Module):
    """Space-to-depth.  Output channel order ``c*r*r + dy*r + dx`` -- identical to the
    reference's one-hot grouped conv (networks.py:173-187) and to F.pixel_unshuffle."""

    def __init__(self, downscale_factor):
        super().__init__()
        self.downscale_factor = downscale_factor

    def forward(self, x):
        return ops.pixel_unshuffle(x, self.downscale_factor)


def pixel_unshuffle(x, downscale_factor):
    return ops.pixel_unshuffle(x, downscale_factor)


class PixelShuffle(nn.PixelShuffle):
    """Depth-to-space on the op layer (NHWC HIP kernel on the native path)."""

    def forward(self, x):
        return ops.pixel_shuffle(x, self.upscale_factor)


class ConvLayer(nn.Module):
    """ReflectionPad2d(k//2) + Conv2d(k, stride) -- pad folded into the conv."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, act_out=None):
        super().__init__()
        self.conv2d = Conv2d(in_channels, out_channels, kernel_size, stride=stride,
                             padding=kernel_size // 2, pad_mode="reflect", act_out=act_out)

    def forward(self, x):
        return self.conv2d(x)


class UpsampleConvLayer(nn.Module):
    """[nearest Upsample(x s)] + ReflectionPad2d(k//2) + Conv2d -- all one conv."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, upsample=None):
        super().__init__()
        self.upsample = upsample
        self.conv2d = Conv2d(in_channels, out_channels, kernel_size, stride=stride,
                             padding=kernel_size // 2, pad_mode="reflect",
                             upsample=int(upsample) if upsample else 1)

    def forward(self, x):
        return self.conv2d(x)


class ResidualBlock(nn.Module):
    """relu(BN(conv(relu(BN(conv(x))))) + x); BN attributes keep the reference's
    misleading ``in1``/``in2`` names (networks.py:429-444)."""

    def __init__(self, channels):
        super().__init__()
        self.conv1 = ConvLayer(channels, channels, kernel_size=3, stride=1)
        self.in1 = BatchNorm2d(channels, affine=True, act="relu")
        self.relu = nn.ReLU()
        self.conv2 = ConvLayer(channels, channels, kernel_size=3, stride=1)
        self.in2 = BatchNorm2d(channels, affine=True)
        # x is read by conv1 and by the residual add: the add's gradient for x is folded into
        # conv1's input-gradient pass (HIP path) instead of an autograd accumulate
        self.conv1.conv2d.skip_grad = "take"
        # the BN statistics come from the conv epilogues (no separate statistics pass)
        if _FUSED_STATS:
            link_norm(self.conv1.conv2d, self.in1)
            link_norm(self.conv2.conv2d, self.in2)

    def forward(self, x):
        h = self.conv2(self.in1(self.conv1(x)))
        if _RES_FUSE:
            # relu(BN(h) + x) in the BN apply pass; x's gradient goes to conv1's dgrad epilogue
            return self.in2(h, residual=x, act="relu", defer_residual=True)
        return ops.add_act(self.in2(h), x, "relu", defer_b=True)


class ExpandNetwork(nn.Module):
    """Generator "G": bit-depth expansion ResNet (networks.py:447-523)."""

    def __init__(self):
        super().__init__()
        self.relu = PReLU()              # ONE scalar shared by all 5 PReLU sites (quirk A9)
        self.leakyRelu = nn.LeakyReLU(0.2)
        self.tanh = nn.Tanh()
        self.inversePixel = PixelUnshuffle(2)
        self.upsclaing = nn.Upsample(scale_factor=2, mode="nearest")
        self.conv1 = ConvLayer(12, 32, kernel_size=9, stride=1)
        self.in1_e = BatchNorm2d(32, affine=True)
        self.conv2 = ConvLayer(32, 64, kernel_size=3, stride=2)
        self.in2_e = BatchNorm2d(64, affine=True)
        self.conv3 = ConvLayer(64, 128, kernel_size=3, stride=2)
        self.in3_e = BatchNorm2d(128, affine=True)
        for k in range(1, 10):
            setattr(self, f"res{k}", ResidualBlock(128))
        self.deconv3 = UpsampleConvLayer(128, 64, kernel_size=3, stride=1, upsample=2)
        self.in3_d = BatchNorm2d(64, affine=True)
        self.deconv2 = UpsampleConvLayer(64, 32, kernel_size=3, stride=1, upsample=2)
        self.in2_d = BatchNorm2d(32, affine=True)
        self.deconv1 = UpsampleConvLayer(32, 3, kernel_size=9, stride=1)
        self.in1_d = BatchNorm2d(3, affine=True, act="tanh")
        for conv, bn in ((self.conv2, self.in2_e), (self.conv3, self.in3_e), (self.deconv3, self.in3_d),
                         (self.deconv2, self.in2_d), (self.deconv1, self.in1_d)):
            if _FUSED_STATS:
                link_norm(conv.conv2d, bn)

    def forward(self, x):
        if x.shape[-1] % 4 or x.shape[-2] % 4:
            raise ValueError(f"ExpandNetwork needs H, W divisible by 4, got {tuple(x.shape[-2:])}"
                             " (quirk A16: the reference silently returns a wrong-size image)")
        # pixel-unshuffle(2) followed by nearest x2: the conv sees 12 channels at full res.
        # (as a conv input only: the quantiser may have written it unshuffled and padded)
        y = ops.pixel_unshuffle(x, self.inversePixel.downscale_factor, conv_input=True)
        y = ops.conv2d(y, self.conv1.conv2d.weight, self.conv1.conv2d.bias, 1, 4, "reflect", 2,
                       stats=self.training and _FUSED_STATS)
        pw = self.relu.weight            # PReLU fused into the BN passes (fwd and bwd)
        y = self.in1_e(y, prelu=pw)
        y = self.in2_e(self.conv2(y), prelu=pw)
        y = self.in3_e(self.conv3(y), prelu=pw)
        y, res = ops.fan_out(y, 2)   # the trunk and the long skip: one HIP-summed gradient
        for k in range(1, 10):
            res = getattr(self, f"res{k}")(res)
        y = ops.add_act(res, y, "lrelu")
        y = self.in3_d(self.deconv3(y), prelu=pw)
        y = self.in2_d(self.deconv2(y), prelu=pw)
        return self.in1_d(self.deconv1(y))


class CompressionNetwork(nn.Module):
    """Compressor "C": x + l2normalize_c(PixelShuffle2(conv s2(...))) (networks.py:201-236)."""

    def __init__(self):
        super().__init__()
        self.conv_input = nn.Sequential(ConvLayer(3, 64, kernel_size=5, stride=1), PReLU())
        self.conv_block1 = nn.Sequential(ConvLayer(64, 64, kernel_size=3, stride=1),
                                         BatchNorm2d(64), PReLU())
        self.conv_block2 = nn.Sequential(ConvLayer(64, 12, kernel_size=3, stride=2),
                                         PixelShuffle(2))
        if _FUSED_STATS:
            link_norm(self.conv_block1[0].conv2d, self.conv_block1[1])

    def forward(self, x):
        conv, bn, act = self.conv_block1
        h = bn(conv(self.conv_input(x)), prelu=act.weight)   # BN + PReLU: one pass
        # conv s2 -> PixelShuffle(2) -> l2-normalise + x: the shuffle is the normalising
        # pass's addressing (both directions), not a pass of its own
        conv2, shuf = self.conv_block2
        return ops.l2_normalize_channels(conv2(h), residual=x, shuffle=shuf.upscale_factor)


# ----------------------------------------------------------------- spectral norm
def l2normalize(v, eps=1e-12):
    return v / (v.norm() + eps)


class SpectralNorm(nn.Module):
    """Spectral-norm wrapper with the reference's parameter layout.

    ``weight`` is removed from the wrapped conv and replaced by ``weight_bar``
    (trainable) plus ``weight_u``/``weight_v`` (Parameters, requires_grad=False).  Each
    forward runs ``power_iterations`` steps of the power method (u, v updated in place,
    no gradient) and convolves with ``weight_bar / sigma`` where
    ``sigma = u . (W v)`` carries the gradient into ``weight_bar``.
    """

    def __init__(self, module, name="weight", power_iterations=1):
        super().__init__()
        self.module = module
        self.name = name
        self.power_iterations = power_iterations
        if not all(hasattr(module, name + s) for s in ("_u", "_v", "_bar")):
            w = getattr(module, name)
            h = w.shape[0]
            wd = w.detach().reshape(h, -1).shape[1]
            u = nn.Parameter(l2normalize(w.detach().new_empty(h).normal_(0, 1)), requires_grad=False)
            v = nn.Parameter(l2normalize(w.detach().new_empty(wd).normal_(0, 1)), requires_grad=False)
            w_bar = nn.Parameter(w.detach().clone())
            del module._parameters[name]
            module.register_parameter(name + "_u", u)
            module.register_parameter(name + "_v", v)
            module.register_parameter(name + "_bar", w_bar)

    def normalized_weight(self):
        m = self.module
        u = getattr(m, self.name + "_u")
        v = getattr(m, self.name + "_v")
        w = getattr(m, self.name + "_bar")
        h = w.shape[0]
        w2 = w.reshape(h, -1)
        # ``.data`` assignment like the reference (networks.py:543-546): it swaps storage
        # without bumping the version counter, so a backward through an EARLIER forward of
        # this step sees the newest u / v (what the reference computes) instead of
        # raising an in-place-modification error.
        # fp32 always (also under an autocast region: sigma is a norm, and u / v are state)
        with torch.autocast(device_type=w.device.type, enabled=False):
            if w.is_cuda and _native.use_native(w):
                # HIP power iteration (csrc/sn.hip): 4 short launches, u / v in place
                sigma = ops_hip().spectral_sigma(w2, u, v, self.power_iterations)
                return w / sigma
            for _ in range(self.power_iterations):
                v.data = l2normalize(torch.mv(w2.detach().t(), u.data))
                u.data = l2normalize(torch.mv(w2.detach(), v.data))
            sigma = torch.dot(u, torch.mv(w2, v))
            return w / sigma

    def forward(self, x):
        m = self.module
        w = getattr(m, self.name + "_bar")
        pad_mode = getattr(m, "pad_mode", "zeros")
        if w.is_cuda and _native.use_native(w) and pad_mode == "zeros" and m.padding[0] == m.padding[1]:
            # 1 / sigma stays a device scalar applied in the conv epilogues (ops/hip.py SNConvFn)
            u = getattr(m, self.name + "_u")
            v = getattr(m, self.name + "_v")
            # (the sigma path of the weight_bar gradient is fused into the conv's weight
            # gradient: csrc/sn.hip sn_wgrad)
            with torch.autocast(device_type=w.device.type, enabled=False):
                scale = ops_hip().sn_scale(w.reshape(w.shape[0], -1), u, v, self.power_iterations)
            return ops_hip().sn_conv2d(x, w, m.bias, scale, m.stride, m.padding,
                                       getattr(m, "act_in", None), getattr(m, "act_out", None),
                                       getattr(m, "grad_gate", None), getattr(m, "out_gated", False),
                                       uv=(u, v), skip_grad=getattr(m, "skip_grad", None))
        w = self.normalized_weight()
        return ops.conv2d(x, w, m.bias, m.stride, m.padding, pad_mode, 1,
                          getattr(m, "act_in", None), getattr(m, "act_out", None))


class NLayerDiscriminatorSN(nn.Module):
    """70x70 PatchGAN with spectral norm on the middle convs, padding 2, no norm layers,
    LeakyReLU(0.2) fused into each conv (networks.py:758-806)."""

    def __init__(self, input_nc, ndf=64, n_layers=3, norm_layer=None, use_sigmoid=False,
                 getIntermFeat=False):
        super().__init__()
        self.getIntermFeat = getIntermFeat
        self.n_layers = n_layers
        kw, padw = 4, 2
        seq = [[Conv2d(input_nc, ndf, kw, stride=2, padding=padw, act_out="lrelu")]]
        nf = ndf
        for _ in range(1, n_layers):
            nf_prev, nf = nf, min(nf * 2, 512)
            seq.append([SpectralNorm(Conv2d(nf_prev, nf, kw, stride=2, padding=padw,
                                            act_out="lrelu"))])
        nf_prev, nf = nf, min(nf * 2, 512)
        seq.append([SpectralNorm(Conv2d(nf_prev, nf, kw, stride=1, padding=padw, act_out="lrelu"))])
        seq.append([Conv2d(nf, 1, kw, stride=1, padding=padw,
                           act_out="sigmoid" if use_sigmoid else None)])
        self._chain = [s[0].module if isinstance(s[0], SpectralNorm) else s[0] for s in seq]
        self.feature_grad_gate = None
        if getIntermFeat:
            for k, s in enumerate(seq):
                setattr(self, f"model{k}", nn.Sequential(*s))
        else:
            self.model = nn.Sequential(*[m for s in seq for m in s])

    def set_feature_grad_gate(self, on=True):
        """Opt-in (the family-R training step enables it): every LeakyReLU derivative moves
        into the next conv's dgrad epilogue (HIP path) -- no separate gate pass per layer.
        Only valid when every OTHER consumer of the intermediate features applies lrelu' to
        its own gradient, as the step's feature-matching L1 does (``ops.l1(..., gate_a=
        self.feature_grad_gate)``).  The next conv also takes a feature gradient the L1 parked
        for it (``ops.l1(defer=True)``, ``skip_grad="take"``): added in its dgrad epilogue
        instead of an autograd accumulate of the two consumers' gradients.  The oracle path
        ignores the flags."""
        for prod, cons in zip(self._chain[:-1], self._chain[1:]):
            if getattr(prod, "act_out", None) == "lrelu":
                prod.out_gated = bool(on)
                cons.grad_gate = "lrelu" if on else None
                cons.skip_grad = "take" if (on and _FEAT_DEFER) else None
        self.feature_grad_gate = "lrelu" if on else None

    def forward(self, x):
        if self.getIntermFeat:
            out = []
            for k in range(self.n_layers + 2):
                x = getattr(self, f"model{k}")(x)
                out.append(x)
            return out
        return self.model(x)


class MultiscaleDiscriminator(nn.Module):
    """num_D PatchGANs on an AvgPool pyramid.  Modules registered flat as
    ``scale{i}_layer{j}``; the full-resolution input goes to ``scale{num_D-1}`` (A10)."""

    def __init__(self, input_nc, ndf=64, n_layers=3, norm_layer=None, use_sigmoid=False, num_D=3,
                 getIntermFeat=False):
        super().__init__()
        self.num_D = num_D
        self.n_layers = n_layers
        self.getIntermFeat = getIntermFeat
        self.feature_grad_gate = None
        self._subs = []   # plain list (not registered): the per-scale gate chains
        for i in range(num_D):
            d = NLayerDiscriminatorSN(input_nc, ndf, n_layers, norm_layer, use_sigmoid, getIntermFeat)
            self._subs.append(d)
            if getIntermFeat:
                for j in range(n_layers + 2):
                    setattr(self, f"scale{i}_layer{j}", getattr(d, f"model{j}"))
            else:
                setattr(self, f"layer{i}", d.model)

    def set_feature_grad_gate(self, on=True):
        """See NLayerDiscriminatorSN.set_feature_grad_gate."""
        for d in self._subs:
            d.set_feature_grad_gate(on)
        self.feature_grad_gate = "lrelu" if on else None

    def downsample(self, x):
        if isinstance(x, (tuple, list)):  # virtual concat: pool each half
            return tuple(ops.avg_pool3_s2(t) for t in x)
        return ops.avg_pool3_s2(x)

    def _single(self, i, x):
        if self.getIntermFeat:
            out = []
            for j in range(self.n_layers + 2):
                x = getattr(self, f"scale{i}_layer{j}")(x)
                out.append(x)
            return out
        return [getattr(self, f"layer{i}")(x)]

    def forward(self, x):
        result = []
        for i in range(self.num_D):
            xs = x
            if i != self.num_D - 1:
                # this scale's PatchGAN and the next pyramid level both read x: their
                # gradients meet in one fan-out node (HIP adds) instead of autograd's add
                if isinstance(x, (tuple, list)):
                    pairs = [ops.fan_out(t, 2) for t in x]
                    xs, x = tuple(p[0] for p in pairs), tuple(p[1] for p in pairs)
                else:
                    xs, x = ops.fan_out(x, 2)
            result.append(self._single(self.num_D - 1 - i, xs))
            if i != self.num_D - 1:
                x = self.downsample(x)
        return result
