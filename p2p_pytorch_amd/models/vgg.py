"""Frozen VGG19 feature extractor + perceptual loss (reference ``Vgg19`` / ``VGGLoss``,
/root/reference/networks.py:18-62).

torchvision is not available, so the VGG19 'E' configuration is built in-repo with the
same module indices (``slice{k}.{idx}``) as ``torchvision.models.vgg19().features``
sliced at relu1_1 / relu2_1 / relu3_1 / relu4_1 / relu5_1.  ImageNet weights are read
from a local file when ``P2P_VGG19_WEIGHTS`` points at one (a safetensors file or a
``torch.save``d state dict, loaded with ``weights_only=True``); otherwise the network
is random-initialised (there is no network access) -- the loss is then a random-feature
perceptual loss with identical cost.  Inputs are fed in [-1, 1] with no ImageNet
normalisation, exactly like the reference (quirk A15).

Every ReLU is fused into its conv's epilogue and each max-pool is a separate kernel.  In the
perceptual loss the taps' gradients (relu' included) go straight into the next slice's first
conv's dgrad epilogue (``Vgg19.set_tap_fusion``).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d

# torchvision vgg19 'E' features: (index, kind, cin, cout)
_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
        512, 512, 512, 512, "M"]
_SLICES = [(0, 2), (2, 7), (7, 12), (12, 21), (21, 30)]


class _ReLU(nn.Module):
    def forward(self, x):
        return x  # fused into the preceding conv's epilogue


class _MaxPool(nn.Module):
    def forward(self, x):
        return ops.max_pool2(x)


def _vgg19_features():
    layers = []
    cin = 3
    for v in _CFG:
        if v == "M":
            layers.append(_MaxPool())
        else:
            layers.append(Conv2d(cin, v, 3, padding=1, act_out="relu"))
            layers.append(_ReLU())
            cin = v
    return layers


class Vgg19(nn.Module):
    def __init__(self, requires_grad=False, weights_path=None):
        super().__init__()
        feats = _vgg19_features()
        for k, (a, b) in enumerate(_SLICES, 1):
            seq = nn.Sequential()
            for idx in range(a, b):
                seq.add_module(str(idx), feats[idx])
            setattr(self, f"slice{k}", seq)
        self._init(weights_path or os.environ.get("P2P_VGG19_WEIGHTS"))
        # ReLU' of every conv whose output is not a loss tap moves into the next conv's dgrad
        # epilogue (a max-pool in between passes it through: the pooled value is the arg-max
        # input, so relu'(pool(y)) is relu'(y) where the gradient lands) -- no separate gate
        # pass in the perceptual loss's backward (HIP path; the oracle ignores the flags)
        for prod, cons in ((2, 5), (7, 10), (12, 14), (14, 16), (16, 19), (21, 23), (23, 25), (25, 28)):
            feats[prod].out_gated = True
            feats[cons].grad_gate = "relu"
        self._feats = feats
        self.tap_fusion = False
        if not requires_grad:
            for p in self.parameters():
                p.requires_grad = False

    # the loss taps (relu1_1 .. relu5_1 outputs) and the conv reading each of them
    _TAPS = ((0, 2), (5, 7), (10, 12), (19, 21), (28, None))

    def set_tap_fusion(self, on: bool = True):
        """HIP path, for a loss whose gradient w.r.t. every tap carries the tap's relu' and
        is parked for the tap's consumer conv (VGGLoss: ``ops.l1(gate_a="relu",
        defer=True)``): the tap convs leave relu' to their consumers, which add the parked
        loss gradient in their dgrad epilogue -- no accumulate or relu' pass per tap.  Off
        (default), the taps are ordinary outputs."""
        self.tap_fusion = bool(on)
        for prod, cons in self._TAPS:
            self._feats[prod].out_gated = self.tap_fusion
            if cons is not None:
                self._feats[cons].grad_gate = "relu" if self.tap_fusion else None
                self._feats[cons].skip_grad = "take" if self.tap_fusion else None
        return self

    def _init(self, path):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(m.bias)
        self.pretrained = False
        if path and os.path.exists(path):
            if path.endswith(".safetensors"):
                from safetensors.torch import load_file
                sd = load_file(path)
            else:
                sd = torch.load(path, map_location="cpu", weights_only=True)
            mapped = {}
            for k, v in sd.items():  # accept torchvision 'features.N.weight' keys
                key = k[len("features."):] if k.startswith("features.") else k
                idx, _, leaf = key.partition(".")
                if not idx.isdigit():
                    continue
                i = int(idx)
                for s, (a, b) in enumerate(_SLICES, 1):
                    if a <= i < b:
                        mapped[f"slice{s}.{i}.{leaf}"] = v
            self.load_state_dict(mapped, strict=False)
            self.pretrained = True

    def forward(self, x):
        h1 = self.slice1(x)
        h2 = self.slice2(h1)
        h3 = self.slice3(h2)
        h4 = self.slice4(h3)
        h5 = self.slice5(h4)
        return [h1, h2, h3, h4, h5]


class VGGLoss(nn.Module):
    """sum_i w_i * L1(phi_i(x), phi_i(y).detach()), w = [1/32, 1/16, 1/8, 1/4, 1]."""

    weights = [1.0 / 32, 1.0 / 16, 1.0 / 8, 1.0 / 4, 1.0]

    def __init__(self, device=None):
        super().__init__()
        self.vgg = Vgg19().set_tap_fusion(True)
        if device is not None:
            self.vgg = self.vgg.to(device)

    def target_features(self, y):
        """phi(y) without a graph: pass it as ``fy`` to every loss against the same target
        (the reference step evaluates VGG(real_b) twice, train.py:377 and :395 -- identical
        frozen-network features, so the second forward is skipped)."""
        with torch.no_grad():
            return self.vgg(y)

    def forward(self, x, y, fy=None):
        fx = self.vgg(x)
        if fy is None:
            fy = self.target_features(y)
        terms = []
        fused = self.vgg.tap_fusion
        for i, (a, b) in enumerate(zip(fx, fy)):
            if fused:   # relu' of the tap in the L1 gradient, parked for the next slice's conv
                terms.append(ops.l1(a, b.detach(), gate_a="relu", defer=i < len(fx) - 1))
            else:
                terms.append(ops.l1(a, b.detach()))
        # the weighted sum in one launch each way on the native path (ops.lincomb_n)
        return ops.lincomb_n(terms, self.weights[:len(terms)])
