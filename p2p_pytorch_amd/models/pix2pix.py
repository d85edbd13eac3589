"""Model family P: the classic pix2pix U-Net generator and PatchGAN / pixel discriminators.

The reference repository has no U-Net; BASELINE.json's benchmark
configs name "U-Net-256 + 70x70 PatchGAN" and "4-layer U-Net + 1x1 PatchGAN".  The
reference carries the knobs for this family (``--ngf`` /root/reference/train.py:148,
``--lamb`` "weight on L1 term" train.py:156 and the commented L1 term train.py:341) and
its D is built from the same 70x70 PatchGAN recipe (networks.py:758-806).

Design (MI355X-first): the U-Net is kept *flat* -- explicit encoder/decoder lists --
instead of the recursive skip-block nesting of the pix2pix template, and every
activation is stored *pre-applied by its producer* so the conv loaders stay cheap:
  * encoder level i stores ``LeakyReLU(norm(conv(.)))`` (the outermost conv: LeakyReLU in
    its epilogue) -- the next encoder conv reads it as is;
  * the innermost conv stores ``ReLU(conv(.))`` (its only consumer is ReLU -> ConvT);
  * decoder levels store ``ReLU(norm(convT(.)))`` (dropout after it: ReLU commutes with
    the positive 2x/0 dropout scale);
  * every ``ReLU -> ConvT(cat(skip, up))`` is one fused transposed conv reading the two
    halves of the concat through two base pointers (no ``torch.cat`` materialised) with
    a packed-int16 ReLU in its loader: ``relu(lrelu(x)) == relu(x)`` exactly, and
    ``relu(relu(u)) == relu(u)``;
  * the final ``Tanh`` is the epilogue of the last ConvT.
Numerically this is the standard U-Net (every derivative is exact too: d relu(lrelu(x))
= [x > 0]): level ``i`` has ``ngf*min(2^i, 8)`` channels, no norm on the outermost /
innermost down convs, dropout on the ``num_downs-5`` decoder levels right outside the
innermost one.
"""
from __future__ import annotations

import torch.nn as nn

from .layers import Conv2d, ConvTranspose2d, Dropout, link_gate, link_norm, link_skip, norm_layer


class UnetGenerator(nn.Module):
    def __init__(self, input_nc=3, output_nc=3, num_downs=8, ngf=64, norm="instance",
                 use_dropout=True):
        super().__init__()
        if num_downs < 2:
            raise ValueError("num_downs must be >= 2")
        self.num_downs = num_downs
        use_bias = norm != "batch"
        ch = [ngf * min(2 ** i, 8) for i in range(num_downs)]
        self.channels = ch
        n = num_downs
        self.downs = nn.ModuleList()
        self.down_norms = nn.ModuleList()
        for i in range(n):
            cin = input_nc if i == 0 else ch[i - 1]
            has_norm = 0 < i < n - 1
            act_out = None if has_norm else ("relu" if i == n - 1 else "lrelu")
            self.downs.append(Conv2d(cin, ch[i], 4, stride=2, padding=1, bias=use_bias,
                                     act_out=act_out))
            self.down_norms.append(norm_layer(norm, ch[i], act="lrelu") if has_norm
                                   else nn.Identity())
        self.ups = nn.ModuleList()
        self.up_norms = nn.ModuleList()
        self.drop_levels = set(range(max(1, n - 1 - max(0, n - 5)), n - 1)) if use_dropout else set()
        for i in range(n):
            cin = ch[i] if i == n - 1 else 2 * ch[i]
            cout = output_nc if i == 0 else ch[i - 1]
            self.ups.append(ConvTranspose2d(cin, cout, 4, stride=2, padding=1,
                                            bias=True if i == 0 else use_bias,
                                            act_in=None if i == n - 1 else "relu",
                                            act_out="tanh" if i == 0 else None))
            self.up_norms.append(norm_layer(norm, cout, act="relu") if i > 0 else nn.Identity())
        self.dropouts = nn.ModuleList(
            [Dropout(0.5, salt=1000 + i) if i in self.drop_levels else nn.Identity()
             for i in range(n)])
        for c, m in list(zip(self.downs, self.down_norms)) + list(zip(self.ups, self.up_norms)):
            link_norm(c, m)
        # outermost encoder output feeds downs[1] and (skip) ups[0]; innermost feeds ups[n-1]
        link_gate(self.downs[0], [self.downs[1], self.ups[0]])
        link_gate(self.downs[n - 1], [self.ups[n - 1]])
        # skip i is read by ups[i] (backward first) and downs[i + 1]: one gradient write
        for i in range(n - 1):
            link_skip(self.ups[i], self.downs[i + 1])
            # the up half u = [dropout](ReLU(norm(.))) is ReLU'd by its producer, whose
            # backward applies the same gate [norm > 0]: the ConvT's input ReLU' on u is
            # redundant, so its dgrad epilogue gates (and re-reads) the skip half only
            self.ups[i].gate_x2 = False

    def forward(self, x):
        n = self.num_downs
        skips = []
        h = x
        for i in range(n):
            h = self.down_norms[i](self.downs[i](h))
            skips.append(h)
        u = self.dropouts[n - 1](self.up_norms[n - 1](self.ups[n - 1](skips[n - 1])))
        for i in range(n - 2, -1, -1):
            u = self.ups[i]((skips[i], u))
            u = self.dropouts[i](self.up_norms[i](u))
        return u

    def packed_ok(self, x) -> bool:
        """The packed-image path (ops/hip.py, image head) applies: 3 -> 3 channels, the
        standard outermost 4x4 s2 p1 layers, channel groups of 64."""
        from ..ops import hip
        n = self.num_downs
        return (n >= 2 and self.downs[0].in_channels == 3 and self.ups[0].out_channels == 3
                and self.channels[0] % 64 == 0 and x.shape[-1] % 2 == 0 and x.shape[-2] % 2 == 0
                and tuple(self.downs[0].kernel_size) == (4, 4) and self.downs[0].stride[0] == 2
                and self.downs[0].padding[0] == 1 and hip.image_head_ok(
                    self.ups[0], _Shape(self.channels[0]), _Shape(self.channels[0])))

    def forward_packed(self, dd, scale):
        """Training forward on the packed pair tensor ``dd`` = [(unset); (A | B)] (2N x 8
        channels, see ops/hip.py image head): reads A from ``dd[N:]``, writes the generated
        image into ``dd[:N]`` as (A | fake) and returns (that view, ``scale * sum|fake - B|``)."""
        from ..ops import hip
        n = self.num_downs
        N = dd.shape[0] // 2
        ab = dd.narrow(0, N, N)
        ab._p2p_packed = (3, 3)          # e1's weight is zero on the B channels
        skips = []
        h = ab
        for i in range(n):
            h = self.down_norms[i](self.downs[i](h))
            skips.append(h)
        u = self.dropouts[n - 1](self.up_norms[n - 1](self.ups[n - 1](skips[n - 1])))
        for i in range(n - 2, 0, -1):
            u = self.ups[i]((skips[i], u))
            u = self.dropouts[i](self.up_norms[i](u))
        return hip.image_head(skips[0], u, self.ups[0], dd, scale)


class _Shape:
    """Channel-count stand-in for ``image_head_ok`` checks before any tensor exists."""

    def __init__(self, c):
        self.shape = (1, c)


class NLayerDiscriminator(nn.Module):
    """PatchGAN.  With n_layers=3 and 4x4 kernels the receptive field is 70x70
    (reference networks.py:758-787 builds the same ladder with padding 2; pix2pix uses 1)."""

    def __init__(self, input_nc, ndf=64, n_layers=3, norm="instance", use_sigmoid=False, padw=1):
        super().__init__()
        use_bias = norm != "batch"
        # LeakyReLU stored pre-applied: first conv's epilogue, then fused into each norm
        layers = [Conv2d(input_nc, ndf, 4, stride=2, padding=padw, act_out="lrelu")]
        norms = [nn.Identity()]
        nf = ndf
        for k in range(1, n_layers):
            nf_prev, nf = nf, ndf * min(2 ** k, 8)
            layers.append(Conv2d(nf_prev, nf, 4, stride=2, padding=padw, bias=use_bias))
            norms.append(norm_layer(norm, nf, act="lrelu"))
        nf_prev, nf = nf, ndf * min(2 ** n_layers, 8)
        layers.append(Conv2d(nf_prev, nf, 4, stride=1, padding=padw, bias=use_bias))
        norms.append(norm_layer(norm, nf, act="lrelu"))
        layers.append(Conv2d(nf, 1, 4, stride=1, padding=padw,
                             act_out="sigmoid" if use_sigmoid else None))
        norms.append(nn.Identity())
        self.convs = nn.ModuleList(layers)
        self.norms = nn.ModuleList(norms)
        for c, m in zip(self.convs, self.norms):
            link_norm(c, m)
        link_gate(self.convs[0], [self.convs[1]])

    def forward(self, x):
        for conv, norm in zip(self.convs, self.norms):
            x = norm(conv(x))
        return x


class PixelDiscriminator(nn.Module):
    """1x1 PatchGAN ('pixel' D): BASELINE config 1's discriminator."""

    def __init__(self, input_nc, ndf=64, norm="instance", use_sigmoid=False):
        super().__init__()
        use_bias = norm != "batch"
        self.convs = nn.ModuleList([
            Conv2d(input_nc, ndf, 1, act_out="lrelu"),
            Conv2d(ndf, ndf * 2, 1, bias=use_bias),
            Conv2d(ndf * 2, 1, 1, bias=use_bias, act_out="sigmoid" if use_sigmoid else None),
        ])
        self.norms = nn.ModuleList([nn.Identity(), norm_layer(norm, ndf * 2, act="lrelu"),
                                    nn.Identity()])
        for c, m in zip(self.convs, self.norms):
            link_norm(c, m)
        link_gate(self.convs[0], [self.convs[1]])

    def forward(self, x):
        for conv, norm in zip(self.convs, self.norms):
            x = norm(conv(x))
        return x
