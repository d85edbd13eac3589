"""Model-zoo tests on CPU (fp32 oracle path).

The flat U-Net / PatchGAN store activations pre-applied by their producers (see
models/pix2pix.py); these tests pin that they are numerically the canonical pix2pix
architectures: a textbook recursive U-Net (skip-block nesting, LeakyReLU -> conv -> norm
down, ReLU -> convT -> norm up, cat(x, sub(x))) and a textbook Sequential PatchGAN are
built here, weights are copied, and outputs / input gradients are compared.
"""
import pytest
import torch
import torch.nn as nn

from p2p_pytorch_amd.models import (NLayerDiscriminator, PixelDiscriminator, UnetGenerator,
                                    count_params, define_D, define_G)


class _Block(nn.Module):
    """Canonical pix2pix UnetSkipConnectionBlock (instance norm, use_bias=True)."""

    def __init__(self, outer_nc, inner_nc, input_nc=None, sub=None, outermost=False,
                 innermost=False, use_dropout=False):
        super().__init__()
        self.outermost = outermost
        input_nc = input_nc or outer_nc
        self.downconv = nn.Conv2d(input_nc, inner_nc, 4, 2, 1, bias=True)
        self.downnorm = nn.InstanceNorm2d(inner_nc)
        self.upnorm = nn.InstanceNorm2d(outer_nc)
        if outermost:
            self.upconv = nn.ConvTranspose2d(inner_nc * 2, outer_nc, 4, 2, 1)
            down = [self.downconv]
            up = [nn.ReLU(), self.upconv, nn.Tanh()]
            model = down + [sub] + up
        elif innermost:
            self.upconv = nn.ConvTranspose2d(inner_nc, outer_nc, 4, 2, 1, bias=True)
            down = [nn.LeakyReLU(0.2), self.downconv]
            up = [nn.ReLU(), self.upconv, self.upnorm]
            model = down + up
        else:
            self.upconv = nn.ConvTranspose2d(inner_nc * 2, outer_nc, 4, 2, 1, bias=True)
            down = [nn.LeakyReLU(0.2), self.downconv, self.downnorm]
            up = [nn.ReLU(), self.upconv, self.upnorm]
            model = down + [sub] + up + ([nn.Dropout(0.5)] if use_dropout else [])
        self.model = nn.Sequential(*model)

    def forward(self, x):
        if self.outermost:
            return self.model(x)
        return torch.cat([x, self.model(x)], 1)


def _canonical_unet(num_downs, ngf=8, input_nc=3, output_nc=3):
    blocks = []
    b = _Block(ngf * 8, ngf * 8, innermost=True)
    blocks.append(b)
    for _ in range(num_downs - 5):
        b = _Block(ngf * 8, ngf * 8, sub=b)
        blocks.append(b)
    b = _Block(ngf * 4, ngf * 8, sub=b)
    blocks.append(b)
    b = _Block(ngf * 2, ngf * 4, sub=b)
    blocks.append(b)
    b = _Block(ngf, ngf * 2, sub=b)
    blocks.append(b)
    b = _Block(output_nc, ngf, input_nc=input_nc, sub=b, outermost=True)
    blocks.append(b)
    return b, blocks[::-1]  # outermost first


def _copy_unet(flat: UnetGenerator, blocks):
    with torch.no_grad():
        for i, blk in enumerate(blocks):
            flat.downs[i].weight.copy_(blk.downconv.weight)
            flat.downs[i].bias.copy_(blk.downconv.bias)
            flat.ups[i].weight.copy_(blk.upconv.weight)
            flat.ups[i].bias.copy_(blk.upconv.bias)


@pytest.mark.parametrize("num_downs", [5, 6, 7])
def test_flat_unet_equals_canonical(num_downs):
    torch.manual_seed(0)
    ngf = 8
    canon, blocks = _canonical_unet(num_downs, ngf)
    flat = UnetGenerator(3, 3, num_downs, ngf, "instance", use_dropout=False)
    _copy_unet(flat, blocks)
    s = 2 ** num_downs
    x = torch.randn(2, 3, s, s, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    y1 = canon(x)
    y2 = flat(x2)
    assert torch.allclose(y1, y2, atol=1e-5)
    g = torch.randn_like(y1)
    y1.backward(g)
    y2.backward(g)
    assert torch.allclose(x.grad, x2.grad, atol=1e-5, rtol=1e-4)
    for i, blk in enumerate(blocks):
        assert torch.allclose(blk.downconv.weight.grad, flat.downs[i].weight.grad, atol=1e-5,
                              rtol=1e-3)
        assert torch.allclose(blk.upconv.weight.grad, flat.ups[i].weight.grad, atol=1e-5,
                              rtol=1e-3)


def test_patchgan_equals_canonical():
    torch.manual_seed(1)
    d = NLayerDiscriminator(6, 16, 3, "instance")
    ndf = 16
    seq = [nn.Conv2d(6, ndf, 4, 2, 1), nn.LeakyReLU(0.2)]
    nf = ndf
    for k in range(1, 3):
        nf_prev, nf = nf, ndf * min(2 ** k, 8)
        seq += [nn.Conv2d(nf_prev, nf, 4, 2, 1), nn.InstanceNorm2d(nf), nn.LeakyReLU(0.2)]
    nf_prev, nf = nf, ndf * 8
    seq += [nn.Conv2d(nf_prev, nf, 4, 1, 1), nn.InstanceNorm2d(nf), nn.LeakyReLU(0.2),
            nn.Conv2d(nf, 1, 4, 1, 1)]
    canon = nn.Sequential(*seq)
    convs = [m for m in canon if isinstance(m, nn.Conv2d)]
    with torch.no_grad():
        for a, b in zip(d.convs, convs):
            a.weight.copy_(b.weight)
            a.bias.copy_(b.bias)
    x = torch.randn(2, 6, 64, 64)
    assert torch.allclose(d(x), canon(x), atol=1e-5)
    # receptive field 70 -> a 64x64 input gives 6x6 patches (pad 1)
    assert d(x).shape == (2, 1, 6, 6)
    # virtual concat input == materialised concat
    a, b = x[:, :3], x[:, 3:]
    assert torch.allclose(d((a, b)), d(x), atol=1e-6)


def test_param_counts_north_star():
    g = define_G(netG="unet_256", gpu_id="cpu", verbose=False)
    d = define_D(6, 64, norm="instance", netD="basic", gpu_id="cpu", verbose=False)
    assert count_params(g) == 54_409_603
    assert count_params(d) == 2_767_809
    assert g.num_downs == 8


def test_plumbing_config_shapes():
    # BASELINE config 1: 64x64, 4-layer U-Net + 1x1 (pixel) PatchGAN
    g = define_G(netG="unet_4", gpu_id="cpu", verbose=False)
    d = define_D(6, 64, norm="instance", netD="pixel", gpu_id="cpu", verbose=False)
    x = torch.rand(1, 3, 64, 64) * 2 - 1
    y = g(x)
    assert y.shape == x.shape and y.abs().max() <= 1.0
    p = d((x, y))
    assert p.shape == (1, 1, 64, 64)
    assert isinstance(d, PixelDiscriminator)


def test_dropout_levels():
    g = UnetGenerator(3, 3, 8, 64, "instance", use_dropout=True)
    assert g.drop_levels == {4, 5, 6}
    g7 = UnetGenerator(3, 3, 7, 64, "instance", use_dropout=True)
    assert g7.drop_levels == {4, 5}


def test_vgg_tap_fusion_flags_and_cpu_loss_unchanged():
    """VGGLoss turns on tap fusion (HIP path: tap relu' + parked L1 gradient added in the next
    slice's conv); on the CPU oracle the flags are inert, so the loss and its gradient equal
    the plain VGG19 perceptual loss."""
    import torch
    from p2p_pytorch_amd.models.vgg import VGGLoss, Vgg19
    torch.manual_seed(0)
    loss_f = VGGLoss()
    feats = loss_f.vgg._feats
    assert loss_f.vgg.tap_fusion
    for prod, cons in Vgg19._TAPS:
        assert feats[prod].out_gated
        if cons is not None:
            assert feats[cons].skip_grad == "take" and feats[cons].grad_gate == "relu"
    plain = Vgg19()
    plain.load_state_dict(loss_f.vgg.state_dict())
    assert not plain.tap_fusion and not plain._feats[0].out_gated
    x = (torch.rand(1, 3, 32, 32) * 2 - 1).requires_grad_(True)
    y = torch.rand(1, 3, 32, 32) * 2 - 1
    l1 = loss_f(x, y)
    g1, = torch.autograd.grad(l1, x)
    fx, fy = plain(x), plain(y)
    l2 = sum(w * (a - b.detach()).abs().mean() for w, a, b in zip(VGGLoss.weights, fx, fy))
    g2, = torch.autograd.grad(l2, x)
    assert torch.allclose(l1, l2, rtol=1e-5, atol=1e-6)
    assert torch.allclose(g1, g2, rtol=1e-4, atol=1e-7)
    # the target features reused across losses give the same value
    fyc = loss_f.target_features(y)
    assert torch.allclose(loss_f(x, y, fy=fyc), l1)


def test_lincomb_n_torch_path_matches_expression():
    """ops.lincomb_n off the native path is the plain weighted sum in term order (the
    reference's own expression order: bitwise on CPU) and differentiates like it."""
    import torch
    from p2p_pytorch_amd import ops
    ts = [torch.tensor(v, requires_grad=True) for v in (0.3, -1.7, 2.5)]
    ws = [1.0, 10.0, 0.25]
    out = ops.lincomb_n(ts, ws)
    ref_ = 0 + 1.0 * ts[0] + 10.0 * ts[1] + 0.25 * ts[2]
    assert torch.equal(out, ref_)
    out.backward()
    assert [t.grad.item() for t in ts] == ws
