"""Parity against the reference's own module definitions (/root/reference/networks.py).

The reference is imported unmodified with a stand-in ``torchvision`` (not installed here;
only ``models.vgg19(...).features`` and ``transforms`` are touched at import / construction
time, and the stand-in builds torchvision's VGG19 'E' layer list).  Weights are copied
reference -> ours with ``load_state_dict(strict=True)``, so these tests pin checkpoint
key/shape compatibility AND forward numerics (fp32, CPU) of every family-R network.
Skipped when the reference checkout is not mounted (e.g. on the GPU box).
"""
import importlib.util
import os
import sys
import types

import pytest
import torch
import torch.nn as nn

REF = "/root/reference/networks.py"
pytestmark = pytest.mark.skipif(not os.path.exists(REF), reason="reference checkout not mounted")


def _fake_torchvision():
    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")
    transforms = types.ModuleType("torchvision.transforms")

    def vgg19(pretrained=False, **kw):
        cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
               512, 512, 512, 512, "M"]
        layers, cin = [], 3
        for v in cfg:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
                cin = v
        m = nn.Module()
        m.features = nn.Sequential(*layers)
        return m

    models.vgg19 = vgg19
    tv.models = models
    tv.transforms = transforms
    return {"torchvision": tv, "torchvision.models": models, "torchvision.transforms": transforms}


@pytest.fixture(scope="module")
def refnet():
    saved = {k: sys.modules.get(k) for k in ("torchvision", "torchvision.models",
                                             "torchvision.transforms")}
    sys.modules.update(_fake_torchvision())
    try:
        spec = importlib.util.spec_from_file_location("ref_networks", REF)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        yield mod
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def _copy(dst, src):
    sd = src.state_dict()
    assert list(dst.state_dict().keys()) == list(sd.keys())
    for k, v in dst.state_dict().items():
        assert v.shape == sd[k].shape, k
    dst.load_state_dict(sd, strict=True)


def test_expand_network_keys_and_forward(refnet):
    from p2p_pytorch_amd.models import ExpandNetwork
    torch.manual_seed(0)
    r = refnet.ExpandNetwork()
    m = ExpandNetwork()
    _copy(m, r)
    assert len(m.state_dict()) == 169
    x = torch.rand(2, 3, 32, 32) * 2 - 1
    r.train(), m.train()
    yr, ym = r(x), m(x)
    assert torch.allclose(ym, yr, atol=2e-5, rtol=1e-4)
    # BN running stats evolve identically
    assert torch.allclose(m.in1_e.running_mean, r.in1_e.running_mean, atol=1e-6)
    r.eval(), m.eval()
    assert torch.allclose(m(x), r(x), atol=2e-5, rtol=1e-4)


def test_expand_network_grads(refnet):
    from p2p_pytorch_amd.models import ExpandNetwork
    torch.manual_seed(1)
    r = refnet.ExpandNetwork()
    m = ExpandNetwork()
    _copy(m, r)
    x = torch.rand(1, 3, 16, 16) * 2 - 1
    r(x).square().mean().backward()
    m(x).square().mean().backward()
    gr = dict(r.named_parameters())
    for n, p in m.named_parameters():
        assert torch.allclose(p.grad, gr[n].grad, atol=1e-6, rtol=1e-3), n


def test_compression_network(refnet):
    from p2p_pytorch_amd.models import CompressionNetwork
    torch.manual_seed(2)
    r = refnet.CompressionNetwork()
    m = CompressionNetwork()
    _copy(m, r)
    x = torch.rand(2, 3, 32, 32) * 2 - 1
    assert torch.allclose(m(x), r(x), atol=1e-5)


def test_multiscale_discriminator(refnet):
    from p2p_pytorch_amd.models import MultiscaleDiscriminator
    torch.manual_seed(3)
    r = refnet.MultiscaleDiscriminator(6, 64, n_layers=3, norm_layer=None, use_sigmoid=False,
                                       num_D=3, getIntermFeat=True)
    m = MultiscaleDiscriminator(6, 64, n_layers=3, norm_layer=None, use_sigmoid=False, num_D=3,
                                getIntermFeat=True)
    _copy(m, r)
    x = torch.rand(2, 6, 64, 64) * 2 - 1
    outr, outm = r(x), m(x)
    assert len(outr) == len(outm) == 3
    for sr, sm in zip(outr, outm):
        assert len(sr) == len(sm) == 5
        for a, b in zip(sr, sm):
            assert a.shape == b.shape
            assert torch.allclose(b, a, atol=1e-5, rtol=1e-4)
    # spectral-norm u/v were advanced identically by the power iteration
    for (n1, t1), (n2, t2) in zip(r.state_dict().items(), m.state_dict().items()):
        assert n1 == n2
        assert torch.allclose(t1, t2, atol=1e-6), n1


def test_vgg19_slices(refnet):
    from p2p_pytorch_amd.models import Vgg19
    torch.manual_seed(4)
    r = refnet.Vgg19()
    m = Vgg19()
    _copy(m, r)
    x = torch.rand(1, 3, 64, 64) * 2 - 1
    for a, b in zip(r(x), m(x)):
        assert torch.allclose(b, a, atol=1e-4, rtol=1e-4)


def test_define_factories_and_init(refnet):
    from p2p_pytorch_amd.models import define_C, define_D, define_G
    g_ref = refnet.define_G(gpu_id="cpu")
    g = define_G(gpu_id="cpu", verbose=False)
    assert [k for k in g.state_dict()] == [k for k in g_ref.state_dict()]
    d_ref = refnet.define_D(6, 64, "batch", gpu_id="cpu")
    d = define_D(6, 64, "batch", gpu_id="cpu", verbose=False)
    assert [k for k in d.state_dict()] == [k for k in d_ref.state_dict()]
    c_ref = refnet.define_C(gpu_id="cpu")
    c = define_C(gpu_id="cpu", verbose=False)
    assert [k for k in c.state_dict()] == [k for k in c_ref.state_dict()]
    # quirk A8: spectral-norm convs keep PyTorch's default kaiming-uniform init (bounded by
    # 1/sqrt(fan_in)); the plain convs get N(0, 0.02) (unbounded tails)
    for dd in (d, d_ref):
        w = dd.state_dict()["scale0_layer1.0.module.weight_bar"]
        assert w.abs().max() <= 1.0 / (64 * 16) ** 0.5 + 1e-6
        w0 = dd.state_dict()["scale0_layer0.0.weight"]
        assert abs(w0.std().item() - 0.02) < 0.002


def test_scheduler_lambda_rule(refnet):
    from types import SimpleNamespace
    from p2p_pytorch_amd.models import get_scheduler
    opt = SimpleNamespace(lr_policy="lambda", epoch_count=1, niter=3, niter_decay=4,
                          lr_decay_iters=50)
    p1 = [nn.Parameter(torch.zeros(1))]
    p2 = [nn.Parameter(torch.zeros(1))]
    o1 = torch.optim.Adam(p1, lr=1.0)
    o2 = torch.optim.Adam(p2, lr=1.0)
    s1, s2 = get_scheduler(o1, opt), refnet.get_scheduler(o2, opt)
    for _ in range(8):
        s1.step()
        s2.step()
        assert o1.param_groups[0]["lr"] == pytest.approx(o2.param_groups[0]["lr"])


def test_compress_gan_step_matches_reference_loop(refnet):
    """One family-R training iteration: the reference's own loop body (train.py:291-402,
    transcribed with the reference modules; GANLoss' hard-coded CUDA tensor type pointed
    at CPU) vs CompressGANStep on our modules with copied weights -- same losses, same
    updated G / D parameters."""
    from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
    from p2p_pytorch_amd.models import (CompressionNetwork, ExpandNetwork,
                                        MultiscaleDiscriminator, VGGLoss)
    torch.manual_seed(5)
    rg, rd, rc = (refnet.ExpandNetwork(),
                  refnet.MultiscaleDiscriminator(6, 64, 3, None, False, 3, True),
                  refnet.CompressionNetwork())
    g, d, c = ExpandNetwork(), MultiscaleDiscriminator(6, 64, 3, None, False, 3, True), \
        CompressionNetwork()
    _copy(g, rg)
    _copy(d, rd)
    _copy(c, rc)
    rvgg = refnet.VGGLoss("cpu")
    vgg = VGGLoss()
    _copy(vgg.vgg, rvgg.vgg)
    a = torch.rand(1, 3, 32, 32) * 2 - 1
    b = torch.rand(1, 3, 32, 32) * 2 - 1

    # ---- reference loop body
    def compress(t, bit):
        m = 2 ** bit - 1
        return torch.round(torch.clamp(t, 0.0, 1.0) * m) / m

    gan = refnet.GANLoss()
    gan.Tensor = torch.FloatTensor
    l1 = nn.L1Loss()
    opt_g = torch.optim.Adam(rg.parameters(), lr=2e-4, betas=(0.5, 0.999))
    opt_d = torch.optim.Adam(rd.parameters(), lr=2e-4, betas=(0.5, 0.999))
    compressed = compress(rc(b), 3)
    fake_b = rg(compressed.detach())
    pred_fake = rd.forward(torch.cat((a, fake_b.detach()), 1))
    loss_d_fake = gan(pred_fake, False)
    pred_real = rd.forward(torch.cat((a, b.detach()), 1))
    loss_d_real = gan(pred_real, True)
    loss_d = (loss_d_fake + loss_d_real) * 0.5
    pred_fake = rd.forward(torch.cat((a, fake_b), 1))
    loss_g_gan = gan(pred_fake, True)
    feat = 0
    for i in range(3):
        for j in range(len(pred_fake[i]) - 1):
            feat += (1.0 / 3) * (4.0 / 4) * l1(pred_fake[i][j], pred_real[i][j].detach()) * 10.0
    content = rvgg(fake_b, b) * 10.0
    tv = torch.mean(torch.abs(fake_b[:, :, :, :-1] - fake_b[:, :, :, 1:])) + \
        torch.mean(torch.abs(fake_b[:, :, :-1, :] - fake_b[:, :, 1:, :]))
    loss_g = loss_g_gan + feat + content + tv
    opt_g.zero_grad()
    loss_g.backward()
    opt_g.step()
    opt_d.zero_grad()
    loss_d.backward()
    opt_d.step()
    locc = torch.nn.functional.mse_loss(rg(compressed), b) + rvgg(compressed, b) * 10.0

    # ---- ours
    step = CompressGANStep(g, d, c, vgg=vgg)
    out = step.step(a, b)
    assert out["D"].item() == pytest.approx(loss_d.item(), rel=1e-4)
    assert out["G"].item() == pytest.approx(loss_g.item(), rel=1e-4)
    assert out["C"].item() == pytest.approx(locc.item(), rel=1e-4)
    for (n1, t1), (n2, t2) in zip(rg.state_dict().items(), g.state_dict().items()):
        assert n1 == n2
        assert torch.allclose(t1.float(), t2.float(), atol=1e-5, rtol=1e-4), n1
    for (n1, t1), (n2, t2) in zip(rd.state_dict().items(), d.state_dict().items()):
        assert torch.allclose(t1, t2, atol=1e-5, rtol=1e-4), n1


def test_networks_nlayer_discriminator_is_reference_class(refnet):
    """``networks.NLayerDiscriminator`` takes the reference signature and builds the
    spectral-norm PatchGAN with the reference's keys (networks.py:758-806)."""
    import networks
    torch.manual_seed(0)
    ours = networks.NLayerDiscriminator(6, 64, 3, None, False, True)
    ref = refnet.NLayerDiscriminator(6, 64, 3, None, False, True)
    assert list(ours.state_dict()) == list(ref.state_dict())
    for (k, a), (_, b) in zip(ours.state_dict().items(), ref.state_dict().items()):
        assert a.shape == b.shape, k
    ours.load_state_dict(ref.state_dict())
    x = torch.rand(1, 6, 32, 32) * 2 - 1
    with torch.no_grad():
        yo, yr = ours(x), ref(x)
    assert len(yo) == len(yr) == 5
    for a, b in zip(yo, yr):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4)
    assert networks.PatchGANDiscriminator is not networks.NLayerDiscriminator
