"""Packed-image layer kernels (csrc/image.hip, halo_conv.hip, conv_dev.h d2s epilogue)
against fp32 PyTorch references of the same ops, for both union-GEMM implementations
(16 columns: halo-tile kernel; 32 columns: implicit-GEMM glds tile).

  * image forward: (A | fake) packed pixels with fake = tanh(ConvT4x4s2p1(relu(cat(skip,
    u))) + b), A copied exactly, pad channels zero; the L1 term scale * sum|fake - B|;
  * head gradient: slots 0..2 = (dX[3..5] + scale * sign(f - b)) * (1 - f^2) with dX the
    input gradient of the 6-channel 4x4 s2 p1 conv.
"""
import pytest
import torch
import torch.nn.functional as F

from p2p_pytorch_amd import _native
from p2p_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf(x):
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


@pytest.fixture(autouse=True, scope="module")
def _native_backend():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()


@pytest.mark.parametrize("rows", [16, 32])
@pytest.mark.parametrize("N,H", [(2, 64), (1, 40)])
def test_image_forward(rows, N, H):
    g = torch.Generator(device=DEV).manual_seed(1)
    skip = bf(torch.randn(N, 64, H, H, device=DEV, generator=g))
    u = bf(torch.randn(N, 64, H, H, device=DEV, generator=g))
    w = torch.randn(128, 3, 4, 4, device=DEV, generator=g) * 0.05
    b = torch.randn(3, device=DEV, generator=g) * 0.1
    A = bf(torch.rand(N, 3, 2 * H, 2 * H, device=DEV, generator=g) * 2 - 1)
    B = bf(torch.rand(N, 3, 2 * H, 2 * H, device=DEV, generator=g) * 2 - 1)
    dd = torch.empty(2 * N, 8, 2 * H, 2 * H, device=DEV, dtype=torch.bfloat16,
                     memory_format=torch.channels_last)
    hip.P().pad_channels_into(A, B, dd.narrow(0, N, N))
    img, bu = hip.P().union_weight(w, 0, 3, rows, 128, b)
    scale = 7.0 / (N * 3 * 4 * H * H)
    l1 = hip.P().conv_d2s(skip, u, img, bu, 1, hip.ACT["tanh"], 1, dd.narrow(0, 0, N),
                          dd.narrow(0, N, N), None, scale)
    ref = torch.tanh(F.conv_transpose2d(F.relu(torch.cat((skip, u), 1).float()), w, b, 2, 1))
    out = dd[:N].float()
    assert torch.equal(out[:, 0:3], A.float())
    assert (out[:, 6:8] == 0).all()
    assert rel(out[:, 3:6], ref) < 2e-2
    l1_ref = scale * (out[:, 3:6] - B.float()).abs().sum()
    assert abs(l1.item() - l1_ref.item()) <= 1e-4 * abs(l1_ref.item())


@pytest.mark.parametrize("rows", [16, 32])
def test_head_gradient(rows):
    N, H = 2, 64
    g = torch.Generator(device=DEV).manual_seed(2)
    gy = bf(torch.randn(N, 64, H, H, device=DEV, generator=g))
    w = torch.randn(64, 6, 4, 4, device=DEV, generator=g) * 0.05
    af = bf(torch.rand(N, 8, 2 * H, 2 * H, device=DEV, generator=g) * 1.6 - 0.8)
    ab = bf(torch.rand(N, 8, 2 * H, 2 * H, device=DEV, generator=g) * 2 - 1)
    img, _ = hip.P().union_weight(w, 3, 3, rows, 64, None)
    zb = torch.zeros(rows, device=DEV)
    dz = torch.empty_like(af, memory_format=torch.channels_last)
    scale = 0.01
    hip.P().conv_d2s(gy, None, img, zb, 0, 0, 2, dz, ab, af, scale)
    dx = F.conv_transpose2d(gy.float(), w, None, 2, 1)[:, 3:6]
    f, t = af.float()[:, 3:6], ab.float()[:, 3:6]
    ref = (dx + scale * torch.sign(f - t)) * (1 - f * f)
    got = dz.float()
    assert (got[:, 3:8] == 0).all()
    assert rel(got[:, 0:3], ref) < 2e-2


@pytest.mark.parametrize("rows", [16, 32])
def test_head_gradient_device_weight(rows):
    """The L1 sign term scaled by a device scalar (dL/dl1 written by the loss's gradient tap)."""
    N, H = 2, 32
    g = torch.Generator(device=DEV).manual_seed(3)
    gy = bf(torch.randn(N, 64, H, H, device=DEV, generator=g))
    w = torch.randn(64, 6, 4, 4, device=DEV, generator=g) * 0.05
    af = bf(torch.rand(N, 8, 2 * H, 2 * H, device=DEV, generator=g) * 1.6 - 0.8)
    ab = bf(torch.rand(N, 8, 2 * H, 2 * H, device=DEV, generator=g) * 2 - 1)
    img, _ = hip.P().union_weight(w, 3, 3, rows, 64, None)
    zb = torch.zeros(rows, device=DEV)
    dz = torch.empty_like(af, memory_format=torch.channels_last)
    scale, wdev = 0.01, torch.tensor([-2.5], device=DEV)
    hip.P().conv_d2s(gy, None, img, zb, 0, 0, 2, dz, ab, af, scale, wdev)
    dx = F.conv_transpose2d(gy.float(), w, None, 2, 1)[:, 3:6]
    f, t = af.float()[:, 3:6], ab.float()[:, 3:6]
    ref = (dx - 2.5 * scale * torch.sign(f - t)) * (1 - f * f)
    assert rel(dz.float()[:, 0:3], ref) < 2e-2


def _g_grads(G, D, A, B, packed, tap, w_gan, w_l1, lam):
    from p2p_pytorch_amd.models import GANLoss
    from p2p_pytorch_amd.ops import l1
    crit = GANLoss(gan_mode="vanilla")
    hip.begin_step()
    hip.prepare_weights(G, D)
    G.zero_grad(set_to_none=True)
    N, _, H, W = A.shape
    if packed:
        dd = torch.empty(2 * N, 8, H, W, device=DEV, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        hip.P().pad_channels_into(A, B, dd.narrow(0, N, N))
        dd._p2p_packed = (3, 3)
        fake, loss_l1 = G.forward_packed(dd, lam / float(N * 3 * H * W))
        gan = crit(D(fake), True)
        loss = w_gan * gan + w_l1 * (hip.head_l1_tap(loss_l1) if tap else loss_l1)
    else:
        fake = G(A)
        gan = crit(D((A, fake)), True)
        loss = w_gan * gan + w_l1 * l1(fake, B) * lam
    loss.backward()
    return {n: p.grad.detach().float().clone() for n, p in G.named_parameters()}


@pytest.mark.parametrize("tap", [True, False])
def test_packed_head_honours_loss_weights(tap):
    """W5: the packed image head's fused L1 gradient follows the loss's weighting (tapped:
    the weight reaches the fused dgrad on the device; untapped: the head's backward adds the
    term) -- G's gradients match the unpacked path under a non-unit recomposition."""
    from p2p_pytorch_amd.models import define_D, define_G
    from p2p_pytorch_amd.models.pix2pix import UnetGenerator
    torch.manual_seed(0)
    G = define_G(netG="unet_64", gpu_id=DEV, verbose=False, use_dropout=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=DEV, verbose=False)
    for p in D.parameters():
        p.requires_grad_(False)
    g = torch.Generator(device=DEV).manual_seed(4)
    A = bf(torch.rand(2, 3, 64, 64, device=DEV, generator=g) * 2 - 1)
    B = bf(torch.rand(2, 3, 64, 64, device=DEV, generator=g) * 2 - 1)
    assert isinstance(G, UnetGenerator) and G.packed_ok(A)
    ref = _g_grads(G, D, A, B, False, tap, 0.5, 3.0, 100.0)
    got = _g_grads(G, D, A, B, True, tap, 0.5, 3.0, 100.0)
    for n in ref:
        assert rel(got[n], ref[n]) < 5e-2, n
