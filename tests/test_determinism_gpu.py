"""Bitwise repeatability: with ``set_deterministic(True)`` two training
steps from the same init and data give bit-identical losses and parameters -- including
the split-K conv layers (U-Net bottleneck), whose default fp32-atomic reduction is
order-dependent."""
import pytest
import torch

import p2p_pytorch_amd as p2p
from p2p_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu


def _run():
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    dev = torch.device("cuda")
    hip.reset_rng(0)                        # same dropout stream for both runs
    G = define_G(netG="unet_256", gpu_id=dev, verbose=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
    step = Pix2PixStep(G, D)
    g = torch.Generator(device=dev).manual_seed(3)
    A = (torch.rand(2, 3, 256, 256, device=dev, generator=g) * 2 - 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    B = (torch.rand(2, 3, 256, 256, device=dev, generator=g) * 2 - 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    for _ in range(2):
        losses = step.step(A, B)
    torch.cuda.synchronize()
    params = torch.cat([p.detach().reshape(-1) for p in list(G.parameters()) + list(D.parameters())])
    return {k: v.item() for k, v in losses.items()}, params


def test_deterministic_mode_is_bitwise_repeatable():
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    try:
        l1, p1 = _run()
        l2, p2 = _run()
    finally:
        p2p.set_deterministic(False)
    assert l1 == l2
    assert torch.equal(p1, p2)
