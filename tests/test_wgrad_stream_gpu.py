"""Weight gradients on the side stream (ops/hip.py ``wgrad_overlap``) change no bit.

The side stream only moves WHERE each wgrad kernel runs; every kernel and operand is the
same, so with ordered split-K reductions (``set_deterministic(True)``) the parameters after
K steps must be bitwise those of the all-on-one-stream step -- eager, and under hipGraph
replay (the capture records the fork/join).  A missing stream join or an operand recycled
under the side stream shows up as a mismatch.
"""
import pytest
import torch

import p2p_pytorch_amd as p2p
from p2p_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu

STEPS = 3


def _build(net="unet_256"):
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    dev = torch.device("cuda")
    hip.reset_rng(0)
    torch.manual_seed(0)
    G = define_G(netG=net, gpu_id=dev, verbose=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
    return Pix2PixStep(G, D), G, D


def _data(n, size):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    return [[(torch.rand(n, 3, size, size, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
             .contiguous(memory_format=torch.channels_last) for _ in range(2)] for _ in range(STEPS)]


def _params(G, D):
    return torch.cat([p.detach().reshape(-1) for p in list(G.parameters()) + list(D.parameters())])


def _run(monkeypatch, flag, graph, net="unet_256", n=8, size=256):
    from p2p_pytorch_amd.engine.graph import CapturedStep
    monkeypatch.setenv("P2P_WGRAD_STREAM", flag)
    step, G, D = _build(net)
    data = _data(n, size)
    if graph:
        cap = CapturedStep(step.step, *data[0])
        for a, b in data:
            losses = cap(a, b)
    else:
        for a, b in data:
            losses = step.step(a, b)
    torch.cuda.synchronize()
    return {k: v.item() for k, v in losses.items()}, _params(G, D)


@pytest.mark.parametrize("graph", [False, True])
def test_wgrad_side_stream_bitwise(monkeypatch, graph):
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    try:
        l0, p0 = _run(monkeypatch, "0", False)
        l1, p1 = _run(monkeypatch, "1", graph)
    finally:
        p2p.set_deterministic(False)
    assert l0 == l1
    assert torch.equal(p0, p1)


def test_wgrad_side_stream_repeat_weight(monkeypatch):
    """A weight used twice in one backward (two gradients, autograd adds them on the compute
    stream): the first must be joined before the add -- same result as one stream."""
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    dev = torch.device("cuda")
    try:
        out = []
        for flag in ("0", "1"):
            monkeypatch.setenv("P2P_WGRAD_STREAM", flag)
            torch.manual_seed(1)
            conv = torch.nn.Conv2d(64, 128, 4, 2, 1).to(dev)
            x = (torch.randn(16, 64, 64, 64, device=dev)).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            from p2p_pytorch_amd import ops
            with hip.wgrad_overlap(dev):
                y1 = ops.conv2d(x, conv.weight, conv.bias, stride=2, padding=1)
                y2 = ops.conv2d(x * 0.5, conv.weight, conv.bias, stride=2, padding=1)
                (y1.float().square().mean() + y2.float().abs().mean()).backward()
            torch.cuda.synchronize()
            out.append(conv.weight.grad.clone())
        assert torch.equal(out[0], out[1])
    finally:
        p2p.set_deterministic(False)


def _one_conv_grad(monkeypatch, flag, kind):
    """conv weight gradient with the side stream on/off for a weight AccumulateGrad cannot
    steal: ``nonleaf`` (weight = w * 0.5 feeds the conv, MulBackward reads gw), ``accum`` (the
    leaf already has a gradient, autograd adds into it)."""
    from p2p_pytorch_amd import ops
    dev = torch.device("cuda")
    monkeypatch.setenv("P2P_WGRAD_STREAM", flag)
    torch.manual_seed(2)
    conv = torch.nn.Conv2d(64, 128, 4, 2, 1).to(dev)
    x = torch.randn(16, 64, 64, 64, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if kind == "accum":
        conv.weight.grad = torch.full_like(conv.weight, 0.25)
    with hip.wgrad_overlap(dev):
        w = conv.weight * 0.5 if kind == "nonleaf" else conv.weight
        y = ops.conv2d(x, w, conv.bias, stride=2, padding=1)
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    return conv.weight.grad.clone()


@pytest.mark.parametrize("kind", ["nonleaf", "accum"])
def test_wgrad_side_stream_unstealable_grad(monkeypatch, kind):
    """the side stream is bypassed when autograd would read gw on the compute stream
    (non-leaf weight, existing gradient) -- bitwise the one-stream result."""
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    try:
        g0 = _one_conv_grad(monkeypatch, "0", kind)
        g1 = _one_conv_grad(monkeypatch, "1", kind)
    finally:
        p2p.set_deterministic(False)
    assert torch.isfinite(g0).all()
    assert torch.equal(g0, g1)


def _run_ref_family(monkeypatch, flag):
    from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
    from p2p_pytorch_amd.models import define_C, define_D, define_G
    dev = torch.device("cuda")
    monkeypatch.setenv("P2P_WGRAD_STREAM", flag)
    hip.reset_rng(0)
    torch.manual_seed(0)
    G = define_G(netG="expand", gpu_id=dev, verbose=False)
    D = define_D(6, 64, gpu_id=dev, netD="multiscale", verbose=False)
    C = define_C(gpu_id=dev, verbose=False)
    step = CompressGANStep(G, D, C)
    g = torch.Generator(device=dev).manual_seed(5)
    for _ in range(2):
        a, b = [(torch.rand(2, 3, 128, 128, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
                .contiguous(memory_format=torch.channels_last) for _ in range(2)]
        losses = step.step(a, b)
    torch.cuda.synchronize()
    return ({k: float(v) for k, v in losses.items()},
            torch.cat([p.detach().reshape(-1) for p in list(G.parameters()) + list(D.parameters())]))


def test_wgrad_side_stream_ref_family_bitwise(monkeypatch):
    """The reference family's step (CompressGANStep) with its G weight gradients on the side
    stream is bitwise the one-stream step."""
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    try:
        l0, p0 = _run_ref_family(monkeypatch, "0")
        l1, p1 = _run_ref_family(monkeypatch, "1")
    finally:
        p2p.set_deterministic(False)
    assert l0 == l1
    assert torch.equal(p0, p1)
