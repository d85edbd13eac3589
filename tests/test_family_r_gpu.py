"""The reference-family training step on the GPU (HIP kernels, bf16 activations) against
the same step on the CPU fp32 oracle path, at 64x64 (/root/reference/train.py:291-402).

lr = 0 keeps the parameters fixed, so what is compared is everything one step computes:
the seven logged losses, every G and D gradient the optimizers would apply, the BatchNorm
running statistics (advanced by both G forwards) and the spectral-norm u / v vectors
(advanced by all three D forwards).  A second run with the default lr checks that the
native update moves each parameter in the oracle's direction.

Bounds (bf16 activations against fp32): losses 3 %, each gradient tensor 10 % of its own
max-abs (absolute floor 1e-3 of the largest gradient in the network: BN-fed conv biases
have an exactly-zero true gradient), running stats 3 %.
"""
import copy

import pytest
import torch

import p2p_pytorch_amd as p2p

pytestmark = pytest.mark.gpu


def _nets():
    from p2p_pytorch_amd.models import VGGLoss, define_C, define_D, define_G
    torch.manual_seed(11)
    G = define_G(gpu_id="cpu", verbose=False)
    D = define_D(6, 64, gpu_id="cpu", verbose=False)
    C = define_C(gpu_id="cpu", verbose=False)
    vgg = VGGLoss()
    return G, D, C, vgg


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


def _run_pair(lr):
    from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
    p2p.set_backend("native")
    G, D, C, vgg = _nets()
    Gg, Dg, Cg, vggg = (copy.deepcopy(m).cuda() for m in (G, D, C, vgg))
    g = torch.Generator().manual_seed(5)
    a = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    b = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    cpu = CompressGANStep(G, D, C, lr=lr, vgg=vgg)
    out_c = cpu.step(a, b)
    gpu = CompressGANStep(Gg, Dg, Cg, lr=lr, vgg=vggg)

    def dev(x):
        return x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    out_g = gpu.step(dev(a), dev(b))
    torch.cuda.synchronize()
    return (G, D, C), (Gg, Dg, Cg), out_c, out_g


def test_family_r_step_gpu_matches_cpu_oracle():
    (G, D, _), (Gg, Dg, _), out_c, out_g = _run_pair(lr=0.0)
    for k in out_c:
        ref, got = float(out_c[k]), float(out_g[k])
        assert abs(got - ref) <= 3e-2 * abs(ref) + 1e-4, (k, got, ref)
    bad = []
    for net, netg in ((G, Gg), (D, Dg)):
        grads = [(n, p.grad, pg.grad) for (n, p), (_, pg) in
                 zip(net.named_parameters(), netg.named_parameters()) if p.grad is not None]
        assert grads
        gscale = max(gr.abs().max().item() for _, gr, _ in grads)
        for n, gr, gg in grads:
            assert gg is not None and torch.isfinite(gg).all(), n
            err = (gg.cpu().float() - gr.float()).abs().max().item()
            if err > 0.10 * gr.abs().max().item() and err > 1e-3 * gscale:
                bad.append((n, err, gr.abs().max().item()))
    assert not bad, bad
    for (n, t), (_, tg) in zip(G.named_buffers(), Gg.named_buffers()):
        if t.dtype.is_floating_point:
            assert _rel(tg.cpu(), t) < 3e-2, n
    for (n, t), (_, tg) in zip(D.named_parameters(), Dg.named_parameters()):
        if n.endswith("_u") or n.endswith("_v"):
            assert _rel(tg.cpu(), t) < 3e-2, n


def test_family_r_update_direction_matches_oracle():
    nets, nets_g, _, _ = _run_pair(lr=2e-4)
    fresh = _nets()
    agree = total = 0
    for net0, net, netg in zip(fresh, nets, nets_g):
        for p0, p, pg in zip(net0.parameters(), net.parameters(), netg.parameters()):
            d_ref = (p.detach() - p0.detach()).sign()
            d_gpu = (pg.detach().cpu() - p0.detach()).sign()
            moved = d_ref != 0
            agree += int(((d_ref == d_gpu) & moved).sum())
            total += int(moved.sum())
    assert total > 0
    assert agree / total > 0.9, agree / total
