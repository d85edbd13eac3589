"""The reference-family training step on the GPU (HIP kernels, bf16 activations) against
the same step on the CPU fp32 oracle path, at 64x64 (/root/reference/train.py:291-402).

lr = 0 keeps the parameters fixed, so what is compared is everything one step computes:
the seven logged losses, every G and D gradient the optimizers would apply, the BatchNorm
running statistics (advanced by both G forwards) and the spectral-norm u / v vectors
(advanced by all three D forwards).  A second run with the default lr checks that the
native update moves each parameter in the oracle's direction.

Per-dtype bounds: the same step in stock PyTorch bf16 autocast on the GPU (the eager
baseline) measures how far bf16 arithmetic alone moves each quantity from the fp32
oracle; the native step may be at most 2x that far (+1 % of the quantity's scale) --
losses, every gradient tensor (absolute floor 1e-3 of the network's largest gradient:
BN-fed conv biases have an exactly-zero true gradient), running stats and u / v.
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


_COND = {}


class _PReLUConditioning:
    """Wraps the oracle's PReLU (ops.reference.prelu) for one step and sums |dy * x| over the
    negative inputs of every site: S, the absolute mass of the cancelling sum that is the
    shared slope's gradient (sum dy * x over x <= 0).  kappa = S / |gradient| is its condition
    number: bf16 errors of relative size e in the dy / x feeding the sum move it by ~e * S."""

    def __enter__(self):
        from p2p_pytorch_amd.ops import reference as R
        self._mod, self._orig, self.S = R, R.prelu, 0.0

        def prelu(x, w):
            y = self._orig(x, w)
            if y.requires_grad:
                xd = x.detach()

                def hook(gy):
                    self.S += float(((gy * xd) * (xd <= 0)).abs().sum())
                y.register_hook(hook)
            return y
        R.prelu = prelu
        return self

    def __exit__(self, *exc):
        self._mod.prelu = self._orig


class _NativeSlopeTerms:
    """The native step's own slope-gradient terms: at every BN + shared-PReLU site of the
    native G (``BatchNorm2d(..., prelu=G.relu.weight)``: BN, PReLU and, backward, the slope
    gradient reduced in the norm's partial-sum pass) the fused output y = prelu(z) and its
    incoming gradient dy are captured, and sum_{y <= 0} dy * y / w (= dy * z over z <= 0) is
    accumulated in fp64 -- the value the kernels' fp32 reduction must reproduce from the same
    bf16 tensors, whatever the rest of the network's bf16 rounding did to dy."""

    def __init__(self, G):
        self.G, self.sum, self.abs, self.sites, self.hs = G, 0.0, 0.0, 0, []

    def __enter__(self):
        from p2p_pytorch_amd.models.layers import BatchNorm2d
        pw = self.G.relu.weight

        def fwd(mod, args, kwargs, out):
            if kwargs.get("prelu") is pw and out.requires_grad:
                self.sites += 1
                w = float(pw.detach())
                yd = out.detach().double()

                def hook(gy):
                    t = gy.detach().double() * yd / w * (yd <= 0)
                    self.sum += float(t.sum())
                    self.abs += float(t.abs().sum())
                out.register_hook(hook)
        for m in self.G.modules():
            if isinstance(m, BatchNorm2d):
                self.hs.append(m.register_forward_hook(fwd, with_kwargs=True))
        return self

    def __exit__(self, *exc):
        for h in self.hs:
            h.remove()


def _run_pair(lr, eager_bf16=False):
    from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
    p2p.set_backend("native")
    G, D, C, vgg = _nets()
    Gg, Dg, Cg, vggg = (copy.deepcopy(m).cuda() for m in (G, D, C, vgg))
    Ge, De, Ce, vgge = (copy.deepcopy(m).cuda() for m in (G, D, C, vgg))
    g = torch.Generator().manual_seed(5)
    a = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    b = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    cpu = CompressGANStep(G, D, C, lr=lr, vgg=vgg)
    with _PReLUConditioning() as cond:
        out_c = cpu.step(a, b)
    _COND["slope_abs_sum"] = cond.S
    gpu = CompressGANStep(Gg, Dg, Cg, lr=lr, vgg=vggg)

    def dev(x):
        return x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    p2p.set_deterministic(True)          # ordered split-K: a repeatable native result
    try:
        with _NativeSlopeTerms(Gg) as terms:
            out_g = gpu.step(dev(a), dev(b))
    finally:
        p2p.set_deterministic(False)
    _COND["native_terms"] = (terms.sum, terms.abs, terms.sites)
    out_e = None
    if eager_bf16:            # stock PyTorch kernels, bf16 autocast: the dtype's own error
        p2p.set_backend("torch")
        try:
            eager = CompressGANStep(Ge, De, Ce, lr=lr, vgg=vgge)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out_e = eager.step(a.cuda(), b.cuda())
        finally:
            p2p.set_backend("native")
    torch.cuda.synchronize()
    return (G, D, C), (Gg, Dg, Cg), (Ge, De, Ce), out_c, out_g, out_e


def _record(tag, rows):
    import json
    import os
    if os.path.isdir("gpurun_out"):
        with open("gpurun_out/bounds.jsonl", "a") as f:
            f.write(json.dumps({"test": tag, "rows": rows}) + "\n")


def test_family_r_step_gpu_matches_cpu_oracle():
    (G, D, _), (Gg, Dg, _), (Ge, De, _), out_c, out_g, out_e = _run_pair(0.0, eager_bf16=True)
    rows, bad = [], []
    for k in out_c:
        ref, got, eb = float(out_c[k]), float(out_g[k]), float(out_e[k])
        rows.append(("loss:" + k, abs(got - ref), abs(eb - ref), abs(ref)))
        if abs(got - ref) > 2 * abs(eb - ref) + 1e-2 * abs(ref) + 1e-5:
            bad.append(("loss", k, got, ref, eb))
    for net, netg, nete in ((G, Gg, Ge), (D, Dg, De)):
        grads = [(n, p.grad, pg.grad, pe.grad) for (n, p), (_, pg), (_, pe) in
                 zip(net.named_parameters(), netg.named_parameters(), nete.named_parameters())
                 if p.grad is not None]
        assert grads
        gscale = max(gr.abs().max().item() for _, gr, _, _ in grads)
        for n, gr, gg, ge in grads:
            assert gg is not None and torch.isfinite(gg).all(), n
            err = (gg.cpu().float() - gr.float()).abs().max().item()
            erre = (ge.cpu().float() - gr.float()).abs().max().item()
            scale = gr.abs().max().item()
            rows.append((n, err, erre, scale))
            floor = 1e-2 * scale
            if gr.numel() == 1 and n.endswith("relu.weight"):
                # the single-scalar shared-PReLU slope gradient: a heavily cancelling sum of
                # dy * z over every negative PReLU input of five sites (S = sum |dy * z| = 36.5
                # for |g| = 0.084 on the oracle: kappa = S / |g| ~ 430).  Against the fp32
                # oracle it cannot be bounded tighter than the network's bf16 rounding moves
                # dy: the eager bf16 step is off by 0.0014 - 0.049 over repeated runs (its
                # MIOpen reductions are not deterministic) and the native one by 0.025 - 0.060
                # as upstream roundings changed.  Two checks that do catch a wrong gradient:
                #  (1) the kernels' fp32 reduction against an fp64 sum of the SAME native
                #      terms (dy * y / w over y <= 0 at the five fused sites, captured by
                #      _NativeSlopeTerms): within 5 % of the value or 2^-12 of the native
                #      S (~10 % of the value at kappa 430) -- a sign flip, a dropped site or a
                #      wrong scale is off by >= 100 %;
                #  (2) end to end: the same sign as the fp32 oracle's gradient.
                S = _COND.get("slope_abs_sum", 0.0)
                tsum, tabs, sites = _COND.get("native_terms", (0.0, 0.0, 0))
                got = float(gg.float().item())
                self_err = abs(got - tsum)
                rows.append(("relu.weight:abs_sum_S,kappa", S, S / max(scale, 1e-12), scale))
                rows.append(("relu.weight:native_terms_sum,err,S_native,sites", tsum, self_err, tabs, sites))
                if sites != 5 or self_err > max(0.05 * abs(tsum), tabs * 2.0 ** -12):
                    bad.append((n, "native terms", got, tsum, tabs, sites))
                if (got > 0) != (float(gr.item()) > 0):
                    bad.append((n, "sign vs oracle", got, float(gr.item())))
                #  (3) a loose magnitude bound against the oracle: an upstream
                #      error in dy that keeps the sign (a dropped fan-out or pairing
                #      contribution) still moves the value by O(|g|); measured 0.025 - 0.060
                #      against max(S * 2^-8, 1.5 |g|) = 0.14
                mag_bound = max(S * 2.0 ** -8, 1.5 * abs(float(gr.item())))
                rows.append(("relu.weight:err_vs_oracle,bound", abs(got - float(gr.item())), mag_bound, scale))
                if abs(got - float(gr.item())) > mag_bound:
                    bad.append((n, "magnitude vs oracle", got, float(gr.item()), mag_bound))
                continue
            if err > 2 * erre + floor and err > 1e-3 * gscale:
                bad.append((n, err, erre, scale))
    for net, netg, nete, it in ((G, Gg, Ge, "buffers"), (D, Dg, De, "uv")):
        src = (lambda m: m.named_buffers()) if it == "buffers" else (lambda m: m.named_parameters())
        for (n, t), (_, tg), (_, te) in zip(src(net), src(netg), src(nete)):
            if not t.dtype.is_floating_point or (it == "uv" and not n.endswith(("_u", "_v"))):
                continue
            err, erre = _rel(tg.cpu(), t), _rel(te.cpu(), t)
            rows.append((n, err, erre, 1.0))
            if err > 2 * erre + 1e-2:
                bad.append((n, err, erre))
    _record("family_r_step_vs_oracle", rows)
    assert not bad, bad


def test_family_r_update_direction_matches_oracle():
    nets, nets_g, _, _, _, _ = _run_pair(lr=2e-4)
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


def _native_step_grads(monkeypatch, pair):
    """One native family-R step (lr 0, deterministic split-K) with gradient pairing on or off
    (``P2P_GRAD_PAIR``, read per call): every D gradient and the shared PReLU slope's."""
    from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
    from p2p_pytorch_amd.ops import hip
    monkeypatch.setenv("P2P_GRAD_PAIR", "1" if pair else "0")
    p2p.set_backend("native")
    hip.reset_rng(0)
    G, D, C, vgg = (copy.deepcopy(m).cuda() for m in _nets())
    g = torch.Generator().manual_seed(5)
    a, b = (torch.rand(2, 3, 64, 64, generator=g) * 2 - 1 for _ in range(2))

    def dev(x):
        return x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    step = CompressGANStep(G, D, C, lr=0.0, vgg=vgg)
    p2p.set_deterministic(True)
    try:
        step.step(dev(a), dev(b))
    finally:
        p2p.set_deterministic(False)
    torch.cuda.synchronize()
    out = {"G.relu.weight": G.relu.weight.grad.detach().float().clone()}
    for n, p in D.named_parameters():
        if p.grad is not None:
            out["D." + n] = p.grad.detach().float().clone()
    return out


def test_grad_pairing_matches_autograd_sum(monkeypatch):
    """gradient pairing adds a paired leaf's later contributions into the FIRST
    tensor handed to autograd; a contribution that bypassed the pairing would be summed out
    of place by autograd and the in-place adds silently lost.  With pairing off every
    contribution goes through autograd's own sum: the two steps must give the same D
    gradients (fake + real passes of every SN conv) and the same slope gradient (five
    sites).  A lost contribution is an O(1) relative difference; fp32 summation order
    differences are ~1e-7."""
    on = _native_step_grads(monkeypatch, True)
    off = _native_step_grads(monkeypatch, False)
    assert on.keys() == off.keys() and len(on) > 10
    bad = []
    for k in on:
        scale = off[k].abs().max().item()
        err = (on[k] - off[k]).abs().max().item()
        if err > 1e-3 * scale + 1e-7:
            bad.append((k, err, scale))
    assert not bad, bad
