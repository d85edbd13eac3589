"""The headline step at its production geometry against an fp32 oracle.

``bench.py`` runs U-Net-256 + 70x70 PatchGAN at 256x256; the kernels it selects there (the
256x256 LATE-ring forward tile, the 256x128 3-stage tile, MODE-1 class-fastest order for the
stride-2 transposed convs / dgrads, the EXT dgrad epilogue with fused norm partials, the
packed image head, and since round 3 the class-shared halo kernel of the stride-2 transposed
convs, csrc/conv_s2t.hip) are chosen by layer shape, and several only engage at the real M of a
256x256 batch.  This test runs ONE packed native ``Pix2PixStep`` (lr = 0) at 256x256,
B = 64 (the smallest batch at which the 256x256 tiles engage: they need >= 256 tiles per
launch), and bounds every loss and every G / D gradient against the same step in fp32 on stock
PyTorch (MIOpen fp32, no autocast), with the rule of tests/test_pix2pix_step_gpu.py:

    |native - fp32| <= 2 |eager bf16 autocast - fp32| + 1 % of the quantity's scale

per tensor, with no network-wide floor: only the structurally-zero gradients (biases of convs
feeding an instance norm, ZERO_REL below) get an absolute bound.  It also checks which kernels
ran, so the bound is known to cover the production tiles.  The same step in fp8 (BASELINE
config 5) has its own, fp8-derived bound (F8_REL / F8_COS below).
"""
import copy
import json
import os

import pytest
import torch

import p2p_pytorch_amd as p2p

pytestmark = pytest.mark.gpu
B, S = 64, 256


def _nets():
    from p2p_pytorch_amd.models import define_D, define_G
    torch.manual_seed(11)
    G = define_G(netG="unet_256", gpu_id="cpu", verbose=False, use_dropout=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id="cpu", verbose=False)
    return G, D


def _grads(*nets):
    out = {}
    for tag, net in zip("GD", nets):
        for n, p in net.named_parameters():
            if p.grad is not None:
                out[tag + "." + n] = p.grad.detach().float().cpu().clone()
    return out


def _run(kind, G0, D0, a, b):
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    G, D = copy.deepcopy(G0).cuda(), copy.deepcopy(D0).cuda()
    if kind in ("fp32", "eager"):
        p2p.set_backend("torch")
        try:
            step = Pix2PixStep(G, D, lr=0.0,
                               autocast_dtype=torch.bfloat16 if kind == "eager" else None)
            out = step.step(a.cuda(), b.cuda())
        finally:
            p2p.set_backend("native")
    else:
        p2p.set_backend("native")
        step = Pix2PixStep(G, D, lr=0.0, packed=True)

        def dev(x):
            return x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

        assert step._packed_ok(dev(a), dev(b))
        out = step.step(dev(a), dev(b))
    torch.cuda.synchronize()
    res = ({k: float(v) for k, v in out.items()}, _grads(G, D))
    del G, D, step
    torch.cuda.empty_cache()
    return res


@pytest.fixture(scope="module")
def refs():
    """The fp32 oracle and the eager bf16 autocast step, shared by the bf16 and fp8 tests."""
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    G0, D0 = _nets()
    g = torch.Generator().manual_seed(13)
    a = torch.rand(B, 3, S, S, generator=g) * 2 - 1
    b = torch.rand(B, 3, S, S, generator=g) * 2 - 1
    lc, gc = _run("fp32", G0, D0, a, b)
    le, ge = _run("eager", G0, D0, a, b)
    return G0, D0, a, b, lc, gc, le, ge


# A gradient whose fp32 magnitude is below ZERO_REL of the network's largest is structurally
# zero (the bias of a conv feeding an instance norm: the norm removes any per-channel shift, so
# its true gradient is exactly 0 and fp32 shows rounding noise); the native step returns exact
# zeros there (the norm backward's column sums), bounded by the same absolute ZERO_REL.
ZERO_REL = 1e-5
# bf16-unresolvable gradients: where the eager bf16 autocast step itself is off by more than
# ILL_REL of the tensor's own magnitude, the tensor carries no bf16-resolvable signal -- the
# innermost normalised U-Net levels (instance norm over 4x4 / 2x2 planes): against an fp64
# oracle fp32 is within 1.2 %, eager bf16 34-89 % and native 36-190 % off there in MAX-ABS
# terms.  That max-abs error is decided by the few (n, c) planes whose 4 values happen to
# nearly coincide, so it is a lottery: over 5 seeds the native / eager max-abs ratio on
# downs.6.weight is 3.42 / 1.65 / 0.75 / 1.12 / 1.11 (median 1.12), and an eager variant that
# keeps those planes' pre-norm values in fp32 (VERDICT r4 W7's proposal, emulated) scatters
# the same way, 0.61-1.64 (median 1.03) -- fp32 storage buys nothing: the noise comes from
# the bf16 operands upstream (profiles/diag_inner_grad_r5.txt, tools/diag_inner_grad.py).
# These tensors are bounded in relative L2 instead, where two equally precise bf16 steps
# agree: ||native - fp32|| <= ILL_K ||eager - fp32|| + 1 % ||fp32|| (measured ratios
# 0.91-1.09 at this seed, profiles/bounds_production_r4.jsonl).
ILL_REL = 0.25
ILL_K = 1.5


def _log(test, rows, extra):
    if os.path.isdir("gpurun_out"):
        with open("gpurun_out/bounds.jsonl", "a") as f:
            f.write(json.dumps({"test": test, "rows": rows, **extra}) + "\n")


def test_headline_step_at_production_shape_matches_fp32(refs):
    """Per tensor: |native - fp32|_max <= 2 |eager - fp32|_max + 1 % of that tensor's own
    scale (no network-wide floor), or the structurally-zero class above."""
    G0, D0, a, b, lc, gc, le, ge = refs
    # the native run under the profiler's kernel list: the production tiles must be among them
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        ln, gn = _run("native", G0, D0, a, b)
    names = {e.name for e in prof.events()}
    # (any pattern of a class counts: the 32x32x16 tiles of round 5 took over the round-4
    # 16x16x32 tiles on most layers, the latter still serve shapes the former reject)
    want = {"256x256 fwd tile": ("conv_fwd_m32_kernel<256, 0", "conv_fwd_glds_kernel<256, 256, 2, 4, 0, 2"),
            "256-row MODE-1 tile": ("conv_fwd_m32_kernel<256, 1", "conv_fwd_m32_kernel<128, 1",
                                    "conv_fwd_glds_kernel<256, 256, 2, 4, 1, 2"),
            "256x128 tile": ("conv_fwd_m32_kernel<128, ", "conv_fwd_glds_kernel<256, 128, 4, 2,"),
            "EXT epilogue": ("true>(p2p::ConvFwdArgs)",),
            "256-row wgrad tile": ("conv_wgrad_m32_kernel", "conv_wgrad_glds_kernel<256, 128"),
            "image head": ("halo_union_kernel",),
            # the class-shared halo kernel of the stride-2 transposed convs / dgrads onto
            # 64x64 grids (d2 forward with input ReLU, the EXT dgrads)
            "s2t halo ConvT": ("conv_s2t_kernel<64, true, false, 0>",),
            "s2t halo EXT dgrad": ("conv_s2t_kernel<64, false, true, 0>",)}
    missing = [k for k, pats in want.items() if not any(pat in n for pat in pats for n in names)]
    rows, bad = [], []
    for k in lc:
        err, erre = abs(ln[k] - lc[k]), abs(le[k] - lc[k])
        rows.append(("loss:" + k, err, erre, abs(lc[k]), "loss"))
        if err > 2 * erre + 1e-2 * abs(lc[k]) + 1e-5:
            bad.append(("loss", k, ln[k], lc[k], le[k]))
    assert set(gn) == set(gc), set(gn) ^ set(gc)
    for tag in "GD":
        names_t = [n for n in gc if n.startswith(tag)]
        gscale = max(gc[n].abs().max().item() for n in names_t)
        for n in names_t:
            assert torch.isfinite(gn[n]).all(), n
            err = (gn[n] - gc[n]).abs().max().item()
            erre = (ge[n] - gc[n]).abs().max().item()
            scale = gc[n].abs().max().item()
            if scale <= ZERO_REL * gscale:
                cls, ok = "zero", err <= ZERO_REL * gscale
            elif erre > ILL_REL * scale:
                nrm = gc[n].norm().item()
                err = (gn[n] - gc[n]).norm().item()
                erre = (ge[n] - gc[n]).norm().item()
                scale = nrm
                cls, ok = "ill_l2", err <= ILL_K * erre + 1e-2 * nrm
            else:
                cls, ok = "bound", err <= 2 * erre + 1e-2 * scale
            rows.append((n, err, erre, scale, cls))
            if not ok:
                bad.append((n, cls, err, erre, scale))
    _log("headline_step_production_shape", rows, {"missing_kernels": missing})
    n_ill = sum(1 for r in rows if r[-1] == "ill_l2")
    print(f"production-shape bf16: {len(rows)} rows, {n_ill} bf16-unresolvable (relative L2 bound)")
    assert not missing, f"production tiles not exercised: {missing}"
    assert not bad, bad


# fp8 (BASELINE config 5): e4m3 activations / weights (3 mantissa bits) and e5m2 gradients
# (2 bits) against bf16's 7 -- per-element rounding 2^4 - 2^5 times bf16's, so the max-error
# rule above does not transfer.  Bounded instead per tensor by the relative L2 error against
# the eager bf16 step's: ||native - fp32|| <= F8_K ||eager - fp32|| + F8_ABS ||fp32||
# (structurally-zero tensors as above), the whole network's gradient direction (cosine >=
# F8_COS) and the losses within 5 % + 0.02.  The fp8 conv operands cost a near-constant factor
# over eager bf16 -- 2.8-3.5x on the first MI355X run (G.downs.0 0.63 vs 0.21, D.convs.0 0.30
# vs 0.086; 4.2x on G.ups.1 at 3.5 % absolute), cosines 0.99995 (G) / 0.9990 (D).
F8_K = 4.0
F8_ABS = 0.05
F8_COS = 0.995


def test_fp8_step_at_production_shape_close_to_fp32(refs):
    from p2p_pytorch_amd.ops import fp8 as _f8
    G0, D0, a, b, lc, gc, le, ge = refs
    _f8.set_precision("fp8")
    try:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            ln, gn = _run("native", G0, D0, a, b)
    finally:
        _f8.set_precision("bf16")
    names = {e.name for e in prof.events()}
    assert any("conv_wgrad_f8_kernel" in n for n in names), "fp8 weight gradient not exercised"
    rows, bad = [], []
    for k in lc:
        err = abs(ln[k] - lc[k])
        rows.append(("loss:" + k, err, abs(le[k] - lc[k]), abs(lc[k]), "loss"))
        if err > 0.05 * abs(lc[k]) + 0.02:
            bad.append(("loss", k, ln[k], lc[k]))
    for tag in "GD":
        names_t = [n for n in gc if n.startswith(tag)]
        gscale = max(gc[n].abs().max().item() for n in names_t)
        vn = torch.cat([gn[n].reshape(-1) for n in names_t])
        vc = torch.cat([gc[n].reshape(-1) for n in names_t])
        cos = (vn @ vc / (vn.norm() * vc.norm()).clamp_min(1e-30)).item()
        rows.append((tag + ":cosine", cos, None, None, "cosine"))
        if cos < F8_COS:
            bad.append((tag, "cosine", cos))
        for n in names_t:
            assert torch.isfinite(gn[n]).all(), n
            d = gn[n] - gc[n]
            scale = gc[n].abs().max().item()
            if scale <= ZERO_REL * gscale:
                err = d.abs().max().item()
                cls, ok = "zero", err <= ZERO_REL * gscale
            else:
                err = (d.norm() / gc[n].norm()).item()
                erre = ((ge[n] - gc[n]).norm() / gc[n].norm()).item()
                cls, ok = "rel_l2", err <= F8_K * erre + F8_ABS
                rows.append((n, err, erre, scale, cls))
                if not ok:
                    bad.append((n, cls, err, erre))
                continue
            rows.append((n, err, None, scale, cls))
            if not ok:
                bad.append((n, cls, err))
    _log("fp8_step_production_shape", rows, {})
    assert not bad, bad
