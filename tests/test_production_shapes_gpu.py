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

(gradients: absolute floor 1e-3 of the network's largest gradient -- biases of convs feeding
an instance norm have an exactly-zero true gradient).  It also checks which kernels ran, so
the bound is known to cover the production tiles.
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


def test_headline_step_at_production_shape_matches_fp32():
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    G0, D0 = _nets()
    g = torch.Generator().manual_seed(13)
    a = torch.rand(B, 3, S, S, generator=g) * 2 - 1
    b = torch.rand(B, 3, S, S, generator=g) * 2 - 1
    # the native run under the profiler's kernel list: the production tiles must be among them
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        ln, gn = _run("native", G0, D0, a, b)
    names = {e.name for e in prof.events()}
    lc, gc = _run("fp32", G0, D0, a, b)
    le, ge = _run("eager", G0, D0, a, b)
    want = {"256x256 LATE fwd": "conv_fwd_glds_kernel<256, 256, 2, 4, 0, 2",
            "256x256 MODE-1": "conv_fwd_glds_kernel<256, 256, 2, 4, 1, 2",
            "256x128 3-stage": "conv_fwd_glds_kernel<256, 128, 4, 2,",
            "EXT epilogue": "true>(p2p::ConvFwdArgs)",
            "wgrad 256x128": "conv_wgrad_glds_kernel<256, 128",
            "image head": "halo_union_kernel",
            # round 3: the class-shared halo kernel of the stride-2 transposed convs / dgrads
            # onto 64x64 grids (d2 forward with input ReLU, the EXT dgrads)
            "s2t halo ConvT": "conv_s2t_kernel<64, true, false, 0>",
            "s2t halo EXT dgrad": "conv_s2t_kernel<64, false, true, 0>"}
    missing = [k for k, pat in want.items() if not any(pat in n for n in names)]
    rows, bad = [], []
    for k in lc:
        err, erre = abs(ln[k] - lc[k]), abs(le[k] - lc[k])
        rows.append(("loss:" + k, err, erre, abs(lc[k])))
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
            rows.append((n, err, erre, scale))
            if err > 2 * erre + 1e-2 * scale and err > 1e-3 * gscale:
                bad.append((n, err, erre, scale))
    if os.path.isdir("gpurun_out"):
        with open("gpurun_out/bounds.jsonl", "a") as f:
            f.write(json.dumps({"test": "headline_step_production_shape", "rows": rows,
                                "missing_kernels": missing}) + "\n")
    assert not missing, f"production tiles not exercised: {missing}"
    assert not bad, bad
