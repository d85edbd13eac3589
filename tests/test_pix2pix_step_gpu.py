"""The headline pix2pix training step on the GPU against the CPU fp32 oracle.

Three GPU variants of one ``Pix2PixStep`` (lr = 0, so what is compared is everything the
step computes: the four logged losses and every G / D gradient the optimizers apply):

  * native, packed image path (ops/hip.py image head: (A | B) / (A | fake) pair tensors,
    union-GEMM last layer with the L1 term, fused head gradient) -- what bench.py runs;
  * native, unpacked (3-channel tensors, the round-1 path);
  * stock PyTorch bf16 autocast (the eager baseline): the dtype's own error.

Bound per quantity: |native - fp32| <= 2 |eager bf16 - fp32| + 1 % of its scale (gradients:
absolute floor 1e-3 of the network's largest gradient -- biases of convs feeding an
instance norm have an exactly-zero true gradient).
"""
import copy

import pytest
import torch

import p2p_pytorch_amd as p2p

pytestmark = pytest.mark.gpu


def _nets():
    from p2p_pytorch_amd.models import define_D, define_G
    torch.manual_seed(7)
    G = define_G(netG="unet_64", gpu_id="cpu", verbose=False, use_dropout=False)
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
    if kind == "cpu":
        G, D = copy.deepcopy(G0), copy.deepcopy(D0)
        p2p.set_backend("native")
        out = Pix2PixStep(G, D, lr=0.0).step(a, b)
        return {k: float(v) for k, v in out.items()}, _grads(G, D)
    G, D = copy.deepcopy(G0).cuda(), copy.deepcopy(D0).cuda()
    if kind == "eager":
        p2p.set_backend("torch")
        try:
            step = Pix2PixStep(G, D, lr=0.0, autocast_dtype=torch.bfloat16)
            out = step.step(a.cuda(), b.cuda())
        finally:
            p2p.set_backend("native")
    else:
        p2p.set_backend("native")
        step = Pix2PixStep(G, D, lr=0.0, packed=(kind == "packed"))

        def dev(x):
            return x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

        if kind == "packed":
            assert step._packed_ok(dev(a), dev(b))
        out = step.step(dev(a), dev(b))
    torch.cuda.synchronize()
    return {k: float(v) for k, v in out.items()}, _grads(G, D)


def test_pix2pix_step_packed_and_unpacked_match_oracle():
    G0, D0 = _nets()
    g = torch.Generator().manual_seed(9)
    a = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    b = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    lc, gc = _run("cpu", G0, D0, a, b)
    le, ge = _run("eager", G0, D0, a, b)
    rows, bad = [], []
    for kind in ("packed", "unpacked"):
        ln, gn = _run(kind, G0, D0, a, b)
        for k in lc:
            err, erre = abs(ln[k] - lc[k]), abs(le[k] - lc[k])
            rows.append((kind, "loss:" + k, err, erre, abs(lc[k])))
            if err > 2 * erre + 1e-2 * abs(lc[k]) + 1e-5:
                bad.append((kind, k, ln[k], lc[k], le[k]))
        assert set(gn) == set(gc), set(gn) ^ set(gc)
        for tag in "GD":
            names = [n for n in gc if n.startswith(tag)]
            gscale = max(gc[n].abs().max().item() for n in names)
            for n in names:
                assert torch.isfinite(gn[n]).all(), (kind, n)
                err = (gn[n] - gc[n]).abs().max().item()
                erre = (ge[n] - gc[n]).abs().max().item()
                scale = gc[n].abs().max().item()
                rows.append((kind, n, err, erre, scale))
                if err > 2 * erre + 1e-2 * scale and err > 1e-3 * gscale:
                    bad.append((kind, n, err, erre, scale))
    import json
    import os
    if os.path.isdir("gpurun_out"):
        with open("gpurun_out/bounds.jsonl", "a") as f:
            f.write(json.dumps({"test": "pix2pix_step_vs_oracle", "rows": rows}) + "\n")
    assert not bad, bad
