#!/usr/bin/env python
"""Diagnose eager-vs-graph (and eager-vs-eager) differences of the pix2pix step in
deterministic mode: per step, which parameters / buffers differ first.  Writes JSON lines
to stdout."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import p2p_pytorch_amd as p2p  # noqa: E402
from p2p_pytorch_amd.ops import hip  # noqa: E402

STEPS = 3


def build(netg, size):
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    dev = torch.device("cuda")
    hip.reset_rng(0)
    torch.manual_seed(0)
    G = define_G(netG=netg, gpu_id=dev, verbose=False, use_dropout=os.environ.get("DROP", "1") == "1")
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
    return Pix2PixStep(G, D), G, D


def data(size):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    return [[(torch.rand(2, 3, size, size, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
             .contiguous(memory_format=torch.channels_last) for _ in range(2)] for _ in range(STEPS)]


def snap(G, D):
    return {n: p.detach().clone() for n, p in list(G.named_parameters()) + list(D.named_parameters())}


def run(kind, netg, size):
    step, G, D = build(netg, size)
    ds = data(size)
    fn = step.step
    if kind == "graph":
        from p2p_pytorch_amd.engine.graph import CapturedStep
        fn = CapturedStep(step.step, *ds[0], warmup=2)
    out = []
    for a, b in ds:
        losses = fn(a, b)
        torch.cuda.synchronize()
        out.append(({k: v.item() for k, v in losses.items()}, snap(G, D)))
    return out


def cmp(tag, x, y):
    for i, ((lx, px), (ly, py)) in enumerate(zip(x, y)):
        diff = [n for n in px if not torch.equal(px[n], py[n])]
        print(json.dumps({"cmp": tag, "step": i, "losses_equal": lx == ly, "ndiff": len(diff),
                          "first": diff[:8],
                          "maxabs": max([float((px[n] - py[n]).abs().max()) for n in diff] or [0.0])}),
              flush=True)


def main():
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    netg, size = os.environ.get("NETG", "unet_64"), int(os.environ.get("SIZE", "64"))
    a = run("eager", netg, size)
    b = run("eager", netg, size)
    c = run("graph", netg, size)
    cmp("eager_vs_eager", a, b)
    cmp("eager_vs_graph", a, c)


if __name__ == "__main__":
    main()
