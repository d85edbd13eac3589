"""Run-to-run determinism of the norm-chain step (tests/test_s2t_gpu.py::
test_s2t_norm_chain_fused_partials_and_stats) on the s2t and implicit-GEMM routes.

Runs the chain three times per route and prints, per output tensor, whether the repeats are
bitwise equal and the max-norm relative difference between routes -- separates a
nondeterministic reduction (repeats differ) from a route difference (repeats equal, routes
differ).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from p2p_pytorch_amd import _native, ops

DEV = "cuda"
NAMES = ("u", "dx", "dw1", "dw2", "dwt")


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def main():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    g = torch.Generator(device=DEV).manual_seed(9)
    x = (torch.randn(4, 64, 256, 256, device=DEV, generator=g)
         .to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    torch.manual_seed(0)
    w1 = torch.randn(64, 64, 4, 4, device=DEV) * 0.03
    b1 = torch.randn(64, device=DEV) * 0.1
    w2 = torch.randn(128, 64, 4, 4, device=DEV) * 0.03
    wt = torch.randn(128, 64, 4, 4, device=DEV) * 0.03
    lin = None

    def run():
        nonlocal lin
        leaves = [t.detach().clone().requires_grad_(True) for t in (x, w1, b1, w2, wt)]
        hx, hw1, hb1, hw2, hwt = leaves
        h = ops.instance_norm(ops.conv2d(hx, hw1, hb1, 2, 1, stats=True), act="lrelu")
        z = ops.conv2d(h, hw2, None, 2, 1)
        u = ops.instance_norm(ops.conv_transpose2d(z, hwt, None, 2, 1, act_in="relu", stats=True),
                              act="relu")
        if lin is None:
            lin = torch.linspace(-1, 1, u.numel(), device=DEV).view_as(u)
        (u.float() * lin).sum().backward()
        torch.cuda.synchronize()
        return u.detach(), hx.grad, hw1.grad, hw2.grad, hwt.grad

    outs = {}
    for route in ("s2t", "gemm"):
        if route == "gemm":
            os.environ["P2P_NO_S2T"] = "1"
        outs[route] = [run() for _ in range(3)]
        os.environ.pop("P2P_NO_S2T", None)
    for route, rs in outs.items():
        eq = [all(torch.equal(a, b) for a, b in zip(rs[0], r)) for r in rs[1:]]
        per = [max(rel(a, b) for a, b in zip(rs[0], r)) for r in rs[1:]]
        print(f"{route}: repeats bitwise equal {eq}, max rel diff {per}")
        for i, n in enumerate(NAMES):
            print(f"  {n}: repeat diffs {[round(rel(rs[0][i], r[i]), 5) for r in rs[1:]]}")
    for i, n in enumerate(NAMES):
        d = [round(rel(outs['s2t'][k][i], outs['gemm'][k][i]), 5) for k in range(3)]
        a, b = outs['s2t'][0][i].float(), outs['gemm'][0][i].float()
        k = (a - b).abs().flatten().argmax().item()
        print(f"route diff {n}: {d}  worst elem {k}: s2t {a.flatten()[k].item():.5g} "
              f"gemm {b.flatten()[k].item():.5g} max|gemm| {b.abs().max().item():.5g}")


if __name__ == "__main__":
    main()
