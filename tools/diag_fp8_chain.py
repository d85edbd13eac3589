"""fp8 norm chain (tests/test_fp8_gpu.py::test_fp8_s2t_ext_dgrad_chain_matches_implicit_gemm)
run repeatedly on both routes: per run the max |.| of dx, dw1, dw2 and the difference to the
previous run of the same route -- separates a route bug from run-to-run garbage (a kernel
reading memory nobody wrote shows as repeats that differ)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import p2p_pytorch_amd as p2p
from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import hip

DEV = "cuda"


def main():
    p2p.set_backend("native")
    assert _native.load(), _native.load_error()
    from p2p_pytorch_amd.ops import fp8 as f8
    f8.set_precision("fp8")
    print("fp8 enabled:", f8.enabled(), "P2P_WRED_OLD", os.environ.get("P2P_WRED_OLD"))
    g0 = torch.Generator(device=DEV).manual_seed(9)
    x = (torch.randn(4, 64, 256, 256, device=DEV, generator=g0)
         .to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    g = torch.Generator(device=DEV).manual_seed(11)
    w1 = torch.randn(64, 64, 4, 4, device=DEV, generator=g) * 0.03
    w2 = torch.randn(128, 64, 4, 4, device=DEV, generator=g) * 0.03

    def run():
        hip.begin_step()
        hx, hw1, hw2 = (t.detach().clone().requires_grad_(True) for t in (x, w1, w2))
        h = ops.instance_norm(ops.conv2d(hx, hw1, None, 2, 1, stats=True), act="lrelu")
        z = ops.conv2d(h, hw2, None, 2, 1)
        loss = (z.float() * torch.linspace(-1, 1, z.numel(), device=DEV).view_as(z)).sum()
        loss.backward()
        torch.cuda.synchronize()
        return z.detach().float(), hx.grad.float(), hw1.grad.float(), hw2.grad.float()

    prev = {}
    for route in ("s2t", "gemm", "s2t", "gemm"):
        if route == "gemm":
            os.environ["P2P_NO_S2T"] = "1"
        for k in range(3):
            out = run()
            mx = [round(t.abs().max().item(), 5) for t in out]
            d = ([round((a - b).abs().max().item(), 6) for a, b in zip(out, prev[route])]
                 if route in prev else None)
            print(f"{route} run {k}: max|z,dx,dw1,dw2| {mx}  diff to previous same-route {d}",
                  flush=True)
            prev[route] = out
        os.environ.pop("P2P_NO_S2T", None)


if __name__ == "__main__":
    main()
