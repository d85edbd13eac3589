"""One stride-2 transposed-conv layer geometry, repeated (for rocprofv3 counter passes and
quick timing of the s2t halo kernel vs the implicit GEMM, P2P_NO_S2T=1).

    python tools/s2t_layer.py [--mode convt|dgrad] [--N 256] [--C 128] [--H 64] [--Cout 64]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import p2p_pytorch_amd as p2p  # noqa: E402
from p2p_pytorch_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="convt", choices=["convt", "dgrad"])
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--C", type=int, default=128)
    ap.add_argument("--H", type=int, default=64, help="input grid of the transposed conv")
    ap.add_argument("--Cout", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    p2p.set_backend("native")
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.mode == "convt":
        x = torch.randn(a.N, a.C, a.H, a.H, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(a.C, a.Cout, 4, 4, device=dev) * 0.02

        def fn():
            return ops.conv_transpose2d(x, w, None, 2, 1)
    else:
        # input gradient of lrelu -> conv 4x4 s2 p1 from Cout channels at 2H to C at H
        x = torch.randn(a.N, a.Cout, 2 * a.H, 2 * a.H, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        w = (torch.randn(a.C, a.Cout, 4, 4, device=dev) * 0.02).requires_grad_(False)
        y = ops.conv2d(x, w, None, 2, 1, act_in="lrelu")
        gy = torch.randn_like(y)

        def fn():
            return torch.autograd.grad(y, x, gy, retain_graph=True)[0]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / a.iters * 1e3
    print(f"{a.mode} N{a.N} C{a.C} H{a.H} Cout{a.Cout} s2t={os.environ.get('P2P_NO_S2T') is None}: {ms:.3f} ms")


if __name__ == "__main__":
    main()
