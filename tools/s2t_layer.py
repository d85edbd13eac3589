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
    ap.add_argument("--act", default="lrelu", choices=["lrelu", "none"],
                    help="dgrad: input activation of the conv (lrelu: the act' gate in the epilogue)")
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
        y = ops.conv2d(x, w, None, 2, 1, act_in=None if a.act == "none" else a.act)
        gy = torch.randn_like(y)

        def fn():
            return torch.autograd.grad(y, x, gy, retain_graph=True)[0]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flop = 2.0 * a.N * (2 * a.H) ** 2 * a.Cout * a.C * 4
    print(f"{a.mode} act={a.act} N{a.N} C{a.C} H{a.H} Cout{a.Cout} s2t={os.environ.get('P2P_NO_S2T') is None} "
          f"lib={os.path.basename(os.environ.get('P2P_LIB', 'default'))} grid={os.environ.get('P2P_S2T_GRID', '2')}: "
          f"{ms:.3f} ms {flop / ms / 1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
