"""Timeline probe of the persistent s2t kernel (csrc/conv_s2t.hip, P2P_S2T_DEBUG=1): which
blocks share a CU, per-tile MFMA-loop and epilogue durations, and how much of one block's
epilogue overlaps its CU partner's loop.

    P2P_S2T_DEBUG=1 python tools/s2t_timeline.py [--N 1024 --C 128 --H 64 --Cout 64]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import p2p_pytorch_amd as p2p  # noqa: E402
from p2p_pytorch_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--C", type=int, default=128)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--Cout", type=int, default=64)
    ap.add_argument("--act", default="lrelu")
    a = ap.parse_args()
    os.environ["P2P_S2T_DEBUG"] = "1"
    p2p.set_backend("native")
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(a.N, a.Cout, 2 * a.H, 2 * a.H, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    w = torch.randn(a.C, a.Cout, 4, 4, device=dev) * 0.02
    y = ops.conv2d(x, w, None, 2, 1, act_in=None if a.act == "none" else a.act)
    gy = torch.randn_like(y)
    for _ in range(3):
        torch.autograd.grad(y, x, gy, retain_graph=True)
    torch.cuda.synchronize()
    torch.autograd.grad(y, x, gy, retain_graph=True)
    torch.cuda.synchronize()
    d = torch.ops.p2p.s2t_debug().view(1024, 96, 4)
    nb = int((d[:, 0, 3] != 0).sum())
    t0 = int(d[:nb, 0, 0].min())
    keys = collections.defaultdict(list)
    loop, epi = [], []
    for b in range(nb):
        keys[int(d[b, 0, 3])].append(b)
        for k in range(96):
            s, e0, e1 = (int(v) for v in d[b, k, :3])
            if s == 0 or e1 == 0 or e1 < s:
                break
            loop.append((e0 - s) * 10e-3)
            epi.append((e1 - e0) * 10e-3)
    per = collections.Counter(len(v) for v in keys.values())
    print(f"blocks {nb}, distinct CU keys {len(keys)}, blocks per key {dict(per)}")
    pairs = [v for v in keys.values() if len(v) == 2]
    if pairs:
        print("first co-resident pairs:", pairs[:8])
    loop.sort(), epi.sort()
    med = lambda v: v[len(v) // 2] if v else 0.0  # noqa: E731
    print(f"tiles {len(loop)}: loop median {med(loop):.2f} us (p10 {loop[len(loop) // 10]:.2f}, "
          f"p90 {loop[9 * len(loop) // 10]:.2f}); epilogue median {med(epi):.2f} us "
          f"(p10 {epi[len(epi) // 10]:.2f}, p90 {epi[9 * len(epi) // 10]:.2f})")
    # overlap: for co-resident pairs, fraction of block A's epilogue time during which B is in its loop
    ov, tot = 0.0, 0.0
    for A, B in pairs[:64]:
        ivB = [(int(d[B, k, 0]), int(d[B, k, 1])) for k in range(96) if d[B, k, 2] != 0]
        for k in range(96):
            s0, s1 = int(d[A, k, 1]), int(d[A, k, 2])
            if s1 == 0:
                break
            tot += s1 - s0
            for b0, b1 in ivB:
                ov += max(0, min(s1, b1) - max(s0, b0))
    if tot:
        print(f"epilogue time overlapped by the CU partner's MFMA loop: {100 * ov / tot:.1f} %")
    starts = sorted((int(d[b, 0, 0]) - t0) * 10e-3 for b in range(nb))
    print(f"block start spread: first {starts[0]:.2f} us, median {starts[len(starts) // 2]:.2f}, "
          f"last {starts[-1]:.2f} us")
    # one pair's timeline
    if pairs:
        A, B = pairs[0]
        for blk in (A, B):
            line = []
            for k in range(6):
                s, e0, e1 = (int(v) for v in d[blk, k, :3])
                line.append(f"[{(s - t0) * 1e-2:.1f} L {(e0 - t0) * 1e-2:.1f} E {(e1 - t0) * 1e-2:.1f}]")
            print(f"block {blk}: " + " ".join(line))


if __name__ == "__main__":
    main()
