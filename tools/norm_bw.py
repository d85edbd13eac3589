"""Achieved HBM bandwidth of the normalisation apply passes.

Times the forward apply (y = act(x * scale + shift): read x, write y) and the backward apply
(dx = ca * dy * act' + k0 + k1 * x: read x and dy, write dx; run as the frozen-statistics
norm_bwd, whose only other launch is a tiny per-(n, c) coefficient kernel) on the U-Net-256 /
PatchGAN instance-norm shapes of the headline step, and prints bytes / time per shape.

    python tools/norm_bw.py [--batch 256] [--iters 20]
    P2P_NORM_NT=1|2|3 python tools/norm_bw.py     # nontemporal stores / loads / both
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import p2p_pytorch_amd as p2p  # noqa: E402

# (tag, images per batch image, C, H): encoder e2-e7, decoder d1-d7 outputs, D c2-c4 (fake+real)
SHAPES = [("e2", 1, 128, 64), ("e3", 1, 256, 32), ("e4", 1, 512, 16), ("e5", 1, 512, 8),
          ("d4", 1, 512, 16), ("d5", 1, 256, 32), ("d6", 1, 128, 64), ("d7", 1, 64, 128),
          ("Dc2", 2, 128, 64), ("Dc3", 2, 256, 32), ("Dc4", 2, 512, 31)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    assert p2p._native.load(), p2p._native.load_error()
    P = torch.ops.p2p
    dev = torch.device("cuda")
    rows = []
    tot = {"fwd_ms": 0.0, "bwd_ms": 0.0, "fwd_gb": 0.0, "bwd_gb": 0.0}
    for tag, k, C, H in SHAPES:
        N = k * args.batch
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        mean = torch.randn(N, C, device=dev) * 0.1
        rstd = torch.rand(N, C, device=dev) + 0.5
        nbytes = x.numel() * 2

        def timed(fn):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / args.iters

        tf = timed(lambda: P.norm_apply(x, mean, rstd, None, None, None, 2, False))
        tb = timed(lambda: P.norm_bwd(x, dy, mean, rstd, None, None, 2, None, None, True, False, None,
                                      None, None, 0, None, None, None, True))
        r = {"tag": tag, "shape": [N, C, H, H], "MB": nbytes / 1e6,
             "fwd_ms": tf, "fwd_TBs": 2 * nbytes / tf / 1e9,
             "bwd_ms": tb, "bwd_TBs": 3 * nbytes / tb / 1e9}
        rows.append(r)
        tot["fwd_ms"] += tf
        tot["bwd_ms"] += tb
        tot["fwd_gb"] += 2 * nbytes / 1e9
        tot["bwd_gb"] += 3 * nbytes / 1e9
        print(f"{tag:4s} {str([N, C, H, H]):22s} {nbytes / 1e6:8.1f} MB  fwd {tf:7.3f} ms "
              f"{r['fwd_TBs']:5.2f} TB/s   bwd {tb:7.3f} ms {r['bwd_TBs']:5.2f} TB/s", flush=True)
        del x, dy
    print(json.dumps({"nt": os.environ.get("P2P_NORM_NT", "0"), "batch": args.batch,
                      "fwd_TBs": tot["fwd_gb"] / tot["fwd_ms"], "bwd_TBs": tot["bwd_gb"] / tot["bwd_ms"],
                      "fwd_ms": tot["fwd_ms"], "bwd_ms": tot["bwd_ms"]}))


if __name__ == "__main__":
    main()
