#!/usr/bin/env python
"""Per-layer conv kernel benchmark (fwd / dgrad / wgrad) on the headline model's shapes.

Times each op of every U-Net-256 / PatchGAN layer at per-GPU batch B with HIP events and
reports TFLOP/s (useful FLOPs: 2*M*N*K of the real conv, no padding), so kernel variants can
be A/B-ed in ONE process (interleaved rounds, cdna_hip_programming.md section 5.4 rule 24).

    python tools/conv_bench.py [--batch 64] [--iters 20] [--ops fwd,dgrad,wgrad]
                               [--variants env1,env2]   # values for P2P_CONV_VARIANT
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, kind, Cin1, Cin2, H_in, Cout, k, stride, pad, act_in)
LAYERS = [
    ("e1", "conv", 3, 0, 256, 64, 4, 2, 1, None),
    ("e2", "conv", 64, 0, 128, 128, 4, 2, 1, None),
    ("e3", "conv", 128, 0, 64, 256, 4, 2, 1, None),
    ("e4", "conv", 256, 0, 32, 512, 4, 2, 1, None),
    ("e5", "conv", 512, 0, 16, 512, 4, 2, 1, None),
    ("d5", "convT", 512, 512, 8, 512, 4, 2, 1, "relu"),
    ("d4", "convT", 512, 512, 16, 256, 4, 2, 1, "relu"),
    ("d3", "convT", 256, 256, 32, 128, 4, 2, 1, "relu"),
    ("d2", "convT", 128, 128, 64, 64, 4, 2, 1, "relu"),
    ("d1", "convT", 64, 64, 128, 3, 4, 2, 1, "relu"),
    ("c1", "conv", 3, 3, 256, 64, 4, 2, 1, None),
    ("c2", "conv", 64, 0, 128, 128, 4, 2, 1, None),
    ("c3", "conv", 128, 0, 64, 256, 4, 2, 1, None),
    ("c4", "conv", 256, 0, 32, 512, 4, 1, 1, None),
    ("c5", "conv", 512, 0, 31, 1, 4, 1, 1, None),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--variants", default="")
    ap.add_argument("--layers", default="")
    ap.add_argument("--json_out", default=None)
    ap.add_argument("--m32", default="", help="A/B the 32x32x16 tiles in ONE process: e.g. '1,0' "
                    "(torch.ops.p2p.set_m32 before each timed round; rounds interleaved)")
    ap.add_argument("--rounds", type=int, default=3, help="interleaved rounds per setting (--m32)")
    a = ap.parse_args()
    from p2p_pytorch_amd import _native, ops
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    dev = torch.device("cuda")
    B = a.batch
    variants = a.variants.split(",") if a.variants else [os.environ.get("P2P_CONV_VARIANT", "")]
    want = set(a.layers.split(",")) if a.layers else None
    results = []
    for name, kind, c1, c2, H, cout, k, s, p, act in LAYERS:
        if want and name not in want:
            continue
        cin = c1 + c2
        x1 = torch.randn(B, c1, H, H, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        x2 = (torch.randn(B, c2, H, H, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last) if c2 else None)
        if kind == "conv":
            w = torch.randn(cout, cin, k, k, device=dev) * 0.02
            OH = (H + 2 * p - k) // s + 1
        else:
            w = torch.randn(cin, cout, k, k, device=dev) * 0.02
            OH = (H - 1) * s - 2 * p + k
        M = B * OH * OH if kind == "conv" else B * H * H
        macs = (B * OH * OH * cout * cin * k * k) if kind == "conv" else (B * H * H * cin * cout * k * k)
        flops = 2.0 * macs
        y_first = None
        for var in variants:
            os.environ["P2P_CONV_VARIANT"] = var
            row = {"layer": name, "variant": var}
            for op in a.ops.split(","):
                xa = x1.detach().requires_grad_(op == "dgrad")
                xb = x2.detach().requires_grad_(op == "dgrad") if x2 is not None else None
                wl = w.detach().requires_grad_(op == "wgrad")
                xin = (xa, xb) if xb is not None else xa

                def fwd():
                    if kind == "conv":
                        return ops.conv2d(xin, wl, None, s, p, act_in=act)
                    return ops.conv_transpose2d(xin, wl, None, s, p, act)

                if op == "fwd":
                    fn = fwd
                    # every variant's output against the first variant's (same bf16 inputs)
                    with torch.no_grad():
                        yv = fwd().float()
                    if y_first is None:
                        y_first = yv
                    else:
                        row["fwd_rel_err_vs_first"] = float(
                            ((yv - y_first).abs().max() / y_first.abs().max().clamp_min(1e-6)).item())
                else:
                    y = fwd()
                    gy = torch.randn_like(y)

                    def fn(y=y, gy=gy):
                        torch.autograd.grad(y, [xa] if op == "dgrad" else [wl], gy,
                                            retain_graph=True)
                settings = [int(v) for v in a.m32.split(",")] if a.m32 else [None]
                best = {}
                for _r in range(a.rounds if a.m32 else 1):
                    for sv in settings:
                        if sv is not None:
                            torch.ops.p2p.set_m32(sv)
                        fn()
                        torch.cuda.synchronize()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(a.iters):
                            fn()
                        e1.record()
                        torch.cuda.synchronize()
                        ms = e0.elapsed_time(e1) / a.iters
                        best[sv] = min(best.get(sv, 1e30), ms)
                for sv, ms in best.items():
                    tag = op if sv is None else f"{op}_m32{sv}"
                    row[tag + "_us"] = round(ms * 1e3, 1)
                    row[tag + "_tflops"] = round(flops / (ms * 1e-3) / 1e12, 1)
                if a.m32:
                    torch.ops.p2p.set_m32(1)
            results.append(row)
            print(json.dumps(row), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
