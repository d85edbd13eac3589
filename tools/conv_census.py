"""Conv census: every conv_fwd / conv_wgrad call of one training step, replayed in isolation
and timed with HIP events -> per-geometry time and TF/s (the roofline view by layer shape).

  python tools/conv_census.py --family ref --batch 64 [--top 40] [--json out.json]

The step runs once (after a warm-up step) with the op namespace wrapped; the recorded calls
keep their tensors alive and are replayed ``--reps`` times each.  FLOPs count the real
multiply-adds of the geometry (padded channel counts as passed to the kernel).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="ref", choices=["ref", "pix2pix"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default=None)
    ap.add_argument("--variants", default="",
                    help="comma list of P2P_CONV_VARIANT values also timed per conv_fwd call (e.g. g2,g3)")
    ap.add_argument("--wgrad_variants", default="",
                    help="comma list of NAME=VAL environment settings also timed per conv_wgrad call "
                         "(e.g. P2P_M32=0)")
    args = ap.parse_args()

    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd.ops import hip
    from p2p_pytorch_amd.models import define_D, define_G
    p2p.set_backend("native")
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if args.family == "ref":
        from p2p_pytorch_amd.models import define_C
        from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
        G = define_G(netG="expand", gpu_id=dev, verbose=False)
        D = define_D(6, 64, gpu_id=dev, netD="multiscale", verbose=False)
        C = define_C(gpu_id=dev, verbose=False)
        trainer = CompressGANStep(G, D, C)
    else:
        from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
        G = define_G(netG="unet_256", gpu_id=dev, verbose=False)
        D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
        trainer = Pix2PixStep(G, D, lr=2e-4, beta1=0.5)
    B, S = args.batch, args.size
    a = (torch.rand(B, 3, S, S, device=dev) * 2 - 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    b = (torch.rand(B, 3, S, S, device=dev) * 2 - 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    trainer.step(a, b)
    torch.cuda.synchronize()

    real = hip.P()
    calls = []
    others = collections.Counter()
    other_elems = collections.Counter()

    class Proxy:
        def __getattr__(self, name):
            fn = getattr(real, name)
            if name not in ("conv_fwd", "conv_wgrad"):
                def count(*xs, **kw):
                    t = next((x for x in xs if isinstance(x, torch.Tensor)), None)
                    key = name + (f"(mode {xs[3]})" if name == "act" else "")
                    others[key] += 1
                    other_elems[key] += t.numel() if t is not None else 0
                    return fn(*xs, **kw)
                return count

            def rec(*xs, **kw):
                calls.append((name, xs, kw))
                return fn(*xs, **kw)
            return rec

    proxy = Proxy()
    orig = hip.P
    hip.P = lambda: proxy
    try:
        trainer.step(a, b)
    finally:
        hip.P = orig
    torch.cuda.synchronize()

    rows = []
    for name, xs, kw in calls:
        if name == "conv_fwd":
            x1, x2, w, bias, mode, KH, KW, s, pad, refl, up, act_in, OH, OW, Cout = xs[:15]
            C = x1.shape[1] + (x2.shape[1] if x2 is not None else 0)
            taps = KH * KW if mode == 0 else KH * KW / (s * s)
            flop = 2.0 * x1.shape[0] * OH * OW * Cout * taps * C
            # ideal HBM bytes: every operand read once, the output written once
            byts = 2.0 * (x1.numel() + (x2.numel() if x2 is not None else 0) + w.numel()
                          + x1.shape[0] * OH * OW * Cout)
            # EXT: a dgrad epilogue with an act' gate, a parked skip gradient or norm partials
            ext = bool(xs[19]) or kw.get("res") is not None or kw.get("nb_half") is not None
            geo = f"fwd m{mode} N{x1.shape[0]} C{C} {x1.shape[2]}x{x1.shape[3]} -> {Cout} k{KH} s{s} p{pad}" \
                  f"{' refl' if refl else ''}{' up2' if up == 2 else ''} -> {OH}x{OW}{' EXT' if ext else ''}"
        else:
            p1, p2_, p_act, q1, q2, q_act, KH, KW, s, pad, refl, up, dw = xs[:13]
            R = p1.shape[1] + (p2_.shape[1] if p2_ is not None else 0)
            Cq = q1.shape[1] + (q2.shape[1] if q2 is not None else 0)
            M = p1.shape[0] * p1.shape[2] * p1.shape[3]
            flop = 2.0 * M * R * KH * KW * Cq
            byts = 2.0 * (p1.numel() + (p2_.numel() if p2_ is not None else 0) + q1.numel()
                          + (q2.numel() if q2 is not None else 0)) + 4.0 * R * KH * KW * Cq
            geo = f"wgrad R{R} C{Cq} k{KH} s{s} p{pad}{' refl' if refl else ''}{' up2' if up == 2 else ''}" \
                  f" M{M} (p {p1.shape[2]}x{p1.shape[3]}, q {q1.shape[2]}x{q1.shape[3]})"
        fn = getattr(real, name)

        def timed():
            for _ in range(2):
                fn(*xs, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn(*xs, **kw)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / args.reps
        ms = timed()
        alt = {}
        vlist = args.variants if name == "conv_fwd" else args.wgrad_variants
        if vlist:
            for v in vlist.split(","):
                # "g5" -> P2P_CONV_VARIANT=g5; "NAME=VAL" -> that environment variable
                key, val = v.split("=", 1) if "=" in v else ("P2P_CONV_VARIANT", v)
                os.environ[key] = val
                try:
                    alt[v] = timed()
                finally:
                    os.environ.pop(key, None)
        rows.append((geo, ms, flop, alt, byts))
    agg = collections.OrderedDict()
    altagg = collections.defaultdict(lambda: collections.Counter())
    for geo, ms, flop, alt, byts in rows:
        e = agg.setdefault(geo, [0, 0.0, 0.0, 0.0])
        e[0] += 1
        e[1] += ms
        e[2] += flop
        e[3] += byts
        for v, t in alt.items():
            altagg[geo][v] += t
    tot = sum(v[1] for v in agg.values())
    print(f"{len(rows)} conv calls, {tot:.2f} ms replayed in isolation "
          f"({sum(v[2] for v in agg.values()) / 1e12:.2f} TFLOP)")
    print("ideal MB = every operand read once + output written once (the HBM floor of the call);"
          " floor ms = that at 6.3 TB/s")
    print(f"{'ms':>8} {'%':>5} {'n':>3} {'TF/s':>7} {'idealMB':>8} {'floor':>6}  geometry")
    for geo, (n, ms, flop, byts) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        extra = "".join(f"  [{v}: {t:.3f}]" for v, t in altagg[geo].items())
        print(f"{ms:8.3f} {100 * ms / tot:5.1f} {n:3d} {flop / ms / 1e9:7.1f} {byts / n / 1e6:8.1f} "
              f"{byts / 6.3e9:6.3f}  {geo}{extra}")
    print("\nother HIP ops of the step (calls, Melements of the first tensor argument):")
    for k, n in others.most_common():
        print(f"  {n:4d} {other_elems[k] / 1e6:10.1f}  {k}")
    if args.json:
        with open(args.json, "w") as f:
            json.dump([{"geometry": g, "calls": v[0], "ms": v[1], "flop": v[2], "ideal_bytes": v[3]}
                       for g, v in agg.items()],
                      f, indent=1)


if __name__ == "__main__":
    main()
