"""Trace the DP reducer's direct-gradient bookkeeping on one GPU (force_comm reducers).

Builds the headline pix2pix step (U-Net-256 + PatchGAN, packed path) at a small batch with
GradReducer(direct=True) on a world-1 RCCL group and logs, per backward and per parameter,
the forward use counts, the direct contributions (``direct_done``) and the autograd hook
arrivals (``_on_grad``); any parameter with more than one arrival, or both kinds, is
printed, then the steps run and the reducer's own error (if any) is shown.

    python tools/diag_direct.py [--batch 4] [--size 256] [--steps 2]
"""
import argparse
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import p2p_pytorch_amd as p2p  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    from p2p_pytorch_amd.parallel import GradReducer
    from p2p_pytorch_amd.parallel import dist as pdist
    dev = torch.device("cuda", torch.cuda.current_device())
    p2p.set_backend("native")
    pdist.init_single(dev)
    torch.manual_seed(0)
    G = define_G(netG="unet_256", gpu_id=dev, verbose=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
    rg = rd = None
    log = collections.defaultdict(lambda: collections.Counter())
    names = {}
    for tag, net in (("G", G), ("D", D)):
        for n, p in net.named_parameters():
            names[id(p)] = f"{tag}.{n}"

    orig = {k: getattr(GradReducer, k) for k in ("direct_done", "_on_grad", "zero_grad", "finish", "_launch")}
    history = []   # (reducer, kind, param name, bucket index, pending before)

    def wrap(kind):
        f = orig[kind]

        def g(self, *a, **k):
            tag = "G" if self is rg else "D"
            if kind in ("direct_done", "_on_grad"):
                nm = names.get(id(a[0]), "?%x" % id(a[0]))
                log[nm][kind] += 1
                b = self._param_bucket.get(a[0])
                history.append((tag, kind, nm, None if b is None else b.index,
                                None if b is None else b.pending, id(a[0]) in self._direct_seen))
            elif kind == "_launch":
                history.append((tag, "LAUNCH", "-", a[0].index, a[0].pending, None))
                return f(self, *a, **k)
            else:
                print(f"-- {tag}.{kind}", flush=True)
                history.append((tag, kind.upper(), "-", None, None, None))
                if kind == "finish":
                    bad = {n: dict(c) for n, c in log.items() if n.startswith(tag) and c["_on_grad"] != 1}
                    print(f"   {tag} params with anomalous arrivals: {len(bad)}", flush=True)
                    for n, c in list(bad.items())[:20]:
                        print(f"     {n}: {c}", flush=True)
                    for n in [n for n in log if n.startswith(tag)]:
                        del log[n]
            return f(self, *a, **k)
        return g

    for k in orig:
        setattr(GradReducer, k, wrap(k))
    # built after the patch: the grad hooks bind _on_grad at construction
    rg = GradReducer(G, bucket_mb=16.0, force_comm=True, direct=True)
    rd = GradReducer(D, bucket_mb=16.0, force_comm=True, direct=True)
    step = Pix2PixStep(G, D, reducer_g=rg, reducer_d=rd)
    a = (torch.rand(args.batch, 3, args.size, args.size, device=dev) * 2 - 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    b = (torch.rand(args.batch, 3, args.size, args.size, device=dev) * 2 - 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    try:
        for i in range(args.steps):
            print(f"== step {i}", flush=True)
            step.step(a, b)
        torch.cuda.synchronize()
        print("steps ok")
    except Exception:
        traceback.print_exc()
        snap = {n: dict(c) for n, c in log.items()}
        print("reducer history (tag, event, param, bucket, pending before, uses):", flush=True)
        for h in history[-60:]:
            print("   ", h)
        print("arrivals at the error:", flush=True)
        for n, c in snap.items():
            if c.get("_on_grad", 0) != 1:
                print(f"   {n}: {c}")
    finally:
        for k, f in orig.items():
            setattr(GradReducer, k, f)
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
