"""Which Python lines still launch aten (PyTorch-native) GPU kernels in the headline step.

Builds the bench's U-Net-256 + PatchGAN native step (B = 8, 256^2, bf16 unless --precision),
runs warmup steps, then profiles one eager step with Python stacks and prints every aten op
that launched device work, with the innermost frames from this repository.

    python tools/probes/aten_census.py [--precision fp8] [--batch 8]
"""
import argparse
import collections

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--family", default="pix2pix", choices=["pix2pix", "ref"])
    args = ap.parse_args()
    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    from p2p_pytorch_amd.ops import fp8 as f8
    from torch.profiler import ProfilerActivity, profile

    p2p.set_backend("native")
    f8.set_precision(args.precision)
    dev = torch.device("cuda")
    if args.family == "ref":
        from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
        from p2p_pytorch_amd.models import define_C
        G = define_G(netG="expand", gpu_id=dev, verbose=False)
        D = define_D(6, 64, gpu_id=dev, netD="multiscale", verbose=False)
        step = CompressGANStep(G, D, define_C(gpu_id=dev, verbose=False))
    else:
        G = define_G(netG="unet_256", gpu_id=dev, verbose=False)
        D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
        step = Pix2PixStep(G, D)
    g = torch.Generator(device=dev).manual_seed(1)
    a, b = [(torch.rand(args.batch, 3, 256, 256, device=dev, generator=g) * 2 - 1)
            .to(torch.bfloat16).contiguous(memory_format=torch.channels_last) for _ in range(2)]
    for _ in range(3):
        step.step(a, b)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        step.step(a, b)
        torch.cuda.synchronize()
    # CPU ops -> the device kernels they launched (FunctionEvent.kernels), with the nearest
    # repo frames on the op's (or an ancestor's) Python stack
    rows = collections.Counter()
    for e in prof.events():
        ks = [k.name for k in getattr(e, "kernels", []) or []]
        ks = [k for k in ks if "at::native" in k or "rocclr" in k]
        if not ks:
            continue
        frames, p = [], e
        while p is not None and not frames:
            frames = [f for f in (p.stack or []) if "p2p_pytorch_amd" in f or "tools/" in f][:4]
            p = p.cpu_parent
        op, p, ctx, shp = e.name, e, "", ""
        while p is not None:
            if p.name.startswith("aten::"):
                op = p.name
                shp = str(getattr(p, "input_shapes", ""))[:80]
            elif not ctx and not p.name.startswith("cuda") and not p.name.startswith("hip"):
                ctx = p.name[:70]      # the backward node / custom op / python frame above it
            p = p.cpu_parent
        for k in ks:
            rows[(k[:90], f"{op} {shp} in {ctx}", " <- ".join(frames))] += 1
    for (k, op, st), n in sorted(rows.items(), key=lambda kv: -kv[1]):
        print(f"{n:3d}  {k}\n     op {op}\n     at {st}")


if __name__ == "__main__":
    main()
