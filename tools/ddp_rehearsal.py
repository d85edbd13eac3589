#!/usr/bin/env python
"""Multi-rank rehearsal of the data-parallel training path on ONE GPU.

Launched by ``torch.distributed.run --nproc-per-node N`` with ``P2P_DIST_BACKEND=gloo``:
all ranks share cuda:0 (``pdist.local_device`` wraps), gloo stages the collectives through
the host.  What it checks on the real HIP kernels:

  * rank-specific init is overwritten by the rank-0 broadcast;
  * a full ``Pix2PixStep`` with per-network ``GradReducer`` s (small buckets -> several in
    flight, hooks firing during backward) leaves every rank with bitwise identical G and D
    parameters after Adam;
  * the reduced G gradient equals the mean of the per-shard single-process gradients;
  * the reference-family step (CompressGANStep: C + ExpandNetwork G + 3-scale SN PatchGAN
    D + VGG19 loss) with reducers on G and D: every D bucket is all-reduced exactly once per
    step (the G-loss backward, whose D gradients the reference discards, launches none), the
    reduced D gradient equals the mean of the ranks' local ones, and G / D / C stay bitwise
    identical across ranks over 3 steps (/root/reference/train.py:384-390).

Exit status 0 = pass; rank 0 prints one JSON line.  (The production path is RCCL over xGMI
with one GPU per rank; the driver's 8-GPU bench exercises that.)
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(seed, dev):
    from p2p_pytorch_amd.models import define_D, define_G
    torch.manual_seed(seed)
    # unet_4 at 128x128: every instance norm sees >= 16x16 pixels.  (Deeper U-Nets normalise
    # 2x2 maps, whose bf16 sensitivity makes ANY two batch compositions differ by ~10-20%:
    # tools/debug/batch_consistency.py)
    G = define_G(netG="unet_4", ngf=32, gpu_id=dev, verbose=False, use_dropout=False)
    D = define_D(6, 32, norm="instance", netD="basic", gpu_id=dev, verbose=False)
    return G, D


def data(world, dev, per=2, size=128):
    g = torch.Generator(device=dev).manual_seed(123)
    A = torch.rand(per * world, 3, size, size, device=dev, generator=g) * 2 - 1
    B = torch.rand(per * world, 3, size, size, device=dev, generator=g) * 2 - 1
    cl = torch.channels_last
    return A.to(torch.bfloat16).contiguous(memory_format=cl), B.to(torch.bfloat16).contiguous(memory_format=cl)


def g_grads(G, D, a, b):
    from p2p_pytorch_amd.models import GANLoss
    from p2p_pytorch_amd.ops import l1
    crit = GANLoss(gan_mode="vanilla")
    fake = G(a)
    loss = crit(D((a, fake)), True) + 100 * l1(fake, b)
    loss.backward()
    return loss


def family_r_phase(world, rank, dev, steps=3):
    """Reference-family step with reducers on the GPU kernels (see module docstring)."""
    from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
    from p2p_pytorch_amd.models import VGGLoss, define_C, define_D, define_G
    from p2p_pytorch_amd.parallel import GradReducer
    from p2p_pytorch_amd.parallel import dist as pdist
    torch.manual_seed(300 + rank)
    G = define_G(gpu_id=dev, verbose=False)
    D = define_D(6, 32, gpu_id=dev, verbose=False)
    C = define_C(gpu_id=dev, verbose=False)
    for m in (G, D, C):
        pdist.broadcast_module(m)
    torch.manual_seed(7)
    vgg = VGGLoss().to(dev)
    red_g, red_d = GradReducer(G, bucket_mb=1.0), GradReducer(D, bucket_mb=0.25)
    launches, local = [], {}
    orig = red_d._launch

    def spy(b):
        launches.append(b.index)
        local[b.index] = b.flat.detach().clone()
        orig(b)

    red_d._launch = spy
    step = CompressGANStep(G, D, C, vgg=vgg, reducer_g=red_g, reducer_d=red_d)
    g = torch.Generator(device=dev).manual_seed(321)
    cl = torch.channels_last
    worst, once, same = 0.0, True, True
    for _ in range(steps):
        A = (torch.rand(world, 3, 64, 64, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(world, 3, 64, 64, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        launches.clear()
        local.clear()
        step.step(A[rank:rank + 1].contiguous(memory_format=cl), B[rank:rank + 1].contiguous(memory_format=cl))
        torch.cuda.synchronize()
        once = once and sorted(launches) == list(range(len(red_d.buckets)))
        for bk in red_d.buckets:
            gl = [torch.zeros_like(local[bk.index]) for _ in range(world)]
            dist.all_gather(gl, local[bk.index])
            # the buckets hold the raw local gradients; the reduced bucket is their mean
            stk = torch.stack(gl).float()
            mean = stk.mean(0)
            worst = max(worst, float((bk.flat.float() - mean).abs().max() / mean.abs().max().clamp_min(1e-12)))
        for m in (G, D, C):
            f = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
            gg = [torch.zeros_like(f) for _ in range(world)]
            dist.all_gather(gg, f)
            same = same and all(torch.equal(gg[0], t) for t in gg)
    return {"d_buckets_once_per_step": once, "d_grad_rel_err_vs_rank_mean": worst,
            "params_identical": same, "ok": bool(once and same and worst < 1e-5)}


def direct_phase(world, rank, dev, a, b):
    """Direct bucket gradients: the conv weight gradients written into the
    buckets by the wgrad kernels (accumulate mode, weight-gradient side stream) must give
    bitwise the parameters of the autograd path after two Pix2Pix steps, on every rank, and
    the direct path must actually have been taken."""
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.parallel import GradReducer
    from p2p_pytorch_amd.parallel import dist as pdist
    n_direct = [0]
    orig = GradReducer.direct_done

    def counted(self, p, stream=None):
        n_direct[0] += 1
        return orig(self, p, stream)

    out = {}
    GradReducer.direct_done = counted
    try:
        for direct in (False, True):
            G, D = build(400 + rank, dev)
            pdist.broadcast_module(G)
            pdist.broadcast_module(D)
            rg, rd = GradReducer(G, bucket_mb=0.5, direct=direct), GradReducer(D, bucket_mb=0.5, direct=direct)
            step = Pix2PixStep(G, D, reducer_g=rg, reducer_d=rd)
            for _ in range(2):
                step.step(a, b)
            torch.cuda.synchronize()
            out[direct] = torch.cat([p.detach().reshape(-1) for p in list(G.parameters()) + list(D.parameters())])
            rg.remove()
            rd.remove()
    finally:
        GradReducer.direct_done = orig
    gathered = [torch.zeros_like(out[True]) for _ in range(world)]
    dist.all_gather(gathered, out[True])
    same_ranks = all(torch.equal(gathered[0], t) for t in gathered)
    equal = torch.equal(out[False], out[True])
    diff = float((out[False] - out[True]).abs().max())
    return {"direct_writes": n_direct[0], "direct_equals_autograd": equal, "max_abs_diff": diff,
            "ranks_identical": same_ranks, "ok": bool(n_direct[0] > 0 and equal and same_ranks)}


def main():
    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep, set_requires_grad
    from p2p_pytorch_amd.ops import hip
    from p2p_pytorch_amd.parallel import GradReducer
    from p2p_pytorch_amd.parallel import dist as pdist
    p2p.set_backend("native")
    p2p.set_deterministic(True)     # ordered split-K: the same shard gives the same bits
    world, rank, local_rank = pdist.init_from_env()
    dev = pdist.local_device(local_rank)
    torch.cuda.set_device(dev)
    per = 2
    A, B = data(world, dev, per)
    a, b = A[per * rank:per * (rank + 1)], B[per * rank:per * (rank + 1)]

    # ---- reduced G gradient == single-process gradient of the global batch
    G, D = build(100 + rank, dev)
    pdist.broadcast_module(G)
    pdist.broadcast_module(D)
    red = GradReducer(G, bucket_mb=0.5)
    set_requires_grad(D, False)
    hip.begin_step()
    red.zero_grad()
    g_grads(G, D, a, b)
    red.finish()
    got = {n: p.grad.detach().float().clone() for n, p in G.named_parameters()}
    worst = 0.0
    errs = []
    if rank == 0:
        # reference: the per-shard gradients computed single-process (same batch size as each
        # rank, so the same kernels and tile splits), averaged.  (Comparing against ONE
        # global-batch backward instead mixes in batch-size-dependent reduction orders,
        # which the bf16 U-Net amplifies chaotically -- tools/debug/batch_consistency.py.)
        ref = None
        for r in range(world):
            G1, D1 = build(100, dev)
            set_requires_grad(D1, False)
            hip.begin_step()
            g_grads(G1, D1, A[per * r:per * (r + 1)], B[per * r:per * (r + 1)])
            gr = {n: p.grad.detach().float().clone() for n, p in G1.named_parameters()}
            ref = gr if ref is None else {n: ref[n] + gr[n] for n in ref}
        for n in ref:
            rg = ref[n] / world
            scale = rg.abs().max().item()
            if scale < 1e-8 and got[n].abs().max().item() < 1e-8:
                continue        # exactly-zero grads (biases of norm-fed convs)
            err = ((got[n] - rg).abs().max() / max(scale, 1e-12)).item()
            errs.append((err, n, scale))
            worst = max(worst, err)
        errs.sort(reverse=True)
    # ---- full training steps with both reducers: parameters stay identical across ranks
    G, D = build(200 + rank, dev)
    pdist.broadcast_module(G)
    pdist.broadcast_module(D)
    # (timed reducers + phase timer: the JSONL comm / overlap path of train.py --log_json)
    from p2p_pytorch_amd.utils import PhaseTimer
    rg_, rd_ = GradReducer(G, bucket_mb=0.5).enable_timing(), GradReducer(D, bucket_mb=0.5).enable_timing()
    step = Pix2PixStep(G, D, reducer_g=rg_, reducer_d=rd_)
    step.timer = PhaseTimer()
    for _ in range(2):
        losses = step.step(a, b)
    torch.cuda.synchronize()
    comm = {"G": rg_.comm_stats(), "D": rd_.comm_stats()}
    phases = step.timer.report()
    timed = all(c.get("comm_ms", 0) > 0 and c.get("buckets", 0) > 1 for c in comm.values()) and \
        set(phases) >= {"G_fwd", "D_fwd", "D_bwd_opt", "G_bwd_opt"}
    flat = torch.cat([p.detach().reshape(-1) for p in list(G.parameters()) + list(D.parameters())])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    same = all(torch.equal(gathered[0], t) for t in gathered)
    finite = all(torch.isfinite(v).all().item() for v in losses.values())
    fam_r = family_r_phase(world, rank, dev)
    direct = direct_phase(world, rank, dev, a, b)
    ok = same and finite and worst < 1e-4 and timed and fam_r["ok"] and direct["ok"]
    if rank == 0:
        print(json.dumps({"world": world, "backend": dist.get_backend(), "grad_rel_err_vs_shard_mean": worst,
                          "worst_params": errs[:4],
                          "params_identical": same, "losses_finite": finite, "comm": comm,
                          "phase_ms": phases, "family_r": fam_r, "direct": direct, "ok": ok}), flush=True)
    pdist.destroy()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
