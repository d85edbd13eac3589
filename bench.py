#!/usr/bin/env python
"""Headline benchmark: pix2pix training throughput (train images/sec, whole job).

Config (BASELINE.json): 256x256 paired images, U-Net-256 generator (ngf 64, instance
norm, dropout) + 70x70 PatchGAN (basic, n_layers 3), GAN (BCE-with-logits) + 100*L1,
Adam(2e-4, 0.5/0.999), bf16 compute, synthetic data, random-init weights.  Weak
scaling: ``--batch`` images per GPU, one process per GPU (torchrun env), gradients
all-reduced over RCCL by ``p2p_pytorch_amd.parallel.GradReducer``.

    python bench.py --gpus N --steps K --warmup W [--batch B] [--impl native|torch]

``--impl torch`` runs the same model on stock PyTorch-ROCm eager kernels (MIOpen /
hipBLASLt, bf16 autocast, channels_last) -- the measured baseline of BASELINE.md.
Rank 0 prints one JSON line; ``value`` = total images/sec over all ranks, from the MAX
per-rank time of exactly K timed steps bracketed by barrier + device synchronize.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# Measured stock PyTorch-ROCm eager baseline (images/sec per GPU) for this exact config,
# recorded in BASELINE.md (stock PyTorch-ROCm eager, bf16 autocast, channels_last, per-GPU
# batch 128, cudnn.benchmark; profiles/eager_baseline_r1.jsonl).
EAGER_BASELINE_IMG_S_PER_GPU = 1790.23


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=None,
                   help="images per GPU (default: 2048 for the pix2pix headline; 512 for --family ref -- 256 / "
                        "512 measured 1035 / 1063 img/s captured at 52 / 104 GiB, "
                        "profiles/ab_r5/famr_batch_256_vs_512_r5ar.txt; 256 for --mode infer, 128 for --impl torch), sized for the 288 GB HBM: pix2pix 1024 / 1536 / 2048 measured "
                        "7387 / 7400 / 7444 img/s at 50.8 / 75.3 / 99.8 GiB (profiles/batch_sweep_r4.jsonl; "
                        "fp8 9951 / 10139 at 1024 / 2048); the eager baseline's best batch was 128")
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--family", default="pix2pix", choices=["pix2pix", "ref"],
                   help="pix2pix: the headline U-Net + PatchGAN step (BASELINE.json); ref: the reference "
                        "repo's own compression GAN step (C + ExpandNet G + 3-scale SN PatchGAN + VGG19 loss, "
                        "train.py:291-414), measured for parity, not the headline")
    p.add_argument("--mode", default="train", choices=["train", "infer"],
                   help="train: one full GAN step (the headline); infer: generator forward only "
                        "(test.py's path, eval mode, no grad) -- generated images/sec")
    p.add_argument("--netG", default="unet_256")
    p.add_argument("--netD", default="basic")
    p.add_argument("--impl", default=os.environ.get("P2P_BACKEND", "native"), choices=["native", "torch"])
    p.add_argument("--lamb", type=float, default=100.0)
    p.add_argument("--gan_mode", default="vanilla")
    p.add_argument("--bucket_mb", type=float, default=64.0)
    p.add_argument("--comm_dtype", default="fp32", choices=["fp32", "bf16"],
                   help="gradient all-reduce wire dtype (bf16: pre-scaled, half the xGMI bytes)")
    p.add_argument("--force_comm", action="store_true",
                   help="attach the reducers and issue the RCCL collectives even on one GPU")
    p.add_argument("--no_graph", action="store_true", help="(native) disable hipGraph capture")
    p.add_argument("--graph", action="store_true",
                   help="(native) hipGraph capture (the default for every N; kept for compatibility)")
    p.add_argument("--precision", default=os.environ.get("P2P_PRECISION", "bf16"), choices=["bf16", "fp8"],
                   help="(native) conv GEMM operands: bf16, or fp8 (e4m3 fwd / e5m2 dgrad / e5m2 x e4m3 "
                        "wgrad, image-facing layers bf16; BASELINE config 5)")
    p.add_argument("--c_phase_backward", type=int, default=1, choices=[0, 1],
                   help="(--family ref) run the reference's C-phase backward (locc.backward(),"
                        " train.py:400-402) even though with the reference's optimizer_c it updates"
                        " nothing -- 1 (default) times the reference's full step")
    p.add_argument("--json_out", default=None)
    return p.parse_args()


def main():
    args = parse()
    os.environ["P2P_BACKEND"] = args.impl
    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd.models import define_D, define_G
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.parallel import dist as pdist
    p2p.set_backend(args.impl)
    from p2p_pytorch_amd.ops import fp8 as _fp8
    if args.precision == "fp8" and args.impl != "native":
        raise SystemExit("--precision fp8 needs --impl native")
    _fp8.set_precision(args.precision)

    world, rank, local_rank = pdist.init_from_env()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}; launch with torchrun for N>1")
    dev = pdist.local_device(local_rank) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        torch.backends.cudnn.benchmark = True
    torch.manual_seed(123 + rank)

    ref = args.family == "ref"
    if ref:
        from p2p_pytorch_amd.models import define_C
        netG = define_G(netG="expand", gpu_id=dev, verbose=False)
        netD = define_D(6, 64, gpu_id=dev, netD="multiscale", verbose=False)
        netC = define_C(gpu_id=dev, verbose=False)
        pdist.broadcast_module(netC)
    else:
        netG = define_G(netG=args.netG, gpu_id=dev, verbose=False)
        netD = define_D(6, 64, norm="instance", netD=args.netD, gpu_id=dev, verbose=False)
    pdist.broadcast_module(netG)
    pdist.broadcast_module(netD)

    reducer_g = reducer_d = None
    if world > 1 or args.force_comm:
        from p2p_pytorch_amd.parallel import GradReducer
        if world == 1:
            pdist.init_single(dev)
        cdt = torch.bfloat16 if args.comm_dtype == "bf16" else None
        reducer_g = GradReducer(netG, bucket_mb=args.bucket_mb, comm_dtype=cdt,
                                force_comm=args.force_comm)
        reducer_d = GradReducer(netD, bucket_mb=args.bucket_mb, comm_dtype=cdt,
                                force_comm=args.force_comm)

    if args.impl == "torch":
        act_dtype = torch.float32
        mf = torch.channels_last
        autocast = torch.bfloat16 if dev.type == "cuda" else None
        netG.to(memory_format=mf)
        netD.to(memory_format=mf)
    else:
        act_dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        mf = torch.channels_last
        autocast = None
    if ref:
        from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
        trainer = CompressGANStep(netG, netD, netC, reducer_g=reducer_g, reducer_d=reducer_d,
                                  c_phase_backward=bool(args.c_phase_backward))
    else:
        trainer = Pix2PixStep(netG, netD, lr=2e-4, beta1=0.5, gan_mode=args.gan_mode,
                              lambda_L1=args.lamb, reducer_g=reducer_g, reducer_d=reducer_d,
                              autocast_dtype=autocast)

    if args.batch is None:
        # (fp8 at 2048 captures since round 5: CapturedStep releases the hand-off registries
        # and the allocator cache before capturing; 9908 vs 9679-9763 img/s at 1024, one box)
        args.batch = (512 if args.family == "ref" else 128 if args.impl == "torch"
                      else 256 if args.mode == "infer" else 2048)
    B, S = args.batch, args.size
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    real_A = (torch.rand(B, 3, S, S, device=dev, generator=gen) * 2 - 1).to(act_dtype)
    real_B = (torch.rand(B, 3, S, S, device=dev, generator=gen) * 2 - 1).to(act_dtype)
    real_A = real_A.contiguous(memory_format=mf)
    real_B = real_B.contiguous(memory_format=mf)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    step_fn = trainer.step
    if args.mode == "infer":
        gen_net = netG
        gen_net.eval()
        ctx = (torch.autocast(device_type="cuda", dtype=autocast) if autocast is not None
               else contextlib.nullcontext())

        def step_fn(a, b):    # noqa: ARG001 - same signature as the training step
            if a.is_cuda and args.impl == "native":
                from p2p_pytorch_amd.ops import hip
                hip.begin_step()
                hip.prepare_weights(gen_net)
            with torch.no_grad(), ctx:
                out = gen_net(netC(a) if ref else a)
            return {"out_mean": out.float().mean()}
    step = step_fn
    # one hipGraph per rank, RCCL bucket all-reduces captured inside it (graph-safe reducer,
    # tests/test_graph_gpu.py); ranks agree on graph vs eager so collectives always match
    # (gloo -- the one-GPU multi-rank rehearsal backend -- stages through the host and
    # cannot be captured; a failed capture leaves the process in capture mode, so only
    # RCCL process groups are captured)
    use_graph = (args.impl == "native" and dev.type == "cuda" and not args.no_graph
                 and (world == 1 or (pdist.backend() == "nccl"
                                     and os.environ.get("P2P_GRAPH_MULTI", "1") != "0")))
    cap_info = {"capture_error": None}
    if use_graph:
        from p2p_pytorch_amd.engine.graph import capture_agreed
        # capture runs its own warmup steps on a side stream, then records one step
        step, use_graph = capture_agreed(
            step_fn, real_A, real_B, warmup=2, info=cap_info,
            log=lambda m: print(f"[bench] rank {rank}: {m}", file=sys.stderr, flush=True))
    t_w = time.perf_counter()
    for i in range(args.warmup):
        losses = step(real_A, real_B)
        if rank == 0:   # heartbeat on stderr (eager cudnn.benchmark warmups can take minutes)
            sync()
            print(f"[bench] warmup {i + 1}/{args.warmup} {time.perf_counter() - t_w:.1f}s",
                  file=sys.stderr, flush=True)
    sync()
    pdist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = step(real_A, real_B)
    sync()
    pdist.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_max = pdist.max_scalar(dt, dev)
    loss_vals = {k: float(v) for k, v in losses.items()}
    comm = None
    if reducer_g is not None:
        # after (never inside) the timed region: ONE eager step with the reducers' collectives
        # on a timed side stream -> per-network all-reduce busy ms, the part left exposed
        # after backward's last kernel, and the overlap fraction (max over ranks)
        comm = {"dtype": args.comm_dtype, "bucket_mb": args.bucket_mb}
        if rank == 0:
            print("[bench] timed steps done; one eager step with timed collectives", file=sys.stderr, flush=True)
        for r in (reducer_g, reducer_d):
            r.enable_timing()
        trainer.step(real_A, real_B)
        sync()
        for tag, r in (("G", reducer_g), ("D", reducer_d)):
            st = r.comm_stats()
            r.enable_timing(False)
            if st:
                comm[tag] = {"comm_ms": round(pdist.max_scalar(st["comm_ms"], dev), 3),
                             "exposed_ms": round(pdist.max_scalar(st["exposed_ms"], dev), 3),
                             "overlap": round(pdist.min_scalar(st["overlap"], dev), 3),
                             "buckets": st["buckets"]}
    finite = all(v == v and abs(v) != float("inf") for v in loss_vals.values())

    img_s = world * B * args.steps / dt_max
    # the measured eager baseline is for the headline config only (256x256 pix2pix U-Net-256
    # + 70x70 PatchGAN training); other sizes / families / modes have no baseline
    headline = (not ref and args.mode == "train" and S == 256 and args.netG == "unet_256"
                and args.netD == "basic")
    base = EAGER_BASELINE_IMG_S_PER_GPU if headline else None
    model = (f"pix2pix {args.netG} + PatchGAN {args.netD} (70x70)" if not ref else
             "reference compression GAN: CompressionNetwork + ExpandNetwork + 3-scale SN PatchGAN + VGG19 loss")
    kind = "train" if args.mode == "train" else "inference (generator forward)"
    out = {
        "metric": (f"{kind} images/sec (whole node), {S}x{S} pix2pix U-Net+PatchGAN" if not ref else
                   f"{kind} images/sec (whole node), {S}x{S} reference compression GAN"),
        "value": round(img_s, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * dt_max / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(img_s / (base * world), 3) if base else None,
        "dtype": "fp8+bf16" if args.precision == "fp8" else "bf16",
        "data": "synthetic (random paired images, random-init weights)",
        "config": {"model": model,
                   "global_batch": world * B, "per_gpu_batch": B, "seq_len": None,
                   "image_size": S, "parallelism": f"dp{world}", "impl": args.impl,
                   "gan_mode": args.gan_mode, "lambda_L1": args.lamb,
                   "hipgraph": bool(use_graph),
                   # why a native run is eager (None: captured, or capture not attempted)
                   "capture_error": cap_info["capture_error"],
                   **({"c_phase_backward": bool(args.c_phase_backward)} if ref else {}),
                   "conv_precision": ("fp8: e4m3 fwd, e5m2 dgrad, e5m2 x e4m3 wgrad; image-facing first/last "
                                      "layers bf16" if args.precision == "fp8" else "bf16")},
        "max_mem_gib": (round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)
                        if dev.type == "cuda" else None),
        "comm": comm,
        # every non-default P2P_* knob of this run (an A/B setting must show in its line)
        "knobs": {k: v for k, v in sorted(os.environ.items())
                  if k.startswith("P2P_") and k not in ("P2P_BACKEND", "P2P_PRECISION")},
        "losses_finite": finite,
        "losses": loss_vals,
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    pdist.destroy()


if __name__ == "__main__":
    main()
