#!/usr/bin/env python
"""Training entry point -- flag-compatible with the reference ``train.py``
(/root/reference/train.py:133-157: every reference flag keeps its name and default).

Two model families behind one CLI:
  * reference family (default, ``--netG expand``): CompressionNetwork C + ExpandNetwork G
    + 3-scale spectral-norm PatchGAN D, LSGAN + feature matching + VGG19 + TV
    (engine/compress_gan.py, reference train.py:291-414);
  * pix2pix family (``--netG unet_256`` / ``unet_128`` / ``unet_<levels>``): U-Net + PatchGAN
    (``--netD basic | n_layers | pixel``), GAN + lamb * L1 (engine/pix2pix.py).

MI355X additions: one process per GPU (launch with ``torchrun --nproc-per-node N``), RCCL
gradient all-reduce bucketed and overlapped with backward (parallel/ddp.py), the HIP
kernels (``--backend native``, default on GPU), optional whole-step hipGraph capture on
one GPU (``--graph``), the dataset decoded once into HBM (``--device_cache``) or
synthetic pairs (``--synthetic``), JSONL metrics (``--log_json``), and checkpoints that
really resume (``--epoch_count N`` or ``--resume``).
"""
from __future__ import annotations

import argparse
import os
import random
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# the reference train.py's importable helpers (train.py:33-126), same names and signatures
from p2p_pytorch_amd.engine.ref_helpers import (  # noqa: E402,F401
    calc_c_loss, calc_Gram_Loss, calc_tv_Loss, extract_features, gram, load_checkpoint, psnr,
    ssim, tensor2img, tensor2np)


def build_parser():
    p = argparse.ArgumentParser(description="pix2pix-pytorch-implementation")
    # ---- reference flags (train.py:134-156), same names and defaults
    p.add_argument("--dataset", default=None, help="facades (dataset/<name>/{train,test}/{a,b})")
    p.add_argument("--name", default="run", help="training name")
    p.add_argument("--epoch_count", type=int, default=1, help="the starting epoch count")
    p.add_argument("--nepoch", type=int, default=50, help="# of epoch")
    p.add_argument("--niter", type=int, default=100, help="# of iter at starting learning rate")
    p.add_argument("--niter_decay", type=int, default=100,
                   help="# of iter to linearly decay learning rate to zero")
    p.add_argument("--cuda", action="store_true", help="use cuda?")
    p.add_argument("--epochsave", type=int, default=50, help="checkpoint every N epochs")
    p.add_argument("--batch_size", type=int, default=1, help="training batch size (per GPU)")
    p.add_argument("--test_batch_size", type=int, default=1, help="testing batch size")
    p.add_argument("--direction", type=str, default="b2a", help="a2b or b2a")
    p.add_argument("--input_nc", type=int, default=3, help="input image channels")
    p.add_argument("--output_nc", type=int, default=3, help="output image channels")
    p.add_argument("--ngf", type=int, default=64, help="generator filters in first conv layer")
    p.add_argument("--ndf", type=int, default=64, help="discriminator filters in first conv layer")
    p.add_argument("--lr", type=float, default=0.0002, help="initial learning rate for adam")
    p.add_argument("--lr_policy", type=str, default="lambda",
                   help="learning rate policy: lambda|step|plateau|cosine")
    p.add_argument("--lr_decay_iters", type=int, default=50,
                   help="multiply by a gamma every lr_decay_iters iterations")
    p.add_argument("--beta1", type=float, default=0.5, help="beta1 for adam. default=0.5")
    p.add_argument("--threads", type=int, default=4, help="number of threads for data loader")
    p.add_argument("--seed", type=int, default=123, help="random seed to use. Default=123")
    p.add_argument("--lamb", type=float, default=10, help="weight on L1 term in objective")
    # ---- new
    p.add_argument("--netG", default="expand", help="expand | unet_256 | unet_128 | unet_<levels>")
    p.add_argument("--netD", default=None, help="multiscale | basic | n_layers | pixel")
    p.add_argument("--n_layers_D", type=int, default=3)
    p.add_argument("--norm", default="instance", help="instance | batch | none (pix2pix family)")
    p.add_argument("--no_dropout", action="store_true", help="pix2pix U-Net without dropout")
    p.add_argument("--gan_mode", default=None, help="lsgan | vanilla | bce (default per family)")
    p.add_argument("--backend", default=None, choices=["native", "torch"],
                   help="GPU kernels: native HIP (default) or stock PyTorch eager")
    p.add_argument("--synthetic", action="store_true", help="synthetic paired images, no dataset")
    p.add_argument("--image_size", type=int, default=256, help="synthetic image size")
    p.add_argument("--steps_per_epoch", type=int, default=100, help="synthetic steps per epoch")
    p.add_argument("--device_cache", action="store_true",
                   help="decode the training set once into GPU memory (uint8) and batch there")
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp8"],
                   help="(native) conv GEMM operand precision: bf16, or fp8 (e4m3 fwd / e5m2 dgrad)")
    p.add_argument("--deterministic", action="store_true",
                   help="(native) bitwise-repeatable kernels (ordered split-K reduction)")
    p.add_argument("--graph", action="store_true", help="capture the training step in a hipGraph")
    p.add_argument("--bucket_mb", type=float, default=64.0, help="gradient all-reduce bucket size")
    p.add_argument("--train_c", action="store_true",
                   help="reference family: really train C (straight-through quantiser)")
    p.add_argument("--c_phase_backward", action="store_true",
                   help="reference family: run the C-phase backward the reference runs (no effect)")
    p.add_argument("--bits", type=int, default=3, help="quantiser bits (reference: 3)")
    p.add_argument("--checkpoint_dir", default="checkpoint")
    p.add_argument("--resume", action="store_true", help="resume from the newest checkpoint")
    p.add_argument("--log_every", type=int, default=50)
    p.add_argument("--log_json", default=None, help="append JSONL metrics here (rank 0)")
    p.add_argument("--phase_times", type=int, default=None,
                   help="per-phase HIP-event ms and RCCL comm / overlap stats in the JSONL stream "
                        "(default: on with --log_json and no --graph)")
    p.add_argument("--no_eval", action="store_true")
    p.add_argument("--no_nan_guard", action="store_true",
                   help="apply updates even when a loss is NaN/Inf (default: skip on device)")
    p.add_argument("--watchdog_s", type=float, default=None,
                   help="abort (exit 124) when no step finishes for this long; default 1800 s "
                        "for multi-GPU runs, off for one GPU")
    p.add_argument("--max_eval", type=int, default=0, help="limit eval images (0 = all)")
    p.add_argument("--no_eval_images", dest="eval_images", action="store_false",
                   help="do not write the reference's in/tar/pred/comp.png eval samples")
    return p


def main(argv=None):
    opt = build_parser().parse_args(argv)
    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd.data import (DevicePairCache, SyntheticPairs, get_test_set,
                                      get_training_set)
    from p2p_pytorch_amd.data.image_io import save_img
    from p2p_pytorch_amd.engine.checkpoint import (checkpoint_path, scheduler_offset,
                                                   latest_checkpoint, save_checkpoint)
    from p2p_pytorch_amd.engine.checkpoint import load_checkpoint as load_full_checkpoint
    from p2p_pytorch_amd.engine.metrics import image_metrics
    from p2p_pytorch_amd.models import (define_C, define_D, define_G, get_scheduler,
                                        update_learning_rate)
    from p2p_pytorch_amd.parallel import dist as pdist

    world, rank, local_rank = pdist.init_from_env()
    use_cuda = (opt.cuda or world > 1 or opt.backend == "native") and torch.cuda.is_available()
    if opt.cuda and not torch.cuda.is_available():
        raise Exception("No GPU found, please run without --cuda")
    device = pdist.local_device(local_rank) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    p2p.set_backend(opt.backend or "native")
    p2p.set_precision(opt.precision)
    if opt.deterministic:
        p2p.set_deterministic(True)
    if rank == 0:
        print(opt)
    torch.manual_seed(opt.seed)
    random.seed(opt.seed + rank)
    if use_cuda:
        torch.cuda.manual_seed(opt.seed)
    pix2pix = opt.netG.startswith("unet")
    act_dtype = torch.bfloat16 if (use_cuda and p2p.get_backend() == "native") else torch.float32

    # ---- data
    if opt.synthetic:
        train_src = SyntheticPairs(opt.batch_size, opt.image_size, device, seed=opt.seed + rank,
                                   dtype=act_dtype, bits=opt.bits, direction=opt.direction)
        test_set = None
    else:
        if not opt.dataset:
            raise SystemExit("--dataset is required unless --synthetic")
        root = os.path.join("dataset", opt.dataset)
        train_set = get_training_set(root, opt.direction)
        test_set = get_test_set(root, opt.direction)
        if opt.device_cache and use_cuda:
            train_src = DevicePairCache(train_set, device, rank, world, seed=opt.seed)
        else:
            sampler = (torch.utils.data.distributed.DistributedSampler(
                train_set, num_replicas=world, rank=rank, shuffle=True, seed=opt.seed)
                if world > 1 else None)
            train_src = torch.utils.data.DataLoader(
                train_set, batch_size=opt.batch_size, shuffle=sampler is None, sampler=sampler,
                num_workers=opt.threads, drop_last=world > 1 or opt.graph)

    # ---- models
    if rank == 0:
        print("===> Building models")
    if pix2pix:
        net_g = define_G(netG=opt.netG, input_nc=opt.input_nc, output_nc=opt.output_nc,
                         ngf=opt.ngf, norm=opt.norm, use_dropout=not opt.no_dropout,
                         gpu_id=device, verbose=rank == 0)
        net_d = define_D(opt.input_nc + opt.output_nc, opt.ndf, norm=opt.norm,
                         netD=opt.netD or "basic", n_layers_D=opt.n_layers_D, gpu_id=device,
                         verbose=rank == 0)
        net_c = None
    else:
        net_g = define_G("normal", 0.02, gpu_id=device, verbose=rank == 0)
        net_d = define_D(opt.input_nc + opt.output_nc, opt.ndf, gpu_id=device,
                         netD=opt.netD or "multiscale", n_layers_D=opt.n_layers_D,
                         verbose=rank == 0)
        net_c = define_C("normal", 0.02, gpu_id=device, verbose=rank == 0)
    for net in (net_g, net_d, net_c):
        if net is not None:
            pdist.broadcast_module(net)
    reducer_g = reducer_d = reducer_c = None
    if world > 1:
        from p2p_pytorch_amd.parallel import GradReducer
        reducer_g = GradReducer(net_g, bucket_mb=opt.bucket_mb)
        reducer_d = GradReducer(net_d, bucket_mb=opt.bucket_mb)
        if net_c is not None and opt.train_c:
            # --train_c steps an Adam over C: its gradients are all-reduced like G's and D's
            # (and the NaN-skip decision is agreed through this reducer)
            reducer_c = GradReducer(net_c, bucket_mb=opt.bucket_mb)

    if pix2pix:
        from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
        trainer = Pix2PixStep(net_g, net_d, lr=opt.lr, beta1=opt.beta1,
                              gan_mode=opt.gan_mode or "vanilla", lambda_L1=opt.lamb,
                              reducer_g=reducer_g, reducer_d=reducer_d,
                              autocast_dtype=torch.bfloat16 if (use_cuda and p2p.get_backend() == "torch") else None,
                              nan_guard=not opt.no_nan_guard)
        opt_g, opt_d = trainer.opt_G, trainer.opt_D
    else:
        from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
        from p2p_pytorch_amd.models import ImagePool
        trainer = CompressGANStep(net_g, net_d, net_c, lr=opt.lr, beta1=opt.beta1, bits=opt.bits,
                                  n_layers_d=opt.n_layers_D, image_pool=ImagePool(0),
                                  train_c=opt.train_c, c_phase_backward=opt.c_phase_backward,
                                  reducer_g=reducer_g, reducer_d=reducer_d, reducer_c=reducer_c,
                                  nan_guard=not opt.no_nan_guard)
        opt_g, opt_d = trainer.opt_g, trainer.opt_d
    # the reference's third optimizer / scheduler pair (train.py:243-246, :441-443): over C
    # when --train_c fixes quirk A1, and stepped + checkpointed like the other two
    opt_c = getattr(trainer, "opt_c", None)

    # ---- resume
    start_epoch = opt.epoch_count
    losslogger = []
    ck_path = None
    if opt.resume:
        ck_path, ep = latest_checkpoint(opt.checkpoint_dir, opt.dataset or "synthetic", opt.name)
        if ck_path:
            start_epoch = ep + 1
    elif opt.epoch_count > 1:
        ck_path = checkpoint_path(opt.checkpoint_dir, opt.dataset or "synthetic", opt.name,
                                  opt.epoch_count - 1)
        if not os.path.exists(ck_path):
            raise SystemExit(f"=> No checkpoint found at '{ck_path}'")
    # a restored scheduler already counts the finished epochs (last_epoch): its lambda keeps
    # the offset of the run that built it (saved as sched_epoch_count), not this run's
    # epoch_count; a reference-written file (no scheduler state) starts a fresh scheduler
    # whose lambda is offset by epoch_count, as in the reference
    sched_epoch_count = opt.epoch_count
    if ck_path:
        off = scheduler_offset(ck_path)
        if off is not None:
            sched_epoch_count = off
    sched_opt = argparse.Namespace(**{**vars(opt), "epoch_count": sched_epoch_count})
    sched_g = get_scheduler(opt_g, sched_opt)
    sched_d = get_scheduler(opt_d, sched_opt)
    sched_c = get_scheduler(opt_c, sched_opt) if opt_c is not None else None
    if ck_path:
        if rank == 0:
            print(f"=> Loading checkpoint '{ck_path}'")
        start_epoch, losslogger = load_full_checkpoint(
            ck_path, net_g, net_c, net_d, opt_g, opt_d, sched_g, sched_d, device=device,
            opt_c=opt_c, sched_c=sched_c)

    from p2p_pytorch_amd.utils import JsonlLogger, StepWatchdog
    step_fn = trainer.step
    num_epoch = opt.nepoch + 1
    jlog = JsonlLogger(opt.log_json, rank)
    timing = (opt.phase_times if opt.phase_times is not None else bool(opt.log_json and not opt.graph))
    if timing and use_cuda:
        from p2p_pytorch_amd.utils import PhaseTimer
        trainer.timer = PhaseTimer()
        for r in (reducer_g, reducer_d, reducer_c):
            if r is not None:
                r.enable_timing()
    wd_s = opt.watchdog_s if opt.watchdog_s is not None else (1800.0 if world > 1 else 0.0)
    watchdog = StepWatchdog(wd_s).start()
    graph_tried = False
    for epoch in range(start_epoch, num_epoch):
        net_g.train()
        net_d.train()
        sums, count, t0 = {}, 0, time.perf_counter()
        if hasattr(train_src, "sampler") and hasattr(train_src.sampler, "set_epoch"):
            train_src.sampler.set_epoch(epoch)
        if isinstance(train_src, DevicePairCache):
            train_src.new_epoch()
            n_it = train_src.batches_per_epoch(opt.batch_size)
            batches = (train_src.next_batch(opt.batch_size, act_dtype) for _ in range(n_it))
        elif isinstance(train_src, SyntheticPairs):
            n_it = opt.steps_per_epoch
            batches = (train_src.next_batch() for _ in range(n_it))
        else:
            n_it = len(train_src)
            batches = iter(train_src)
        for iteration, batch in enumerate(batches, 1):
            real_a = batch[0].to(device, act_dtype).contiguous(memory_format=torch.channels_last)
            real_b = batch[1].to(device, act_dtype).contiguous(memory_format=torch.channels_last)
            if opt.graph and use_cuda and step_fn is trainer.step and not graph_tried:
                # RCCL groups only, and every rank agrees on graph vs eager (a capture that
                # fails on one rank must not leave the others blocked in its collectives)
                from p2p_pytorch_amd.engine.graph import capture_agreed
                graph_tried = True
                step_fn, _ = capture_agreed(
                    trainer.step, real_a, real_b,
                    log=lambda m: print(f"[train] rank {rank}: {m}", file=sys.stderr, flush=True))
            losses = step_fn(real_a, real_b)
            watchdog.beat()
            for k, v in losses.items():   # device-side running sums, no host sync
                sums[k] = sums.get(k, 0) + v.detach().float()
            count += 1
            if iteration % opt.log_every == 0 or iteration == n_it:
                keys = sorted(sums)
                vals = torch.stack([torch.as_tensor(sums[k], device=device).float() for k in keys])
                pdist.all_reduce_mean_([vals])
                extra = {}   # every rank drains its timers; rank 0 logs
                if getattr(trainer, "timer", None) is not None:
                    extra["phase_ms"] = {k: v / count for k, v in trainer.timer.report().items()}
                    for tag, r in (("G", reducer_g), ("D", reducer_d), ("C", reducer_c)):
                        st = r.comm_stats() if r is not None else {}
                        if st:
                            extra[f"comm_{tag}"] = st
                if rank == 0:
                    means = {k: float(v) / count for k, v in zip(keys, vals.tolist())}
                    dt = time.perf_counter() - t0
                    ips = count * opt.batch_size * world / max(dt, 1e-9)
                    head = "itr: %d/%d [%3d/%3d] " % (iteration, n_it, epoch, num_epoch - 1)
                    if not pix2pix:
                        # the reference's progress line (train.py:421-436); its "C" field is
                        # the VGG content loss, DGC = D / G-GAN / C-phase losses
                        print(head + "[DGC: %.6f/%.6f/%.6f] [GF: %.6f] [C: %.6f] [TV: %.6f] "
                              "[Tot: %.6f]" % (means["D"], means["G_GAN"], means["C"],
                                               means["G_GAN_Feat"], means["VGG"], means["TV"],
                                               means["G"]) + f" [{ips:.1f} img/s]", flush=True)
                    else:
                        print(head + " ".join(f"[{k}: {means[k]:.6f}]" for k in keys) +
                              f" [{ips:.1f} img/s]", flush=True)
                    skipped = getattr(trainer, "skipped", None)
                    jlog.log(epoch=epoch, iter=iteration, img_s=ips,
                             skipped_updates=float(skipped) if skipped is not None else 0.0,
                             **means, **extra)
        update_learning_rate(sched_g, opt_g, verbose=rank == 0)
        update_learning_rate(sched_d, opt_d, verbose=rank == 0)
        if sched_c is not None:
            update_learning_rate(sched_c, opt_c, verbose=rank == 0)
        for o in (opt_g, opt_d, opt_c):
            if hasattr(o, "sync_lr"):
                o.sync_lr()
        jlog.log(epoch=epoch, lr_g=opt_g.param_groups[0]["lr"], lr_d=opt_d.param_groups[0]["lr"])

        # ---- eval (train.py:450-502), no autograd
        if test_set is not None and not opt.no_eval:
            net_g.eval()
            net_d.eval()
            if net_c is not None:
                net_c.eval()
            ps, ss = [], []
            n_eval = len(test_set) if not opt.max_eval else min(opt.max_eval, len(test_set))
            # one random test image's input / target / prediction / compressed view is dumped
            # to in.png, tar.png, pred.png, comp.png (train.py:462, :469-473; the reference's
            # inclusive randint bound can miss every image, quirk A14)
            # drawn from rank 0's shard (i = 0 mod world): rank 0 writes the images
            rande = random.randrange(0, max(n_eval, 1), world)
            with torch.no_grad():
                for i in range(rank, n_eval, world):
                    inp, tgt = test_set[i]
                    inp = inp.unsqueeze(0).to(device, act_dtype).contiguous(memory_format=torch.channels_last)
                    tgt = tgt.unsqueeze(0).to(device, act_dtype).contiguous(memory_format=torch.channels_last)
                    comp = None
                    if net_c is not None:
                        from p2p_pytorch_amd import ops
                        comp = ops.quantize(net_c(tgt), opt.bits)
                        pred = net_g(comp)
                    else:
                        pred = net_g(inp)
                    if i == rande and opt.eval_images and rank == 0:
                        save_img(inp[0].float().cpu(), "in.png")
                        save_img(tgt[0].float().cpu(), "tar.png")
                        save_img(pred[0].float().cpu(), "pred.png")
                        if comp is not None:
                            save_img(comp[0].float().cpu(), "comp.png")
                    p_i, s_i = image_metrics(pred, tgt)   # one HIP kernel on the GPU
                    ps.append(p_i.clamp(max=60.0))
                    ss.append(s_i)
            if ps:
                pt, st = torch.cat(ps), torch.cat(ss)
                stats = torch.stack([pt.sum(), st.sum(), torch.tensor(float(len(pt)), device=pt.device),
                                     pt.max(), st.max()])
            else:
                stats = torch.zeros(5, device=device)
            if world > 1:
                import torch.distributed as dist
                agg = stats[:3].clone()
                dist.all_reduce(agg)
                mx = stats[3:].clone()
                dist.all_reduce(mx, op=dist.ReduceOp.MAX)
                stats = torch.cat([agg, mx])
            if rank == 0:
                n = max(float(stats[2]), 1.0)
                print("===> Avg. PSNR: {:.4f} dB".format(float(stats[0]) / n))
                print("===> Avg. SSIM: {:.4f}".format(float(stats[1]) / n))
                print("===> Max PSNR: {:.4f} dB".format(float(stats[3])))
                print("===> Max SSIM: {:.4f}".format(float(stats[4])))

        if epoch % opt.epochsave == 0:
            path = checkpoint_path(opt.checkpoint_dir, opt.dataset or "synthetic", opt.name, epoch)
            save_checkpoint(path, epoch, net_g, net_c, net_d, opt_g, opt_d, sched_g, sched_d,
                            losslogger, rank=rank, opt_c=opt_c, sched_c=sched_c,
                            extra={"sched_epoch_count": sched_epoch_count})
            pdist.barrier()
            if rank == 0:
                print("Checkpoint saved to {}".format(path))
    watchdog.stop()
    jlog.close()
    pdist.destroy()


if __name__ == "__main__":
    main()
