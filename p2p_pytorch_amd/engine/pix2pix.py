"""Family-P training step: conditional GAN (U-Net G, PatchGAN D) with GAN + lambda*L1.

Phase order per step (explicit, so the DP reducer can sync each network at its own
backward -- SURVEY.md section 5.8):

  1. ``fake_B = G(real_A)``
  2. D phase: ``D(cat(A, fake_B.detach()))`` vs fake label, ``D(cat(A, B))`` vs real label,
     ``loss_D = 0.5 * (fake + real)`` -> backward -> all-reduce D grads -> Adam(D)
  3. G phase (D params frozen, so D only back-propagates to its input):
     ``D(cat(A, fake_B))`` vs real label + ``lambda_L1 * |fake_B - B|`` -> backward ->
     all-reduce G grads -> Adam(G)

The concat of (A, fake_B) is a *virtual* concat on the native path: D's first conv reads
the two images through two base pointers (``ops.conv2d`` accepts a tuple input).
Loss values stay on the device; nothing syncs the host inside ``step``.
"""
from __future__ import annotations

import contextlib

import torch

from .. import _native
from ..models.compress_gan import MultiscaleDiscriminator
from ..models.layers import BatchNorm2d
from ..models.losses import GANLoss
from ..ops import l1
from ..utils.tracing import trace_range
from .optim import guarded_step, make_adam


def set_requires_grad(nets, flag: bool):
    for net in nets if isinstance(nets, (list, tuple)) else [nets]:
        for p in net.parameters():
            p.requires_grad_(flag)


class Pix2PixStep:
    def __init__(self, netG, netD, lr=2e-4, beta1=0.5, gan_mode="vanilla", lambda_L1=100.0,
                 reducer_g=None, reducer_d=None, autocast_dtype=None, fuse_d_batch=None,
                 nan_guard=True, packed=None):
        self.netG, self.netD = netG, netD
        self.criterionGAN = GANLoss(gan_mode=gan_mode)
        self.lambda_L1 = float(lambda_L1)
        self.opt_G = make_adam(netG.parameters(), lr=lr, betas=(beta1, 0.999))
        self.opt_D = make_adam(netD.parameters(), lr=lr, betas=(beta1, 0.999))
        self.reducer_g, self.reducer_d = reducer_g, reducer_d
        self.autocast_dtype = autocast_dtype
        # D(fake.detach()) and D(real) as ONE 2B-batch forward/backward, halving D launches
        # and doubling GEMM M -- only when D is per-sample: a BatchNorm would take its
        # statistics over fake and real together (and update its running stats once)
        self.d_per_sample = not any(isinstance(m, (BatchNorm2d, torch.nn.BatchNorm2d))
                                    for m in netD.modules())
        self.fuse_d_batch = fuse_d_batch
        # packed-image path (native backend, U-Net + PatchGAN on 3 + 3 channels): None = auto
        self.packed = packed
        # NaN/Inf guard: a non-finite loss skips that network's update on the device (no
        # host sync; agreed across ranks with one 4-byte MAX all-reduce) and is counted
        self.nan_guard = nan_guard
        dev = next(netG.parameters()).device
        self.skipped = torch.zeros((), device=dev) if nan_guard else None
        self.timer = None     # optional utils.PhaseTimer: per-phase HIP-event ms

    def optimizers(self):
        return [self.opt_G, self.opt_D]

    def state_tensors(self):
        """Tensors one step mutates (CapturedStep snapshots them around its warmup)."""
        from .graph import trainer_state_tensors
        extra = [self.skipped] if self.skipped is not None else []
        dev = next(self.netG.parameters()).device
        if dev.type == "cuda" and _native.get_backend() == "native":
            from ..ops import hip
            extra.append(hip._seed(dev))
        return trainer_state_tensors([self.netG, self.netD], self.optimizers(), extra)

    def _phase(self, name):
        return self.timer.phase(name) if self.timer is not None else trace_range(name)

    def _guarded_step(self, opt, reducer, *losses):
        if not self.nan_guard:
            opt.step()
            return
        self.skipped = guarded_step(opt, reducer, self.skipped, *losses)

    def _ctx(self, device):
        if self.autocast_dtype is not None:
            return torch.autocast(device_type=device.type, dtype=self.autocast_dtype)
        return contextlib.nullcontext()

    def _seed_grad(self, loss):
        """d(loss)/d(loss) = 1 as a persistent device tensor (no fill kernel per backward)."""
        seeds = self.__dict__.setdefault("_seeds", {})
        key = (loss.device, loss.dtype, tuple(loss.shape))
        s = seeds.get(key)
        if s is None:
            s = seeds[key] = torch.ones(loss.shape, device=loss.device, dtype=loss.dtype)
        return s

    @staticmethod
    def _zero(opt, reducer):
        # with a reducer, grads are views into its flat buckets: zero in place
        if reducer is not None:
            reducer.zero_grad()
        else:
            opt.zero_grad(set_to_none=True)

    def _d_input(self, a, b):
        # the eager baseline materialises the concat; the native conv reads a tuple
        if a.is_cuda and _native.get_backend() == "native":
            return (a, b)
        return torch.cat((a, b), 1)

    def _packed_ok(self, real_A, real_B):
        """The packed-image path (ops/hip.py image head): U-Net G and a 4x4 s2 p1 PatchGAN
        on 3 + 3 channel images, the 2B D batch, vanilla / lsgan losses."""
        from ..models.pix2pix import NLayerDiscriminator, PixelDiscriminator, UnetGenerator
        if self.packed is False or self.fuse_d_batch is False or not self.d_per_sample:
            return False
        if not (isinstance(self.netG, UnetGenerator) and self.netG.packed_ok(real_A)):
            return False
        if not isinstance(self.netD, NLayerDiscriminator) or isinstance(self.netD, PixelDiscriminator):
            return False
        c0 = self.netD.convs[0]
        return (real_A.shape[1] == 3 and real_B.shape[1] == 3 and c0.in_channels == 6
                and tuple(c0.kernel_size) == (4, 4) and c0.stride[0] == 2 and c0.padding[0] == 1
                and c0.weight.shape[0] % 64 == 0 and real_A.shape == real_B.shape)

    def step(self, real_A, real_B):
        netG, netD = self.netG, self.netD
        native = real_A.is_cuda and _native.get_backend() == "native"
        if native:
            from ..ops import hip
            hip.begin_step()      # weight images re-cast once per step (graph-safe)
            hip.advance_rng(real_A.device)     # new dropout masks
            hip.prepare_weights(netG, netD)   # all bf16 weight images, one launch each
            if self._packed_ok(real_A, real_B):
                return self._step_packed(real_A, real_B)
        return self._step_unpacked(real_A, real_B)

    def _step_packed(self, real_A, real_B):
        """Same phases as ``_step_unpacked`` on the packed pair tensor dd = [(A | fake);
        (A | B)] (2B x 8 channels, 16 B per pixel): G reads (A | B) and writes (A | fake) in
        place with the L1 term; D's two halves are its fused D batch; the G-phase D backward
        returns G's pre-tanh gradient with the L1 term fused (ops/hip.py image head)."""
        from ..ops import hip
        netG, netD = self.netG, self.netD
        B, _, H, W = real_A.shape
        dd = torch.empty(2 * B, 8, H, W, device=real_A.device, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        hip.P().pad_channels_into(hip.to_nhwc_bf16(real_A), hip.to_nhwc_bf16(real_B),
                                  dd.narrow(0, B, B))
        dd._p2p_packed = (3, 3)
        scale = self.lambda_L1 / float(B * 3 * H * W)
        with self._phase("G_fwd"):
            fake_pk, loss_G_L1 = netG.forward_packed(dd, scale)
        with self._phase("D_fwd"):
            set_requires_grad(netD, True)
            pred = netD(dd)                   # [D(A | fake.detach()); D(A | B)], one 2B pass
            pred_fake, pred_real = hip.batch_halves(pred, B)
            loss_D_fake = self.criterionGAN(pred_fake, False)
            loss_D_real = self.criterionGAN(pred_real, True)
            loss_D = hip.lincomb(loss_D_fake, loss_D_real, 0.5, 0.5)
        with self._phase("D_bwd_opt"):
            self._zero(self.opt_D, self.reducer_d)
            with hip.wgrad_overlap(real_A.device):
                loss_D.backward(self._seed_grad(loss_D))
            if self.reducer_d is not None:
                self.reducer_d.finish()
            self._guarded_step(self.opt_D, self.reducer_d, loss_D)
        hip.prepare_weights(netD)             # D moved: fresh images for the G phase
        set_requires_grad(netD, False)
        with self._phase("G_loss_fwd"):
            pred_fake = netD(fake_pk)
            loss_G_GAN = self.criterionGAN(pred_fake, True)
            # the L1 term's gradient is fused into D's first-conv dgrad; the tap hands that
            # kernel dL/d(L1) on the device (any weighting of the L1 term is honoured)
            loss_G = hip.lincomb(loss_G_GAN, hip.head_l1_tap(loss_G_L1))
        with self._phase("G_bwd_opt"):
            self._zero(self.opt_G, self.reducer_g)
            with hip.wgrad_overlap(real_A.device):
                loss_G.backward(self._seed_grad(loss_G))
            hip.assert_no_deferred()          # every parked U-Net skip gradient consumed
            if self.reducer_g is not None:
                self.reducer_g.finish()
            self._guarded_step(self.opt_G, self.reducer_g, loss_G)
        return {"D": loss_D.detach(), "G_GAN": loss_G_GAN.detach(), "G_L1": loss_G_L1.detach(),
                "G": loss_G.detach()}

    def _step_unpacked(self, real_A, real_B):
        netG, netD = self.netG, self.netD
        with self._ctx(real_A.device), self._phase("G_fwd"):
            fake_B = netG(real_A)
        with self._ctx(real_A.device), self._phase("D_fwd"):
            # ---- D
            set_requires_grad(netD, True)
            fuse = self.fuse_d_batch
            if fuse is None:
                fuse = (real_A.is_cuda and _native.get_backend() == "native"
                        and not isinstance(netD, MultiscaleDiscriminator))
            fuse = fuse and self.d_per_sample
            if fuse:
                B = real_A.shape[0]
                if (real_A.is_cuda and _native.get_backend() == "native"
                        and (real_A.shape[1] + real_B.shape[1]) % 8):
                    # packed pad-8 image input, both halves written in place (no cat)
                    from ..ops import hip
                    d_in = hip.pack_pairs([(real_A, fake_B.detach()), (real_A, real_B)])
                else:
                    d_in = self._d_input(torch.cat((real_A, real_A), 0),
                                         torch.cat((fake_B.detach(), real_B), 0))
                pred = netD(d_in)
                loss_D_fake = self.criterionGAN(pred[:B], False)
                loss_D_real = self.criterionGAN(pred[B:], True)
            else:
                pred_fake = netD(self._d_input(real_A, fake_B.detach()))
                loss_D_fake = self.criterionGAN(pred_fake, False)
                pred_real = netD(self._d_input(real_A, real_B))
                loss_D_real = self.criterionGAN(pred_real, True)
            loss_D = (loss_D_fake + loss_D_real) * 0.5
        with self._phase("D_bwd_opt"):
            self._zero(self.opt_D, self.reducer_d)
            loss_D.backward()
            if self.reducer_d is not None:
                self.reducer_d.finish()
            self._guarded_step(self.opt_D, self.reducer_d, loss_D)
        if real_A.is_cuda and _native.get_backend() == "native":
            from ..ops import hip
            hip.prepare_weights(netD)         # D moved: fresh images for the G phase
        # ---- G
        set_requires_grad(netD, False)
        with self._ctx(real_A.device), self._phase("G_loss_fwd"):
            pred_fake = netD(self._d_input(real_A, fake_B))
            loss_G_GAN = self.criterionGAN(pred_fake, True)
            loss_G_L1 = l1(fake_B, real_B) * self.lambda_L1
            loss_G = loss_G_GAN + loss_G_L1
        with self._phase("G_bwd_opt"):
            self._zero(self.opt_G, self.reducer_g)
            loss_G.backward()
            if real_A.is_cuda and _native.get_backend() == "native":
                from ..ops import hip
                hip.assert_no_deferred()      # every parked U-Net skip gradient consumed
            if self.reducer_g is not None:
                self.reducer_g.finish()
            self._guarded_step(self.opt_G, self.reducer_g, loss_G)
        return {"D": loss_D.detach(), "G_GAN": loss_G_GAN.detach(), "G_L1": loss_G_L1.detach(),
                "G": loss_G.detach()}
