"""Family-R training step: the reference's compression + bit-depth-expansion GAN
(/root/reference/train.py:291-414), phase for phase.

  compressed = quantize(C(real_b), 3)                     train.py:297
  fake_b     = G(compressed.detach())                     :300
  D loss     : LSGAN(D(pool(cat(a, fake.detach()))), 0) + LSGAN(D(cat(a, b)), 1), x0.5
  G loss     : LSGAN(D(cat(a, fake)), 1)                  :336-338
               + 10 * sum_scales sum_layers (1/3)(4/4) L1(feat_fake, feat_real.detach())
               + 10 * VGG(fake_b, real_b) + TV(fake_b)     :344-380
  step G, then step D (D's grads from the G loss are discarded: zero_grad first)
  C phase    : G(compressed) forward (updates G's BN running stats) and
               locc = MSE(G(compressed), b) + 10 * VGG(compressed, b)   :392-397

Reference semantics kept by default: optimizer_c is built over
D's parameters (A1) and round() has no gradient (A2), so the C phase changes no
parameter -- its loss is computed and logged, its backward is skipped because it is
provably a no-op (``c_phase_backward=True`` runs it anyway for cost parity).
``train_c=True`` fixes both quirks: a straight-through quantiser and an Adam over C
(``opt_c``, scheduled and checkpointed by train.py like the reference's ``optimizer_c`` /
``net_c_scheduler``, train.py:243-246, :441-443).  Without ``train_c`` no ``opt_c`` exists: the
reference's optimizer_c steps nothing (A1), and a scheduler stepping an optimizer that never
steps only produced PyTorch's order warning on every epoch.

D's gradients from the G loss are discarded by the reference (``optimizer_d.zero_grad()``
before ``loss_d.backward()``, train.py:384-389), so the third D forward (the one the G loss
sees) runs with D frozen: the G backward computes only D's input gradients, and no D
gradient -- hence no D all-reduce under data parallelism -- exists for that backward.
Discarded backwards that still reach a reduced network (the C-phase backward into G) run
under ``reducer.paused()``.

All three D passes go through the fused ops (virtual concat of (a, b) on the native
path; spectral-norm 1/sigma on the weight image).  Losses stay on the device.
"""
from __future__ import annotations

import contextlib
import os

import torch

from .. import _native, ops
from ..models.losses import GANLoss, calc_tv_Loss
from ..models.vgg import VGGLoss
from ..utils.tracing import trace_range
from .optim import guarded_step, make_adam


class _STEQuantize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bits):
        return ops.quantize(x, bits)

    @staticmethod
    def backward(ctx, g):
        return g, None


def set_requires_grad(params, flag):
    for p in params:
        p.requires_grad_(flag)


class CompressGANStep:
    def __init__(self, net_g, net_d, net_c, lr=2e-4, beta1=0.5, bits=3, lambda_feat=10.0,
                 lambda_vgg=10.0, lambda_tv=1.0, n_layers_d=3, num_d=3, image_pool=None,
                 train_c=False, c_phase_backward=False, vgg=None, reducer_g=None,
                 reducer_d=None, reducer_c=None, nan_guard=True):
        self.net_g, self.net_d, self.net_c = net_g, net_d, net_c
        self.criterionGAN = GANLoss()                      # LSGAN, reference default
        self.criterionVGG = vgg if vgg is not None else VGGLoss()
        dev = next(net_g.parameters()).device
        self.criterionVGG.to(dev)
        self.bits = bits
        self.lambda_feat, self.lambda_vgg, self.lambda_tv = lambda_feat, lambda_vgg, lambda_tv
        self.feat_weights = 4.0 / (n_layers_d + 1)
        self.d_weights = 1.0 / num_d
        self.opt_g = make_adam(net_g.parameters(), lr=lr, betas=(beta1, 0.999))
        self.opt_d = make_adam(net_d.parameters(), lr=lr, betas=(beta1, 0.999))
        # D's trainable parameters (SN's weight_u / weight_v are Parameters that never train)
        self._d_trainable = [p for p in net_d.parameters() if p.requires_grad]
        # the D phase runs D's fake and real passes separately (train.py:308-316) and G's one
        # PReLU slope serves five sites: their second and later gradients of a backward are
        # summed in place by the kernels (ops/hip.py _pair_first), not by autograd adds
        for p in self._d_trainable:
            p._p2p_pair = True
        pw = getattr(getattr(net_g, "relu", None), "weight", None)
        if isinstance(pw, torch.Tensor):
            pw._p2p_pair = True
        self.train_c = train_c
        self.opt_c = make_adam(net_c.parameters(), lr=lr, betas=(beta1, 0.999)) if train_c else None
        self.c_phase_backward = c_phase_backward
        if hasattr(net_d, "set_feature_grad_gate"):
            net_d.set_feature_grad_gate(True)   # the feature-matching L1 below applies lrelu
        self.image_pool = image_pool
        self.reducer_g, self.reducer_d, self.reducer_c = reducer_g, reducer_d, reducer_c
        self.nan_guard = nan_guard
        self.skipped = torch.zeros((), device=dev) if nan_guard else None
        self.timer = None     # optional utils.PhaseTimer: per-phase HIP-event ms

    def optimizers(self):
        return [o for o in (self.opt_g, self.opt_d, self.opt_c) if o is not None]

    def state_tensors(self):
        """Tensors one step mutates (CapturedStep snapshots them around its warmup)."""
        from .graph import trainer_state_tensors
        extra = [self.skipped] if self.skipped is not None else []
        return trainer_state_tensors([self.net_g, self.net_d, self.net_c], self.optimizers(),
                                     extra)

    def _phase(self, name):
        return self.timer.phase(name) if self.timer is not None else trace_range(name)

    def _opt_step(self, opt, reducer, *losses):
        if not self.nan_guard:
            opt.step()
        else:
            self.skipped = guarded_step(opt, reducer, self.skipped, *losses)

    def _d_in(self, a, b):
        if a.is_cuda and _native.get_backend() == "native":
            return (a, b)
        return torch.cat((a, b), 1)

    def _quant(self, x):
        if self.train_c:
            return _STEQuantize.apply(x, self.bits)
        # the same pass writes G's pixel-unshuffled head input (ExpandNetwork.forward)
        return ops.quantize(x, self.bits, unshuffle=2)

    @staticmethod
    def _no_deferred(x):
        if x.is_cuda and _native.get_backend() == "native":
            from ..ops import hip
            hip.assert_no_deferred()

    def _vgg(self, x, y, fy):
        return self.criterionVGG(x, y) if fy is None else self.criterionVGG(x, y, fy=fy)

    @staticmethod
    def _wgrad_overlap(x, reducer):
        """G's conv weight gradients on the side stream (ops/hip.py ``wgrad_overlap``): grads
        were just set to None and G runs once in this backward; with a DP reducer the conv
        weight gradients are written straight into its buckets (parallel/ddp.py direct
        gradients), everything else stays on the compute stream."""
        if x.is_cuda and _native.get_backend() == "native":
            from ..ops import hip
            return hip.wgrad_overlap(x.device)
        return contextlib.nullcontext()

    def _seed_grad(self, loss):
        """d(loss)/d(loss) = 1 as a persistent tensor (no fill kernel per backward)."""
        seeds = self.__dict__.setdefault("_seeds", {})
        key = (loss.device, loss.dtype, tuple(loss.shape))
        s = seeds.get(key)
        if s is None:
            s = seeds[key] = torch.ones(loss.shape, device=loss.device, dtype=loss.dtype)
        return s

    def _zero(self, opt, reducer):
        if reducer is not None:
            reducer.zero_grad()
        else:
            opt.zero_grad(set_to_none=True)

    def step(self, real_a, real_b):
        G, D, C = self.net_g, self.net_d, self.net_c
        if real_a.is_cuda and _native.get_backend() == "native":
            from ..ops import hip
            hip.begin_step()
            hip.prepare_weights(G, D, C)
        compressed = self._quant(C(real_b))
        fake_b = G(compressed.detach())
        # ---- D losses (reference computes all losses before any update)
        set_requires_grad(self._d_trainable, True)
        fake_in = self._d_in(real_a, fake_b.detach())
        if self.image_pool is not None and self.image_pool.pool_size > 0:
            fake_in = self.image_pool.query(torch.cat((real_a, fake_b.detach()), 1))
        pred_fake = D(fake_in)
        loss_d_fake = self.criterionGAN(pred_fake, False)
        pred_real = D(self._d_in(real_a, real_b.detach()))
        loss_d_real = self.criterionGAN(pred_real, True)
        if real_a.is_cuda and _native.get_backend() == "native":
            loss_d = ops.lincomb_n([loss_d_fake, loss_d_real], [0.5, 0.5])
        else:
            loss_d = (loss_d_fake + loss_d_real) * 0.5
        # ---- G losses: D frozen (its G-loss gradients are discarded by the reference)
        set_requires_grad(self._d_trainable, False)
        # fake_b feeds D, VGG and TV: one fan-out node sums their gradients with HIP adds
        fake_d, fake_v, fake_t = ops.fan_out(fake_b, 3)
        pred_fake_g = D(self._d_in(real_a, fake_d))
        # back on before any backward: autograd's AccumulateGrad skips a leaf that no longer
        # requires grad, which would silently drop the D-loss gradients
        set_requires_grad(self._d_trainable, True)
        loss_g_gan = self.criterionGAN(pred_fake_g, True)
        fgate = getattr(D, "feature_grad_gate", None)   # D's lrelu' rides in these gradients
        # native: the loss compositions are one HIP launch each way (ops.lincomb_n); the torch
        # path keeps the reference's expression order (bitwise parity on CPU)
        native = real_a.is_cuda and _native.get_backend() == "native"
        # each feature's L1 gradient is parked for the next D conv (skip_grad="take"), which
        # adds it in its dgrad epilogue: no accumulate of the feature's two gradients
        defer = native and fgate is not None and os.environ.get("P2P_FEAT_DEFER", "1") != "0"
        feat = [ops.l1(pred_fake_g[i][j], pred_real[i][j].detach(), gate_a=fgate, defer=defer)
                for i in range(len(pred_fake_g)) for j in range(len(pred_fake_g[i]) - 1)]
        if native and feat:
            fw = self.d_weights * self.feat_weights * self.lambda_feat
            loss_feat = ops.lincomb_n(feat, [fw] * len(feat))
        else:
            loss_feat = 0.0
            for f in feat:
                loss_feat = loss_feat + self.d_weights * self.feat_weights * f * self.lambda_feat
        # VGG(real_b): once per step for both perceptual losses against it (G and C phase)
        fy_real = (self.criterionVGG.target_features(real_b)
                   if hasattr(self.criterionVGG, "target_features")
                   and os.environ.get("P2P_VGG_REUSE", "1") != "0" else None)
        vgg_g = self._vgg(fake_v, real_b, fy_real)
        tv = calc_tv_Loss(fake_t)
        if native:
            terms = [loss_g_gan] + ([loss_feat] if feat else []) + [vgg_g, tv]
            loss_g = ops.lincomb_n(terms, [1.0] + ([1.0] if feat else []) + [self.lambda_vgg,
                                                                           self.lambda_tv])
            with torch.no_grad():
                content = ops.lincomb_n([vgg_g.detach()], [self.lambda_vgg])
        else:
            content = vgg_g * self.lambda_vgg
            loss_g = loss_g_gan + loss_feat + content + tv * self.lambda_tv
        # ---- updates: G first (its backward also reaches D; those grads are dropped)
        with self._phase("G_bwd_opt"):
            self._zero(self.opt_g, self.reducer_g)
            with self._wgrad_overlap(real_a, self.reducer_g):
                loss_g.backward(self._seed_grad(loss_g))
            self._no_deferred(real_a)   # every parked VGG-tap gradient was consumed
            if self.reducer_g is not None:
                self.reducer_g.finish()
            self._opt_step(self.opt_g, self.reducer_g, loss_g)
        with self._phase("D_bwd_opt"):
            self._zero(self.opt_d, self.reducer_d)
            loss_d.backward(self._seed_grad(loss_d))
            if self.reducer_d is not None:
                self.reducer_d.finish()
            self._opt_step(self.opt_d, self.reducer_d, loss_d)
        # ---- C phase
        need_graph = self.train_c or self.c_phase_backward
        with torch.set_grad_enabled(need_graph):
            fake_ac = G(compressed)     # also advances G's BN running stats, as the reference
            mse_c, vgg_c = ops.mse(fake_ac, real_b), self._vgg(compressed, real_b, fy_real)
            loss_c = (ops.lincomb_n([mse_c, vgg_c], [1.0, self.lambda_vgg]) if native
                      else mse_c + vgg_c * self.lambda_vgg)
        paused_g = (self.reducer_g.paused() if self.reducer_g is not None
                    else contextlib.nullcontext())
        if self.train_c:
            self._zero(self.opt_c, self.reducer_c)
            with paused_g:      # the G grads of this backward are discarded (zeroed next step)
                loss_c.backward(self._seed_grad(loss_c))
            self._no_deferred(real_a)
            if self.reducer_c is not None:
                self.reducer_c.finish()
            self._opt_step(self.opt_c, self.reducer_c, loss_c)
        elif self.c_phase_backward:
            if self.reducer_g is None and os.environ.get("P2P_CPHASE_ASSIGN", "1") != "0":
                # G's grads are dead from here (zeroed before the next G backward): let this
                # backward assign them instead of adding onto the G-phase values (one aten
                # add per G parameter saved; the backward's own work is unchanged)
                self.opt_g.zero_grad(set_to_none=True)
            with paused_g:      # reference: grads land on G (zeroed next step) -- no effect
                loss_c.backward(self._seed_grad(loss_c))
            self._no_deferred(real_a)
        return {"D": loss_d.detach(), "G_GAN": loss_g_gan.detach(),
                "C": loss_c.detach(), "G_GAN_Feat": torch.as_tensor(loss_feat).detach(),
                "VGG": content.detach(), "TV": tv.detach(), "G": loss_g.detach()}
