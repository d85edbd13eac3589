"""Factories, init, schedulers and the image history pool
(reference networks.py:64-171 and :708-714).

``define_G`` / ``define_D`` / ``define_C`` keep the reference signatures; extra keyword
arguments select the pix2pix family (``netG='unet_256'``, ``netD='basic'|'pixel'``).
"""
from __future__ import annotations

import random

import torch
import torch.nn as nn
from torch.nn import init
from torch.optim import lr_scheduler

from .compress_gan import CompressionNetwork, ExpandNetwork, MultiscaleDiscriminator
from .pix2pix import NLayerDiscriminator, PixelDiscriminator, UnetGenerator


class ImagePool:
    """History buffer of generated images (networks.py:64-91).  ``pool_size == 0`` is an
    identity passthrough (how the reference uses it, train.py:248)."""

    def __init__(self, pool_size, rng: random.Random | None = None):
        self.pool_size = pool_size
        self.rng = rng or random.Random()
        self.num_imgs = 0
        self.images = []

    def query(self, images):
        if self.pool_size == 0:
            return images
        out = []
        for image in images.detach():
            image = image.unsqueeze(0)
            if self.num_imgs < self.pool_size:
                self.num_imgs += 1
                self.images.append(image)
                out.append(image)
            elif self.rng.uniform(0, 1) > 0.5:
                k = self.rng.randint(0, self.pool_size - 1)
                out.append(self.images[k].clone())
                self.images[k] = image
            else:
                out.append(image)
        return torch.cat(out, 0)


def get_scheduler(optimizer, opt):
    """lambda | step | plateau | cosine, stepped once per epoch (networks.py:104-118).
    Unknown policies raise (the reference *returns* the exception, quirk A12)."""
    if opt.lr_policy == "lambda":
        def lambda_rule(epoch):
            return 1.0 - max(0, epoch + opt.epoch_count - opt.niter) / float(opt.niter_decay + 1)
        return lr_scheduler.LambdaLR(optimizer, lr_lambda=lambda_rule)
    if opt.lr_policy == "step":
        return lr_scheduler.StepLR(optimizer, step_size=opt.lr_decay_iters, gamma=0.1)
    if opt.lr_policy == "plateau":
        return lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=0.2, threshold=0.01,
                                              patience=5)
    if opt.lr_policy == "cosine":
        return lr_scheduler.CosineAnnealingLR(optimizer, T_max=opt.niter, eta_min=0)
    raise NotImplementedError(f"learning rate policy [{opt.lr_policy}] is not implemented")


def update_learning_rate(scheduler, optimizer, metric=None, verbose=True):
    if isinstance(scheduler, lr_scheduler.ReduceLROnPlateau):
        scheduler.step(metric if metric is not None else 0.0)
    else:
        scheduler.step()
    lr = optimizer.param_groups[0]["lr"]
    if verbose:
        print("learning rate = %.7f" % lr)
    return lr


def init_weights(net, init_type="normal", gain=0.02, verbose=True):
    """N(0, gain) / xavier / kaiming / orthogonal for Conv*/Linear (bias 0); BatchNorm2d
    weight N(1, gain), bias 0.  Spectral-norm convs have no ``weight`` attribute and keep
    their default init, like the reference (quirk A8)."""

    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, "weight") and m.weight is not None and (
                classname.find("Conv") != -1 or classname.find("Linear") != -1):
            if init_type == "normal":
                init.normal_(m.weight.data, 0.0, gain)
            elif init_type == "xavier":
                init.xavier_normal_(m.weight.data, gain=gain)
            elif init_type == "kaiming":
                init.kaiming_normal_(m.weight.data, a=0, mode="fan_in")
            elif init_type == "orthogonal":
                init.orthogonal_(m.weight.data, gain=gain)
            else:
                raise NotImplementedError(f"initialization method [{init_type}] is not implemented")
            if getattr(m, "bias", None) is not None:
                init.constant_(m.bias.data, 0.0)
        elif classname.find("BatchNorm2d") != -1:
            init.normal_(m.weight.data, 1.0, gain)
            init.constant_(m.bias.data, 0.0)

    if verbose:
        print("initialize network with %s" % init_type)
    net.apply(init_func)


def init_net(net, init_type="normal", init_gain=0.02, gpu_id="cuda:0", verbose=True):
    net.to(gpu_id)
    init_weights(net, init_type, gain=init_gain, verbose=verbose)
    return net


def define_C(init_type="normal", init_gain=0.02, gpu_id="cuda:0", verbose=True):
    return init_net(CompressionNetwork(), init_type, init_gain, gpu_id, verbose)


def define_G(init_type="normal", init_gain=0.02, gpu_id="cuda:0", netG="expand", input_nc=3,
             output_nc=3, ngf=64, norm="instance", use_dropout=True, verbose=True):
    if netG == "expand":
        net = ExpandNetwork()
    elif netG.startswith("unet_"):
        size = int(netG.split("_")[1])
        # unet_256 -> 8 downsamplings, unet_128 -> 7; small N is a level count (unet_4)
        num_downs = size.bit_length() - 1 if size >= 32 else size
        net = UnetGenerator(input_nc, output_nc, num_downs, ngf, norm, use_dropout)
    else:
        raise NotImplementedError(f"Generator model name [{netG}] is not recognized")
    return init_net(net, init_type, init_gain, gpu_id, verbose)


def define_D(input_nc, ndf, norm="batch", use_sigmoid=False, init_type="normal", init_gain=0.02,
             gpu_id="cuda:0", netD="multiscale", n_layers_D=3, num_D=3, verbose=True):
    if netD == "multiscale":
        net = MultiscaleDiscriminator(input_nc, ndf, n_layers=n_layers_D, norm_layer=None,
                                      use_sigmoid=use_sigmoid, num_D=num_D, getIntermFeat=True)
    elif netD == "basic":
        net = NLayerDiscriminator(input_nc, ndf, 3, norm, use_sigmoid)
    elif netD == "n_layers":
        net = NLayerDiscriminator(input_nc, ndf, n_layers_D, norm, use_sigmoid)
    elif netD == "pixel":
        net = PixelDiscriminator(input_nc, ndf, norm, use_sigmoid)
    else:
        raise NotImplementedError(f"Discriminator model name [{netD}] is not recognized")
    return init_net(net, init_type, init_gain, gpu_id, verbose)


def count_params(net: nn.Module, trainable_only=False) -> int:
    return sum(p.numel() for p in net.parameters() if p.requires_grad or not trainable_only)
