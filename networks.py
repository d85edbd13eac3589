"""Reference-compatible ``networks`` module (/root/reference/networks.py).

Every public name of the reference resolves here, backed by the MI355X model zoo in
``p2p_pytorch_amd.models`` (same constructor signatures, parameter names, state_dict keys
and shapes).  Import-compatible: ``from networks import define_G, GANLoss, ...``.

``NLayerDiscriminator`` is the reference's spectral-norm PatchGAN (networks.py:758-806,
signature ``(input_nc, ndf, n_layers, norm_layer, use_sigmoid, getIntermFeat)``); the
pix2pix-family PatchGAN (instance norm, padding 1) is ``PatchGANDiscriminator``.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from p2p_pytorch_amd.models import (  # noqa: E402,F401
    BatchNorm2d, CompressionNetwork, ConvLayer, ExpandNetwork, GANLoss, ImagePool,
    MultiscaleDiscriminator, NLayerDiscriminatorSN, PatchGANDiscriminator, PixelDiscriminator,
    PixelUnshuffle, PReLU, ResidualBlock, SpectralNorm, UnetGenerator, UpsampleConvLayer,
    VGGLoss, Vgg19, angular_loss, calc_tv_Loss, count_params, define_C, define_D, define_G,
    get_scheduler, init_net, init_weights, l2normalize, pixel_unshuffle, sobelLayer,
    update_learning_rate)

NLayerDiscriminator = NLayerDiscriminatorSN
