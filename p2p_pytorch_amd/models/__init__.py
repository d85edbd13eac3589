from .compress_gan import (CompressionNetwork, ConvLayer, ExpandNetwork, MultiscaleDiscriminator,
                           NLayerDiscriminatorSN, PixelUnshuffle, PReLU, ResidualBlock, SpectralNorm,
                           UpsampleConvLayer, l2normalize, pixel_unshuffle)
from .factory import (ImagePool, count_params, define_C, define_D, define_G, get_scheduler,
                      init_net, init_weights, update_learning_rate)
from .layers import BatchNorm2d, Conv2d, ConvTranspose2d, InstanceNorm2d
from .losses import GANLoss, angular_loss, calc_tv_Loss, sobelLayer
from .pix2pix import NLayerDiscriminator, PixelDiscriminator, UnetGenerator
from .pix2pix import NLayerDiscriminator as PatchGANDiscriminator
from .vgg import VGGLoss, Vgg19

__all__ = [n for n in dir() if not n.startswith("_")]
