from .optim import FusedAdam, make_adam
from .pix2pix import Pix2PixStep, set_requires_grad

__all__ = ["FusedAdam", "make_adam", "Pix2PixStep", "set_requires_grad"]
