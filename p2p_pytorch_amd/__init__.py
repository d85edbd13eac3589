"""p2p_pytorch_amd -- an MI355X-native (gfx950 / CDNA4) pix2pix-style conditional
image-to-image GAN framework: hand-written HIP MFMA kernels for the conv / norm / loss /
optimizer hot path, RCCL-over-xGMI data parallelism, and reference-compatible
``train.py`` / ``test.py`` / ``networks.py`` entrypoints.
"""
from . import _native
from ._native import get_backend, is_deterministic, set_backend, set_deterministic
from .ops.fp8 import get_precision, set_precision

__version__ = "0.1.0"

__all__ = ["_native", "get_backend", "set_backend", "set_deterministic", "is_deterministic",
           "get_precision", "set_precision", "__version__"]
