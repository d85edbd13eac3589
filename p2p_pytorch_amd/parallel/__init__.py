from . import dist
from .ddp import GradReducer

__all__ = ["dist", "GradReducer"]
