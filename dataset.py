"""Reference-compatible ``dataset`` module (/root/reference/dataset.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from p2p_pytorch_amd.data import DatasetFromFolder  # noqa: E402,F401
