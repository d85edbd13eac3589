"""Reference-compatible ``data`` module (/root/reference/data.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from p2p_pytorch_amd.data import get_test_set, get_training_set  # noqa: E402,F401
