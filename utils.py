"""Reference-compatible ``utils`` module (/root/reference/utils.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from p2p_pytorch_amd.data import is_image_file, load_img, save_img  # noqa: E402,F401
