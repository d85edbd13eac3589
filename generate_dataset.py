#!/usr/bin/env python
"""Paired-dataset generator, flag-compatible with the reference generate_dataset.py
(:150-165).  ``compress`` is importable like the reference's (train.py:4 imports it)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from p2p_pytorch_amd.data.generate import compress, crop, generate_patches, main  # noqa: E402,F401


def cli(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--target_dataset_folder", type=str, help="target folder where image saved")
    p.add_argument("--dataset_path", type=str, help="source image folder")
    p.add_argument("--bit_size", type=int, default=3, help="quantisation bits of the b/ images")
    p.add_argument("--max_patches", type=int, default=None, help="max tiles per source image")
    p.add_argument("--pool_size", type=int, default=1, help="worker processes")
    p.add_argument("--crop_size", type=int, default=-1, help="crop size, -1 to save whole images")
    p.add_argument("--img_format", type=str, default="png", help="image format e.g. png")
    p.add_argument("--upsampling", type=int, default=0, help="nearest upsampling factor")
    a = p.parse_args(argv)
    crop_size = [a.crop_size, a.crop_size] if a.crop_size and a.crop_size > 0 else None
    return main(a.target_dataset_folder, a.dataset_path, a.bit_size, a.pool_size, crop_size,
                a.img_format, a.upsampling, a.max_patches)


if __name__ == "__main__":
    cli()
