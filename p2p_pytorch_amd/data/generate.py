"""Offline paired-dataset generator (reference generate_dataset.py:21-148).

For every source image: optional nearest upsampling, non-overlapping ``crop_size`` tiles
(at most ``max_patches``), the original tile -> ``a/`` and its ``bit_size``-bit quantised
copy -> ``b/``.  Differences from the reference, each a documented quirk fix: ``--bit_size``
is honoured (the reference hard-codes 3, quirk A13), file names with several dots keep
their stem (the reference's ``split('.')`` raises), and ``--pool_size`` > 1 really runs a
process pool (the reference's pool is commented out).
"""
from __future__ import annotations

import os
from multiprocessing import Pool

import numpy as np
import torch
from PIL import Image

from .image_io import is_image_file


def compress(tensor: torch.Tensor, bit: int) -> torch.Tensor:
    """round(clamp(x, 0, 1) * (2^b - 1)) / (2^b - 1)  (generate_dataset.py:29-34)."""
    max_val = 2 ** bit - 1
    return torch.round(torch.clamp(tensor, 0.0, 1.0) * max_val) / max_val


def crop(img_arr: np.ndarray, block_size) -> np.ndarray:
    """Non-overlapping tiles, row-major (generate_dataset.py:39-43)."""
    h_b, w_b = block_size
    rows = np.vsplit(img_arr, img_arr.shape[0] // h_b)
    return np.concatenate([np.hsplit(r, img_arr.shape[1] // w_b) for r in rows], 0)


def quantize_uint8(tile: np.ndarray, bit: int) -> np.ndarray:
    t = torch.from_numpy(tile.astype(np.float32) / 255.0)
    q = compress(t, bit).numpy()
    return (q * 255).clip(0, 255).astype(np.uint8)


def generate_patches(src_path, files, set_path, crop_size, img_format, upsampling, max_patches,
                     bit_size=3):
    img = Image.open(os.path.join(src_path, files)).convert("RGB")
    if upsampling and upsampling > 0:
        k = abs(upsampling)
        img = img.resize((img.width * k, img.height * k), Image.NEAREST)
    name = os.path.splitext(files)[0]
    dir_a = os.path.join(set_path, "a")
    dir_b = os.path.join(set_path, "b")
    os.makedirs(dir_a, exist_ok=True)
    os.makedirs(dir_b, exist_ok=True)
    arr = np.array(img)
    h, w = arr.shape[:2]
    if crop_size is None:
        patches = arr[None]
    else:
        arr = arr[:h - h % crop_size[0], :w - w % crop_size[1]]
        patches = crop(arr, crop_size)
    n = min(len(patches), max_patches) if max_patches else len(patches)
    for i in range(n):
        Image.fromarray(patches[i]).save(os.path.join(dir_a, f"{name}_{i}.{img_format}"))
        Image.fromarray(quantize_uint8(patches[i], bit_size)).save(
            os.path.join(dir_b, f"{name}_{i}.{img_format}"))
    return n


def _job(args):
    return generate_patches(*args)


def main(target_dataset_folder, dataset_path, bit_size=3, pool_size=1, crop_size=None,
         img_format="png", upsampling=0, max_patches=None, verbose=True):
    if verbose:
        print("[ Creating Dataset ]")
        print(f"Crop Size : {crop_size}\nTarget       : {target_dataset_folder}\n"
              f"Dataset       : {dataset_path}\nBit       : {bit_size}\nPool       : {pool_size}\n"
              f"Format    : {img_format}")
    if not os.path.exists(dataset_path):
        raise RuntimeError("Source folder not found, please put your dataset there")
    os.makedirs(target_dataset_folder, exist_ok=True)
    files = sorted(f for f in os.listdir(dataset_path) if is_image_file(f))
    jobs = [(dataset_path, f, target_dataset_folder, crop_size, img_format, upsampling, max_patches,
             bit_size) for f in files]
    if pool_size and pool_size > 1:
        with Pool(pool_size) as pool:
            counts = pool.map(_job, jobs)
    else:
        counts = [_job(j) for j in jobs]
    if verbose:
        print("Dataset Created")
    return sum(counts)
