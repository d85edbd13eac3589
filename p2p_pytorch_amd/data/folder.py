"""Paired image folders: ``<root>/{train,test}/{a,b}/<same filename>``.

``DatasetFromFolder`` is the reference dataset (dataset.py:12-54, data.py:6-15): PIL RGB ->
[-1, 1] CHW float, no resize / crop / flip, ``a2b`` returns (a, b), ``b2a`` (the default)
returns (b, a).

``DevicePairCache`` is the MI355X path: the whole paired set is decoded ONCE into two
uint8 NHWC tensors that live in HBM (288 GB per GPU holds ~1.4 M 256x256 pairs), and a
training batch is a device-side gather + uint8->bf16 normalise -- no DataLoader worker
processes, no per-step host->device copies (the reference's only concurrency was
DataLoader workers, train.py:174-175).  Each rank of a data-parallel job draws its own
disjoint slice of a shared per-epoch permutation.
"""
from __future__ import annotations

import os
from os.path import join

import numpy as np
import torch
import torch.utils.data as data
from PIL import Image

from .image_io import is_image_file, normalize, to_tensor


class DatasetFromFolder(data.Dataset):
    def __init__(self, image_dir, direction="b2a"):
        super().__init__()
        self.direction = direction
        self.a_path = join(image_dir, "a")
        self.b_path = join(image_dir, "b")
        self.image_filenames = sorted(x for x in os.listdir(self.a_path) if is_image_file(x))

    def __getitem__(self, index):
        name = self.image_filenames[index]
        a = normalize(to_tensor(Image.open(join(self.a_path, name)).convert("RGB")))
        b = normalize(to_tensor(Image.open(join(self.b_path, name)).convert("RGB")))
        return (a, b) if self.direction == "a2b" else (b, a)

    def __len__(self):
        return len(self.image_filenames)


def get_training_set(root_dir, direction="b2a"):
    return DatasetFromFolder(join(root_dir, "train"), direction)


def get_test_set(root_dir, direction="b2a"):
    return DatasetFromFolder(join(root_dir, "test"), direction)


class DevicePairCache:
    """All pairs of a folder split as uint8 [N, H, W, 3] on ``device``; images must share
    one size (the generator's crops do)."""

    def __init__(self, dataset: DatasetFromFolder, device, rank: int = 0, world: int = 1,
                 seed: int = 123):
        a_list, b_list = [], []
        for name in dataset.image_filenames:
            a_list.append(np.asarray(Image.open(join(dataset.a_path, name)).convert("RGB")))
            b_list.append(np.asarray(Image.open(join(dataset.b_path, name)).convert("RGB")))
        if not a_list:
            raise ValueError(f"no images in {dataset.a_path}")
        shapes = {x.shape for x in a_list + b_list}
        if len(shapes) != 1:
            raise ValueError(f"DevicePairCache needs equally sized images, got {sorted(shapes)[:4]}")
        a = torch.from_numpy(np.stack(a_list))
        b = torch.from_numpy(np.stack(b_list))
        if dataset.direction != "a2b":
            a, b = b, a
        self.a = a.to(device)
        self.b = b.to(device)
        self.n = self.a.shape[0]
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        self._perm = None
        self._pos = 0

    def __len__(self):
        return self.n

    def batches_per_epoch(self, batch_size: int) -> int:
        return self.n // (batch_size * self.world)

    @staticmethod
    def _to_model(x_u8: torch.Tensor, dtype) -> torch.Tensor:
        # uint8 NHWC -> [-1, 1] NCHW-shaped, channels_last memory (no layout copy)
        return x_u8.permute(0, 3, 1, 2).to(dtype).mul_(2.0 / 255.0).sub_(1.0).contiguous(
            memory_format=torch.channels_last)

    def new_epoch(self):
        self._perm = torch.randperm(self.n, generator=self.gen).to(self.device)
        self._pos = 0

    def next_batch(self, batch_size: int, dtype=torch.bfloat16):
        """Next (input, target) batch of this rank; None at the end of the epoch."""
        if self._perm is None:
            self.new_epoch()
        span = batch_size * self.world
        if self._pos + span > self.n:
            return None
        idx = self._perm[self._pos + self.rank * batch_size:self._pos + (self.rank + 1) * batch_size]
        self._pos += span
        return self._to_model(self.a.index_select(0, idx), dtype), self._to_model(
            self.b.index_select(0, idx), dtype)
