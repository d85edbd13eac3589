"""Synthetic paired images (there is no dataset or network access on the benchmark boxes).

``SyntheticPairs`` produces [-1, 1] image pairs of the benchmark shape directly on the
device: a smooth random "photo" (sum of random low-frequency sinusoids, so convolutions
see realistic spatial correlation rather than white noise) and its 3-bit quantised copy
(the reference's paired-data recipe, generate_dataset.py:87-106).
"""
from __future__ import annotations

import math

import torch

from .generate import compress


class SyntheticPairs:
    def __init__(self, batch_size, size=256, device="cpu", seed=0, dtype=torch.float32,
                 bits=3, direction="b2a", n_batches=8):
        self.batch_size, self.size = batch_size, size
        self.device, self.dtype = torch.device(device), dtype
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.batches = [self._make(g, bits, direction) for _ in range(max(1, n_batches))]
        self.i = 0

    def _make(self, g, bits, direction):
        B, S = self.batch_size, self.size
        yy = torch.linspace(0, 1, S).view(1, 1, S, 1)
        xx = torch.linspace(0, 1, S).view(1, 1, 1, S)
        img = torch.zeros(B, 3, S, S)
        for _ in range(6):
            fy = torch.rand(B, 3, 1, 1, generator=g) * 12
            fx = torch.rand(B, 3, 1, 1, generator=g) * 12
            ph = torch.rand(B, 3, 1, 1, generator=g) * 2 * math.pi
            amp = torch.rand(B, 3, 1, 1, generator=g)
            img += amp * torch.sin(2 * math.pi * (fy * yy + fx * xx) + ph)
        img = (img - img.amin((2, 3), keepdim=True)) / (
            img.amax((2, 3), keepdim=True) - img.amin((2, 3), keepdim=True) + 1e-6)
        a = img                                   # original, [0, 1]
        b = compress(img, bits)                   # 3-bit quantised, [0, 1]
        a, b = a * 2 - 1, b * 2 - 1
        if direction != "a2b":
            a, b = b, a
        cl = torch.channels_last
        return (a.to(self.device, self.dtype).contiguous(memory_format=cl),
                b.to(self.device, self.dtype).contiguous(memory_format=cl))

    def next_batch(self):
        out = self.batches[self.i % len(self.batches)]
        self.i += 1
        return out

    def __iter__(self):
        while True:
            yield self.next_batch()
