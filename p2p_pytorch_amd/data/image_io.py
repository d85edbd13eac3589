"""Image file helpers (reference utils.py:5-21, generate_dataset.py:45-53, train.py:33-49).

PIL is the only decoder available here (no torchvision): ``to_tensor`` / ``normalize`` are
the ToTensor / Normalize(0.5, 0.5) pair the reference builds with torchvision.transforms.
"""
from __future__ import annotations

import numpy as np
import torch
from PIL import Image

IMG_EXTENSIONS = (".png", ".PNG", ".jpg", ".jpeg")


def is_image_file(filename: str) -> bool:
    return filename.endswith(IMG_EXTENSIONS)


def load_img(filepath: str, size: int | None = 256) -> Image.Image:
    """RGB + bicubic resize to ``size`` x ``size`` (utils.py:9-12); ``size=None`` keeps it."""
    img = Image.open(filepath).convert("RGB")
    if size:
        img = img.resize((size, size), Image.BICUBIC)
    return img


def to_tensor(img) -> torch.Tensor:
    """PIL / HWC uint8 array -> CHW float in [0, 1] (torchvision ToTensor)."""
    arr = np.asarray(img, dtype=np.uint8)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    return torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1))).float().div_(255.0)


def normalize(t: torch.Tensor) -> torch.Tensor:
    """Normalize((0.5,)*3, (0.5,)*3): [0, 1] -> [-1, 1]."""
    return t.mul(2.0).sub_(1.0)


def save_img(image_tensor: torch.Tensor, filename: str) -> None:
    """CHW tensor in [-1, 1] -> uint8 image file (utils.py:15-21)."""
    image_numpy = image_tensor.detach().float().cpu().numpy()
    image_numpy = (np.transpose(image_numpy, (1, 2, 0)) + 1) / 2.0 * 255.0
    image_numpy = image_numpy.clip(0, 255).astype(np.uint8)
    Image.fromarray(image_numpy).save(filename)


def tensor2np(tensor: torch.Tensor) -> np.ndarray:
    """Reference ``tensor2np`` (train.py:43-49): assumes [0, 1] data -- on the [-1, 1]
    tensors the trainer passes, the negative half clips to 0 (quirk A11, reproduced)."""
    t = tensor.detach().float().cpu().numpy()
    t = np.squeeze(t)
    t = np.moveaxis(t, 0, 2)
    return (t * 255).clip(0, 255).astype(np.uint8)


def tensor2img(tensor: torch.Tensor) -> Image.Image:
    return Image.fromarray(tensor2np(tensor))
