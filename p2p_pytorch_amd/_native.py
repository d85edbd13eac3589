"""Loader for the in-tree HIP/CDNA4 extension (``p2p_pytorch_amd/_C/libp2p_hip.so``).

The extension registers its kernels as ``torch.ops.p2p.*`` (see ``csrc/bindings.cpp``).
It is built by ``python tools/build_ext.py`` (hipcc --offload-arch=gfx950) and travels
with the repository snapshot to the GPU box, so nothing is JIT-compiled at run time.

Device policy (no silent fallbacks):
  * CPU tensors always run the pure-PyTorch oracle in ``ops/reference.py``.
  * GPU tensors run the HIP kernels.  If the extension is missing on a GPU box the
    first GPU op raises -- unless the caller explicitly selected the stock-PyTorch
    *baseline* backend (``P2P_BACKEND=torch`` / ``set_backend('torch')``), which is
    only used to measure the eager MIOpen/hipBLASLt baseline that BASELINE.md asks for.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C")
# P2P_LIB: an alternative build of the extension (kernel A/B experiments, tools/build_ext.py --out)
LIB_PATH = os.environ.get("P2P_LIB") or os.path.join(_LIB_DIR, "libp2p_hip.so")

_lock = threading.Lock()
_loaded = False
_load_error: str | None = None
_backend = os.environ.get("P2P_BACKEND", "native").lower()
if _backend not in ("native", "torch"):
    raise ValueError(f"P2P_BACKEND must be 'native' or 'torch', got {_backend!r}")


def set_backend(name: str) -> None:
    """Select the GPU backend: 'native' (HIP kernels, default) or 'torch' (eager baseline)."""
    global _backend
    name = name.lower()
    if name not in ("native", "torch"):
        raise ValueError(name)
    _backend = name


def get_backend() -> str:
    return _backend


def set_deterministic(flag: bool = True) -> None:
    """Bitwise-repeatable HIP kernels: the conv split-K reduction switches from fp32 atomics
    to per-split slabs summed in a fixed order (every other reduction in the extension --
    wgrad slabs, norm / loss / column-sum partials -- is already order-fixed)."""
    os.environ["P2P_DETERMINISTIC"] = "1" if flag else "0"


def is_deterministic() -> bool:
    return os.environ.get("P2P_DETERMINISTIC", "0") == "1"


def load() -> bool:
    """Load the extension once; returns True when ``torch.ops.p2p`` is available."""
    global _loaded, _load_error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(LIB_PATH):
            _load_error = f"{LIB_PATH} not built (run: python tools/build_ext.py)"
            return False
        try:
            torch.ops.load_library(LIB_PATH)
        except Exception as e:  # pragma: no cover - depends on the box
            _load_error = f"failed to load {LIB_PATH}: {e}"
            return False
        _loaded = True
        return True


def available() -> bool:
    return load()


def load_error() -> str | None:
    return _load_error


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` must be processed by the HIP kernels.

    Raises if ``t`` lives on the GPU, the native backend is selected, and the
    extension cannot be loaded (fail loudly instead of silently running eager code).
    """
    if not t.is_cuda:
        return False
    if _backend == "torch":
        return False
    if not load():
        raise RuntimeError(
            "p2p_pytorch_amd: GPU tensor but the HIP extension is unavailable: "
            f"{_load_error}. Build it with `python tools/build_ext.py` or select the "
            "eager baseline explicitly with P2P_BACKEND=torch.")
    return True


def ops():
    """Return the ``torch.ops.p2p`` namespace (loads the library)."""
    if not load():
        raise RuntimeError(f"p2p_pytorch_amd HIP extension unavailable: {_load_error}")
    return torch.ops.p2p
