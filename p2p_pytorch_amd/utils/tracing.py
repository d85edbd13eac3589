"""roctx ranges and HIP-event phase timers.

``trace_range("G_fwd")`` pushes a roctx range (visible in ``rocprofv3 --marker-trace``
timelines) around a phase; it is a no-op costing one attribute check when the roctx
library is absent or tracing is disabled (``P2P_ROCTX=0``).  ``PhaseTimer`` brackets
phases with HIP events and reports per-phase milliseconds without synchronising inside
the step (the elapsed times are read once, at ``report()``).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if os.environ.get("P2P_ROCTX", "1") == "0":
        return None
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so"):
        for d in ("", "/opt/rocm/lib/"):
            try:
                lib = ctypes.CDLL(d + name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                return _lib
            except (OSError, AttributeError):
                continue
    return None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Per-phase device time from HIP events; ``enabled=False`` makes every call free."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._open = []
        self._acc = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled or torch.cuda.is_current_stream_capturing():
            with trace_range(name):
                yield
            return
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        with trace_range(name):
            yield
        e1.record()
        self._open.append((name, e0, e1))

    def report(self, reset: bool = True) -> dict:
        """Phase -> summed ms since the last report (synchronises on the last event)."""
        if self._open:
            self._open[-1][2].synchronize()
        for name, e0, e1 in self._open:
            self._acc[name] = self._acc.get(name, 0.0) + e0.elapsed_time(e1)
        out = dict(self._acc)
        if reset:
            self._open.clear()
            self._acc.clear()
        return out
