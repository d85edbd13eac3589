#!/usr/bin/env python
"""Phase timeline of the 32x32x16 conv tiles from the diagnostic stamp build.

    python tools/build_ext.py --define P2P_M32_STAMPS --out p2p_pytorch_amd/_C/m32_stamps.so
    P2P_LIB=p2p_pytorch_amd/_C/m32_stamps.so python tools/m32_stamps.py --layers c4,c3 [--op fwd]

Per block (csrc/conv_fwd_m32.hip M32_STAMP): s_memtime at start / after the prologue (first
tile landed + first fragments issued) / after the K loop / after the epilogue, and
s_memrealtime (100 MHz) at start and end.  Prints per layer the median shader-clock cycles of
prologue, K loop and epilogue, their share of a block's life, the in-kernel clock, and how
much of the kernel's wall time the blocks cover.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYERS = {   # name: (kind, C1, C2, H, Cout, k, s, p, act_in)
    "e2": ("conv", 64, 0, 128, 128, 4, 2, 1, None),
    "e3": ("conv", 128, 0, 64, 256, 4, 2, 1, None),
    "e4": ("conv", 256, 0, 32, 512, 4, 2, 1, None),
    "c2": ("conv", 64, 0, 128, 128, 4, 2, 1, None),
    "c3": ("conv", 128, 0, 64, 256, 4, 2, 1, None),
    "c4": ("conv", 256, 0, 32, 512, 4, 1, 1, None),
    "d3": ("convT", 256, 256, 32, 128, 4, 2, 1, None),
    "d4": ("convT", 512, 512, 16, 256, 4, 2, 1, None),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--layers", default="c4,c3,e3,d4")
    a = ap.parse_args()
    from p2p_pytorch_amd import _native, ops
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    lib = ctypes.CDLL(_native.LIB_PATH)
    assert hasattr(lib, "p2p_m32_stamps"), "not a P2P_M32_STAMPS build"
    dev = torch.device("cuda")
    B = a.batch
    for name in a.layers.split(","):
        kind, c1, c2, H, cout, k, s, p, act = LAYERS[name]
        x1 = torch.randn(B, c1, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x2 = (torch.randn(B, c2, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
              if c2 else None)
        xin = (x1, x2) if x2 is not None else x1
        cin = c1 + c2
        if kind == "conv":
            w = torch.randn(cout, cin, k, k, device=dev) * 0.02
            fn = lambda: ops.conv2d(xin, w, None, s, p, act_in=act)   # noqa: E731
        else:
            w = torch.randn(cin, cout, k, k, device=dev) * 0.02
            fn = lambda: ops.conv_transpose2d(xin, w, None, s, p, act)   # noqa: E731
        with torch.no_grad():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            fn()
            torch.cuda.synchronize()
        buf = np.zeros(65536 * 6, dtype=np.uint64)
        rc = lib.p2p_m32_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int(65536))
        assert rc == 0, rc
        st = buf.reshape(-1, 6).astype(np.float64)
        st = st[st[:, 3] > 0]
        pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
        life = st[:, 3] - st[:, 0]
        rt = (st[:, 5] - st[:, 4])
        clk = np.median((life / np.maximum(rt, 1)) * 100e6 / 1e9)
        wall_us = (st[:, 5].max() - st[:, 4].min()) / 100.0
        busy_us = rt.sum() / 100.0
        print(f"{name} {kind}: {len(st)} blocks  kernel wall {wall_us:.1f} us  clock {clk:.2f} GHz  "
              f"block life median {np.median(life):.0f} cyc ({np.median(rt) / 100:.1f} us)")
        print(f"   prologue {np.median(pro):8.0f} cyc ({np.median(pro / life) * 100:4.1f} %)  "
              f"K loop {np.median(loop):8.0f} ({np.median(loop / life) * 100:4.1f} %)  "
              f"epilogue {np.median(epi):8.0f} ({np.median(epi / life) * 100:4.1f} %)   "
              f"sum of block lives / (256 CUs x wall) = {busy_us / (256 * wall_us) * 100:.1f} %")
        print(f"   K loop p10/p90 {np.percentile(loop, 10):.0f} / {np.percentile(loop, 90):.0f}  "
              f"epilogue p10/p90 {np.percentile(epi, 10):.0f} / {np.percentile(epi, 90):.0f}")


if __name__ == "__main__":
    main()
