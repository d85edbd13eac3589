# reproduce one fuzz case and locate the bad elements of dX
import sys, zlib, torch
sys.path.insert(0, ".")
from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import reference as ref
_native.set_backend("native")
DEV = "cuda"
def bf(x): return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
def run(case):
    N, C1, C2, H, Cout, k, s, p, reflect, up, act_in, act_out = case
    g = torch.Generator(device=DEV).manual_seed(zlib.crc32(repr(case).encode()))
    x1 = bf(torch.randn(N, C1, H, H, device=DEV, generator=g))
    w = torch.randn(Cout, C1, k, k, device=DEV, generator=g) * (1.0 / (C1 * k * k) ** 0.5)
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    hx = x1.clone().requires_grad_(True); hw = w.clone().requires_grad_(True); hb = b.clone().requires_grad_(True)
    y = ops.conv2d(hx, hw, hb, s, p, act_out=act_out)
    gy = bf(torch.randn(*y.shape, device=DEV, generator=g))
    y.backward(gy)
    rx = x1.float().requires_grad_(True); rw = w.clone().requires_grad_(True)
    ry = ref.conv2d(rx, rw.to(torch.bfloat16).float(), b, s, p, act_out=act_out)
    ry.backward(gy.float())
    d = (hx.grad.float() - rx.grad).abs()
    print(case, "fwd", ((y.float()-ry).abs().max()/ry.abs().max()).item(), "dx", (d.max()/rx.grad.abs().max()).item())
    bad = (d > 0.02 * rx.grad.abs().max()).nonzero()
    print(" bad", bad.shape[0], "of", d.numel(), bad[:10].tolist())
    # gate check: y sign vs ry sign
    ys, rs = (y.float() > 0), (ry > 0)
    print(" sign mismatches y vs ref:", (ys != rs).sum().item())
for case in [(2, 128, 0, 9, 16, 1, 1, 0, False, 1, None, 'lrelu'), (2, 128, 0, 9, 16, 1, 1, 0, False, 1, None, None),
             (2, 128, 0, 9, 24, 1, 1, 0, False, 1, None, 'lrelu'), (2, 64, 0, 9, 16, 1, 1, 0, False, 1, None, 'lrelu'),
             (2, 128, 0, 9, 16, 3, 1, 1, False, 1, None, 'lrelu')]:
    run(case)
