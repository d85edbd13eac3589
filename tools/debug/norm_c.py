import sys, torch, torch.nn.functional as F
sys.path.insert(0, ".")
from p2p_pytorch_amd import _native
_native.set_backend("native"); assert _native.load()
P = _native.ops()
DEV = "cuda"
def bf(x): return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for (N, C, H, W) in [(1, 8, 4, 4), (2, 16, 4, 4), (2, 24, 4, 4), (2, 32, 4, 4), (2, 64, 4, 4), (2, 8, 32, 32), (2, 64, 32, 32)]:
    g = torch.Generator(device=DEV).manual_seed(7)
    x = bf(torch.randn(N, C, H, W, device=DEV, generator=g) * 2 + 1)
    gy = bf(torch.randn(N, C, H, W, device=DEV, generator=g))
    y, mean, rstd = P.norm_fwd(x, 1e-5, None, None, None, 0, None, None, 0.1, False, None)
    dx = P.norm_bwd(x, gy, mean, rstd, None, None, 0, None, None, True, False, None)
    xr = x.float().cpu().requires_grad_(True)
    z = F.instance_norm(xr, eps=1e-5); z.backward(gy.float().cpu())
    print((N, C, H, W), "dx err", round((dx.float().cpu() - xr.grad).abs().max().item(), 4), "of", round(xr.grad.abs().max().item(), 3))
