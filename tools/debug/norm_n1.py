import sys, torch, torch.nn.functional as F
sys.path.insert(0, ".")
from p2p_pytorch_amd import _native
_native.set_backend("native"); assert _native.load()
P = _native.ops()
DEV = "cuda"
def bf(x): return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
g = torch.Generator(device=DEV).manual_seed(7)
C, H, W = 8, 4, 4
x1 = bf(torch.randn(1, C, H, W, device=DEV, generator=g) * 2 + 1)
gy1 = bf(torch.randn(1, C, H, W, device=DEV, generator=g))
for N in (1, 2):
    x = bf(x1.float().repeat(N, 1, 1, 1)); gy = bf(gy1.float().repeat(N, 1, 1, 1))
    y, mean, rstd = P.norm_fwd(x, 1e-5, None, None, None, 0, None, None, 0.1, False, None)
    dsum = torch.empty(C, device=DEV)
    dx = P.norm_bwd(x, gy, mean, rstd, None, None, 0, None, None, True, False, dsum)
    torch.cuda.synchronize()
    xr = x1.float().cpu().requires_grad_(True)
    z = F.instance_norm(xr, eps=1e-5); z.backward(gy1.float().cpu())
    print("N", N, "mean", mean.flatten()[:4].tolist(), "rstd", rstd.flatten()[:4].tolist())
    print("   ref mean", x1.float().mean((2, 3)).flatten()[:4].tolist())
    print("   dx err img0", (dx[0:1].float().cpu() - xr.grad).abs().max().item(), "strides", dx.stride(), x.stride())
