import sys, torch, torch.nn.functional as F
sys.path.insert(0, ".")
from p2p_pytorch_amd import _native
_native.set_backend("native"); assert _native.load()
P = _native.ops()
DEV = "cuda"
def bf(x): return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for (N, C, H, W) in [(1, 8, 4, 4), (1, 8, 16, 16), (1, 8, 15, 16), (1, 8, 8, 8)]:
    g = torch.Generator(device=DEV).manual_seed(7)
    x = bf(torch.randn(N, C, H, W, device=DEV, generator=g) * 2 + 1)
    gy = bf(torch.randn(N, C, H, W, device=DEV, generator=g))
    y, mean, rstd = P.norm_fwd(x, 1e-5, None, None, None, 0, None, None, 0.1, False, None)
    dx = P.norm_bwd(x, gy, mean, rstd, None, None, 0, None, None, True, False, None).float().cpu()
    xf, gf = x.float().cpu(), gy.float().cpu()
    m, r = mean.cpu().view(N, C, 1, 1), rstd.cpu().view(N, C, 1, 1)
    xh = (xf - m) * r
    ref = r * (gf - gf.mean((2, 3), keepdim=True) - xh * (gf * xh).mean((2, 3), keepdim=True))
    print((N, C, H, W), "err", (dx - ref).abs().max().item())
    for c in range(2):
        A = torch.stack([gf[0, c].flatten(), torch.ones(H * W), xh[0, c].flatten()], 1)
        sol = torch.linalg.lstsq(A, dx[0, c].flatten().unsqueeze(1)).solution.flatten().tolist()
        exp = [r[0, c].item(), (-r[0, c] * gf[0, c].mean()).item(), (-r[0, c] * (gf[0, c] * xh[0, c]).mean()).item()]
        print("  c", c, "fit A,B,Cc", [round(v, 4) for v in sol], "expected", [round(v, 4) for v in exp])
