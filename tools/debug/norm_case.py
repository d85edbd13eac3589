import sys, zlib, torch, torch.nn.functional as F
sys.path.insert(0, ".")
from p2p_pytorch_amd import _native, ops
_native.set_backend("native")
DEV = "cuda"
def bf(x): return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for (N, C, H, W) in [(1, 3, 2, 2), (1, 8, 2, 2), (1, 8, 4, 4), (2, 16, 2, 3), (1, 3, 5, 5)]:
    g = torch.Generator(device=DEV).manual_seed(7)
    x = bf(torch.randn(N, C, H, W, device=DEV, generator=g) * 2 + 1)
    gy = bf(torch.randn(N, C, H, W, device=DEV, generator=g))
    hx = x.clone().requires_grad_(True)
    y = ops.instance_norm(hx)
    y.backward(gy)
    rx = x.float().cpu().requires_grad_(True)
    z = F.instance_norm(rx, eps=1e-5); z.backward(gy.float().cpu())
    print((N, C, H, W), "fwd err", (y.float().cpu() - z).abs().max().item(), "dx err", (hx.grad.float().cpu() - rx.grad).abs().max().item(), "dx max", rx.grad.abs().max().item())
    if (hx.grad.float().cpu() - rx.grad).abs().max().item() > 0.05:
        print(" hip", hx.grad.float().cpu().flatten()[:12].tolist()); print(" ref", rx.grad.flatten()[:12].tolist())
