import sys, torch, torch.nn.functional as F
sys.path.insert(0, ".")
from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import fp8 as f8, hip
_native.set_backend("native"); assert _native.load()
DEV = "cuda"
def bf(x): return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for (C1, C2, s2, tr) in [(64, 64, 40.0, False), (64, 64, 1.0, False), (64, 64, 0.0, False), (128, 128, 40.0, False), (64,64,1/64.,False)]:
    torch.manual_seed(0)
    N, H, Cout, k, s, p = 2, 16, 128, 4, 2, 1
    x1 = bf(torch.randn(N, C1, H, H, device=DEV))
    x2 = bf(torch.randn(N, C2, H, H, device=DEV) * s2)
    w = torch.randn(Cout, C1 + C2, k, k, device=DEV) / ((C1 + C2) * k * k) ** 0.5
    f8.set_precision("bf16"); hip.begin_step()
    yb = ops.conv2d((x1, x2), w, None, s, p).float()
    f8.set_precision("fp8"); hip.begin_step()
    y8 = ops.conv2d((x1, x2), w, None, s, p).float()
    torch.cuda.synchronize()
    e = ((y8 - yb).abs().max() / yb.abs().max()).item()
    # part-wise: only x1, only x2
    f8.set_precision("bf16"); hip.begin_step()
    y1 = ops.conv2d((x1, torch.zeros_like(x2)), w, None, s, p).float()
    y2 = ops.conv2d((torch.zeros_like(x1), x2), w, None, s, p).float()
    r1 = ((y8 - y1).abs().max() / yb.abs().max()).item()
    # best scalar fit y8 ~ a*y1 + b*y2
    A = torch.stack([y1.flatten(), y2.flatten()], 1)
    sol = torch.linalg.lstsq(A.cpu(), y8.flatten().cpu().unsqueeze(1)).solution.flatten().tolist()
    print(f"C1={C1} C2={C2} s2={s2}: rel err vs bf16 {e:.4f}; vs x1-only {r1:.4f}; fit a,b = {sol}")
