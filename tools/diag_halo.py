"""Diag: halo_kxk conv vs the implicit-GEMM fallback on direct torch.ops.p2p.conv_fwd calls."""
import os
import sys
import torch
sys.path.insert(0, ".")
import p2p_pytorch_amd  # noqa: F401  (loads the extension)
from p2p_pytorch_amd.ops import hip

P = hip.P()
dev = "cuda"
torch.manual_seed(0)
for (C, Co, H, up, refl) in ((32, 8, 20, 1, 1), (16, 32, 10, 2, 1), (8, 32, 20, 1, 0)):
    x = torch.randn(1, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(Co, 9, 9, C, device=dev).to(torch.bfloat16).contiguous()
    b = torch.full((Co,), 0.5, device=dev)
    OH = H * up
    outs = []
    for env in (None, "1"):
        if env:
            os.environ["P2P_NO_HALO"] = env
        else:
            os.environ.pop("P2P_NO_HALO", None)
        y = P.conv_fwd(x, None, w, b, 0, 9, 9, 1, 4, refl, up, 0, OH, OH, Co, 0, Co, None, None, 0)[0]
        torch.cuda.synchronize()
        outs.append(y.float())
    d = (outs[0] - outs[1]).abs().max().item()
    print(C, Co, H, up, refl, "halo max", outs[0].abs().max().item(), "gemm max", outs[1].abs().max().item(),
          "diff", d, flush=True)
    print(outs[0][0, :4, 0, :4], outs[1][0, :4, 0, :4], flush=True)
