# G grads at batch 4 vs mean of two batch-2 halves vs the fp32 CPU oracle
import sys, torch
sys.path.insert(0, ".")
import p2p_pytorch_amd as p2p
from p2p_pytorch_amd.engine.pix2pix import set_requires_grad
from p2p_pytorch_amd.ops import hip
sys.path.insert(0, "tools")
from ddp_rehearsal import build, data, g_grads
p2p.set_backend("native")
dev = torch.device("cuda")
A, B = data(2, dev, 2)
def grads(a, b, seed=100, device=dev):
    G, D = build(seed, dev)
    if device.type == "cpu":
        G, D = G.cpu(), D.cpu()
        a, b = a.float().cpu(), b.float().cpu()
    set_requires_grad(D, False)
    hip.begin_step()
    g_grads(G, D, a, b) if device.type == "cuda" else None
    if device.type == "cpu":
        from p2p_pytorch_amd.models import GANLoss
        from p2p_pytorch_amd.ops import l1
        fake = G(a)
        loss = GANLoss(gan_mode="vanilla")(D(torch.cat((a, fake), 1)), True) + 100 * l1(fake, b)
        loss.backward()
    return {n: p.grad.float().cpu() for n, p in G.named_parameters()}
g4 = grads(A, B)
g2a = grads(A[:2], B[:2]); g2b = grads(A[2:], B[2:])
gc = grads(A, B, device=torch.device("cpu"))
gc2a = grads(A[:2], B[:2], device=torch.device("cpu")); gc2b = grads(A[2:], B[2:], device=torch.device("cpu"))
def e(x, r):
    s = r.abs().max().item()
    return ((x - r).abs().max().item() / s) if s > 1e-8 else 0.0
for n in g4:
    print(f"{n:28s} hip4-vs-cpu4 {e(g4[n], gc[n]):.4f}  hip2avg-vs-cpu4 {e((g2a[n]+g2b[n])/2, gc[n]):.4f}  cpu2avg-vs-cpu4 {e((gc2a[n]+gc2b[n])/2, gc[n]):.4f}  hip2a-vs-cpu2a {e(g2a[n], gc2a[n]):.4f}")
