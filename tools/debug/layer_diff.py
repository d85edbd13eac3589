# forward activations of G (unet_128, ngf=32) on HIP vs the fp32 CPU oracle, layer by layer
import sys, torch
sys.path.insert(0, "."); sys.path.insert(0, "tools")
import p2p_pytorch_amd as p2p
from ddp_rehearsal import build, data
p2p.set_backend("native")
dev = torch.device("cuda")
ngf = int(sys.argv[1]) if len(sys.argv) > 1 else 32
netG = sys.argv[2] if len(sys.argv) > 2 else "unet_128"
size = int(sys.argv[3]) if len(sys.argv) > 3 else 128
from p2p_pytorch_amd.models import define_G
torch.manual_seed(0)
G = define_G(netG=netG, ngf=ngf, gpu_id=dev, verbose=False, use_dropout=False)
Gc = define_G(netG=netG, ngf=ngf, gpu_id="cpu", verbose=False, use_dropout=False)
Gc.load_state_dict({k: v.cpu() for k, v in G.state_dict().items()})
A, _ = data(1, dev, 2, size)
outs = {}
def hook(name, store):
    def f(m, i, o):
        store[name] = (o[0] if isinstance(o, tuple) else o).detach().float().cpu()
    return f
hg, hc = {}, {}
for (n, m), (n2, m2) in zip(G.named_modules(), Gc.named_modules()):
    if n and "." in n and n.count(".") == 1:
        m.register_forward_hook(hook(n, hg)); m2.register_forward_hook(hook(n2, hc))
with torch.no_grad():
    G(A); Gc(A.float().cpu())
order = [n for n, _ in G.named_modules() if n in hg]
for n in order:
    a, b = hg[n], hc[n]
    if a.shape != b.shape:
        print(n, "shape", a.shape, b.shape); continue
    s = b.abs().max().item()
    print(f"{n:16s} {tuple(b.shape)} rel {((a-b).abs().max().item()/max(s,1e-12)):.4f} max {s:.3f}")
