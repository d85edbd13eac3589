# which weight images miss the prepare_weights cache in fp8 mode (prints key + shape)
import sys, collections, torch
sys.path.insert(0, ".")
from p2p_pytorch_amd import _native
from p2p_pytorch_amd.ops import fp8 as f8, hip
from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
from p2p_pytorch_amd.models import define_D, define_G
_native.set_backend("native"); f8.set_precision("fp8")
dev = torch.device("cuda")
G = define_G(netG="unet_256", gpu_id=dev, verbose=False)
D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
step = Pix2PixStep(G, D)
A = (torch.rand(4, 3, 256, 256, device=dev) * 2 - 1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for i in range(3):
    miss = collections.Counter()
    orig = hip._weight_image
    def wrapped(w, swap, xp, yp, scale=None, _o=orig):
        c = getattr(w, "_p2p_cache", {}) or {}
        ent = c.get((swap, xp, yp, None))
        if not (ent is not None and ent[0] == w._version and ent[1] == hip._gen[0]):
            miss[(tuple(w.shape), swap, xp, yp)] += 1
        return _o(w, swap, xp, yp, scale)
    hip._weight_image = wrapped
    step.step(A, A)
    hip._weight_image = orig
    torch.cuda.synchronize()
    print("step", i, "misses", dict(miss))
