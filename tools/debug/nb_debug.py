"""Debug helper: which convs of a small graph get the fused norm-backward partials."""
import torch
from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import hip
_native.set_backend("native"); assert _native.load()
DEV = "cuda"
bf = lambda t: t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)  # noqa: E731
orig_call = hip._conv_call
def call(*a, **k):
    outs = orig_call(*a, **k)
    nb = k.get("nb")
    print("conv_call mode", a[4], "Cout", a[14], "Csplit", a[16], "nb", None if nb is None else nb[0], "outs", [tuple(o.shape) for o in outs])
    return outs
hip._conv_call = call
orig_take = hip._take_nbp
def take(g):
    ent = hip._nbp_stash.get((g.data_ptr(), tuple(g.shape)))
    print("take: key hit", ent is not None, "same obj", ent is not None and ent[0] is g, "stash", len(hip._nbp_stash))
    return orig_take(g)
hip._take_nbp = take
hip.begin_step()
skip = bf(torch.randn(32, 64, 32, 32, device=DEV))
v = bf(torch.randn(32, 128, 16, 16, device=DEV)).requires_grad_(True)
wi = (torch.randn(128, 64, 4, 4, device=DEV) * 0.04).requires_grad_(True)
wo = (torch.randn(128, 32, 4, 4, device=DEV) * 0.04).requires_grad_(True)
u = ops.instance_norm(ops.conv_transpose2d(v, wi, None, 2, 1, "relu", None, stats=True), act="relu")
print("registered", len(hip._norm_out), "lookup", hip._norm_lookup(u) is not None)
y = ops.conv_transpose2d((skip, u), wo, None, 2, 1, "relu", None, gate_x2=False)
y.backward(torch.ones_like(y))
print("stash after", len(hip._nbp_stash))
