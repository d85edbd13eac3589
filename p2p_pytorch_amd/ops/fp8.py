"""FP8 conv path (BASELINE config 5: "256x256 pix2pix with fp8 conv MFMA path").

Recipe (MI355X-first, see ``csrc/fp8.hip``):

* conv forward:  x in OCP e4m3 x weight e4m3 -> bf16 output (bias / act / norm stats fused
  as on the bf16 path);
* conv dgrad:    dY in e5m2 (gradient range) x weight e4m3 -> bf16 dX;
* conv wgrad:    dY e5m2 x X e4m3 on the same scaled MFMA, both operands read k-transposed
  with ds_read_b64_tr_b8 (csrc/conv_wgrad.hip ``conv_wgrad_f8_kernel``), from the fp8 copies
  the forward and the dgrad of that conv already made (the per-step quantisation cache keeps
  them until the backward); ``P2P_FP8_WGRAD=0`` keeps it bf16;
* first / last layers stay bf16: their channel counts (3 / 6-channel images, 1-channel
  PatchGAN logits) are below the fp8 kernel's 32-channel granularity, which is also the
  usual "keep the image-facing layers in high precision" rule for GANs.

Every fp8 tensor carries a per-tensor *power-of-two* scale, so dequantisation is an E8M0
exponent handed to the MFMA's own block-scale operands -- free in the matrix core, and the
two halves of a U-Net skip concat keep independent scales.  Scales live on the device in
"sites" (4 int32 words: amax_ref, amax_cur, e8m0, amax_last):

* activations / gradients: *delayed* scaling -- quantised with the amax of the previous two
  steps (``fp8_roll`` shifts the window once per step, one launch for the whole pool); a
  site's first use measures the tensor itself (bootstrap);
* weights: *current* scaling -- exact amax of this step's weight image, then the cast.

Sites are keyed by (consumer weight, operand role), so they are stable across steps and the
whole step stays capturable in one hipGraph (no host sync anywhere).  The object part of a key
is ``obj_key(obj)``, never ``id(obj)``: ids are recycled once an object dies, and a new weight
that inherited a dead one's amax window quantised its first steps with a foreign scale (the
fp8 chain test saw 8-190x gradient errors after other tests' weights died).  A dead object's
sites return to the pool (reset before reuse).
"""
from __future__ import annotations

import itertools
import os
import weakref

import torch

from .. import _native

E4M3, E5M2 = 0, 1
_POOL_SITES = 4096

_precision = [os.environ.get("P2P_PRECISION", "bf16").lower()]
if _precision[0] not in ("bf16", "fp8"):
    raise ValueError(f"P2P_PRECISION must be 'bf16' or 'fp8', got {_precision[0]!r}")


def set_precision(name: str) -> None:
    """Conv GEMM operand precision on the HIP path: 'bf16' (default) or 'fp8'."""
    name = name.lower()
    if name not in ("bf16", "fp8"):
        raise ValueError(name)
    _precision[0] = name


def get_precision() -> str:
    return _precision[0]


def enabled() -> bool:
    return _precision[0] == "fp8"


class _Pool:
    def __init__(self, device):
        self.sites = torch.zeros(_POOL_SITES, 4, dtype=torch.int32, device=device)
        self.index: dict = {}
        self.fresh: set = set()
        self.free: list = []     # rows of released keys (reset when handed out again)
        self.high = 0            # rows ever used: [0, high) is what the per-step roll covers

    def site(self, key):
        i = self.index.get(key)
        if i is None:
            if self.sites.is_cuda and torch.cuda.is_current_stream_capturing():
                # a new site inside a hipGraph capture would bake its (re)initialisation into
                # every replay and its row pointer into the graph: only sites
                # registered by the eager warmup steps may be used under capture
                raise RuntimeError(f"fp8: new scale site {key!r} ({_describe(key)}) requested during "
                                   "graph capture; run an eager warmup step first")
            if self.free:
                i = self.free.pop()
                self.sites[i].zero_()    # no amax window inherited from the previous owner
            else:
                i = self.high
                if i >= _POOL_SITES:
                    raise RuntimeError("fp8: scale-site pool exhausted")
                self.high += 1
            self.index[key] = i
            self.fresh.add(i)
        return i

    def release(self, okey):
        """Drop every site keyed by object key ``okey`` (alone or as a tuple's head)."""
        dead = [k for k in self.index
                if k == okey or (isinstance(k, tuple) and k and k[0] == okey)]
        for k in dead:
            i = self.index.pop(k)
            self.fresh.discard(i)
            self.free.append(i)


# object -> key: id(obj) maps to (weakref, key); a recycled id with a dead weakref gets a new key
_obj_keys: dict = {}
_key_counter = itertools.count(1)
# key -> short description of its object (type / shape / leaf), for the capture error
_key_desc: dict = {}


def _describe(key):
    k = key[0] if isinstance(key, tuple) and key and isinstance(key[0], tuple) else key
    return _key_desc.get(k, "no object")


def obj_key(obj):
    """Process-unique scale-site key of a live object (weight tensor / norm module)."""
    ent = _obj_keys.get(id(obj))
    if ent is not None and ent[0]() is obj:
        return ent[1]
    k = ("obj", next(_key_counter))
    oid = id(obj)
    if isinstance(obj, torch.Tensor):
        _key_desc[k] = f"tensor {tuple(obj.shape)} {obj.dtype} leaf={obj.is_leaf} grad_fn={type(obj.grad_fn).__name__}"
    else:
        _key_desc[k] = type(obj).__name__

    def _dead(_ref, oid=oid, k=k):
        _key_desc.pop(k, None)
        cur = _obj_keys.get(oid)
        if cur is not None and cur[1] == k:
            del _obj_keys[oid]
        for pools in (_pools, _wpools):
            for p in pools.values():
                p.release(k)
    _obj_keys[oid] = (weakref.ref(obj, _dead), k)
    return k


_pools: dict = {}
_wpools: dict = {}   # current-scaling weight sites (never rolled; word 0 recomputed per step)
# per-step cache of quantised activations: (ptr, shape, version, site) -> (x, q)
_qcache: dict = {}
# fp8 "shadows" written by the producer of a bf16 tensor in the same pass (norm apply /
# norm backward / conv epilogue): (ptr, shape, version) -> (x, q, site)
_shadows: dict = {}


def _pool(device) -> _Pool:
    p = _pools.get(device)
    if p is None:
        p = _Pool(device)
        _pools[device] = p
    return p


def site_tensor(device, key) -> torch.Tensor:
    p = _pool(device)
    return p.sites[p.site(key)]


def wpool(device) -> _Pool:
    p = _wpools.get(device)
    if p is None:
        p = _Pool(device)
        _wpools[device] = p
    return p


def producer_site(device, key):
    """(site, fresh) for a producer-side fused shadow.  A fresh site has no amax history
    yet: the caller produces no fused shadow this time and calls ``bootstrap_shadow``."""
    p = _pool(device)
    i = p.site(key)
    fresh = i in p.fresh
    return p.sites[i], fresh


def stash_shadow(x: torch.Tensor, q: torch.Tensor, site: torch.Tensor) -> None:
    _shadows[(x.data_ptr(), tuple(x.shape), x._version)] = (x, q, site)


def bootstrap_shadow(x: torch.Tensor, key, fmt: int) -> None:
    """First step of a producer site: measure the tensor, quantise it standalone, stash it."""
    P = _native.ops()
    p = _pool(x.device)
    i = p.site(key)
    p.fresh.discard(i)
    site = p.sites[i]
    site[0].zero_()
    P.fp8_amax(x, site, 0)
    stash_shadow(x, P.fp8_quant(x, site, fmt, 0), site)


def _shadow_dtype(fmt):
    return torch.float8_e4m3fn if fmt == E4M3 else torch.float8_e5m2


def shadow_buffer(like: torch.Tensor, fmt: int) -> torch.Tensor:
    return torch.empty(like.shape, dtype=_shadow_dtype(fmt), device=like.device,
                       memory_format=torch.channels_last)


def begin_step() -> None:
    """Shift every delayed-scaling window (one launch per device) and drop the per-step
    quantisation cache."""
    _qcache.clear()
    _shadows.clear()
    P = _native.ops()
    for p in _pools.values():
        if p.index:
            P.fp8_roll(p.sites[: p.high])


def quant(x: torch.Tensor, key, fmt: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Delayed-scaled fp8 copy of the bf16 NHWC tensor ``x`` (site ``key``); returns (q, site).
    The same tensor quantised twice for the same site in one step is reused."""
    sh = _shadows.get((x.data_ptr(), tuple(x.shape), x._version))
    if sh is not None and sh[1].dtype == _shadow_dtype(fmt):
        return sh[1], sh[2]
    P = _native.ops()
    pool = _pool(x.device)
    i = pool.site(key)
    site = pool.sites[i]
    ck = (x.data_ptr(), tuple(x.shape), x._version, i)
    ent = _qcache.get(ck)
    if ent is not None:
        return ent[1], site
    if i in pool.fresh:
        # bootstrap: the first quantisation of a site measures the tensor itself
        pool.fresh.discard(i)
        site[0].zero_()
        P.fp8_amax(x, site, 0)
    q = P.fp8_quant(x, site, fmt, 0)
    _qcache[ck] = (x, q)   # the entry holds x: its address cannot be recycled this step
    return q, site


def quant_weight(img: torch.Tensor, key) -> tuple[torch.Tensor, torch.Tensor]:
    """Current-scaled e4m3 copy of a bf16 weight image: exact amax, then the cast."""
    P = _native.ops()
    pool = _pool(img.device)
    i = pool.site(key)
    pool.fresh.discard(i)
    site = pool.sites[i]
    P.fp8_word_zero(site, 1, 0)
    P.fp8_amax(img, site, 0)
    return P.fp8_quant(img, site, E4M3, 0), site


def prepare_weight_pairs(ws, xa, xb, owners=None):
    """e4m3 GEMM images (both layouts) of fp32 masters ``ws`` with current scaling: one
    fill (zero the amax words), one multi-tensor amax launch, one image launch per 24
    tensors.  Returns [(img0, img1, site)].  ``owners``: the parameters the sites are keyed
    by (``ws`` may be per-call ``detach()`` views, new objects every step -- keyed by
    themselves they would take a new site each step, which a hipGraph capture refuses)."""
    if not ws:
        return []
    P = _native.ops()
    wp = wpool(ws[0].device)
    idx = [wp.site(obj_key(o)) for o in (owners if owners is not None else ws)]
    P.fp8_word_zero(wp.sites, wp.high, 0)
    P.fp8_amax_multi(list(ws), wp.sites, idx)
    imgs = P.weight_prep_pairs(list(ws), list(xa), list(xb), wp.sites, idx)
    return [(imgs[2 * j], imgs[2 * j + 1], wp.sites[i]) for j, i in enumerate(idx)]


def pair_ok(A: int, B: int) -> bool:
    """Both GEMM images of a weight [A][B][k][k] feed fp8 convs (fwd and dgrad): the
    channel granularity and N-tile limits of ``conv_ok`` hold for both orientations."""
    return A % 32 == 0 and B % 32 == 0 and A > 32 and B > 32


def conv_ok(C1: int, C2: int, Cout: int, act_in: int) -> bool:
    """Geometries the fp8 kernels take: the LDS-DMA conv with every 32-deep k block inside
    one source tensor, N tile >= 64, input activation none / ReLU."""
    if os.environ.get("P2P_CONV_VARIANT", "").startswith("v"):
        return False
    return Cout > 32 and C1 % 32 == 0 and C2 % 32 == 0 and act_in in (0, 1) and C1 <= 1024 and C2 <= 1024
