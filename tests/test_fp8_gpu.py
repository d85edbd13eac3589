"""FP8 conv path (csrc/fp8.hip, conv_fwd_glds.hip F8 instantiations) on the MI355X.

* quantiser: our e4m3 / e5m2 bytes equal PyTorch's own float8 conversion of x * 2^k
  (round-to-nearest-even, saturated), k the power-of-two scale derived from the amax;
* conv kernels: the fp8 conv equals an fp32 conv of the *dequantised* operands (every fp8
  value times its power-of-two scale is exact in fp32), so the tolerance only absorbs
  accumulation order and the bf16 output rounding;
* end to end: a U-Net-256 + PatchGAN step in fp8 stays close to the bf16 step.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import fp8 as f8
from p2p_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _s2t_f8_all(monkeypatch):
    """Both fp8 halo-kernel variants routed (P2P_S2T_F8 bits, csrc/bindings.cpp): the tests
    that assert the kernel ran keep covering it whatever the step's default routing is."""
    monkeypatch.setenv("P2P_S2T_F8", "3")


@pytest.fixture(autouse=True)
def _fp8_mode():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    f8.set_precision("fp8")
    hip.begin_step()
    yield
    f8.set_precision("bf16")


def bf(x):
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def rand_img(n, c, h, w, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return bf(torch.randn(n, c, h, w, device=DEV, generator=g) * scale)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _pow2_exp(amax, fmax):
    return math.frexp(fmax / amax)[1] - 1


@pytest.mark.parametrize("fmt,tdt,fmax", [(0, torch.float8_e4m3fn, 448.0), (1, torch.float8_e5m2, 57344.0)])
def test_quant_matches_torch_float8(fmt, tdt, fmax):
    x = rand_img(2, 64, 8, 8, scale=3.0, seed=1)
    site = torch.zeros(4, dtype=torch.int32, device=DEV)
    P = _native.ops()
    P.fp8_amax(x, site, 0)
    q = P.fp8_quant(x, site, fmt, 0)
    torch.cuda.synchronize()
    amax = x.float().abs().max().item()
    assert site[0].view(torch.float32).item() == pytest.approx(amax)
    assert site[1].view(torch.float32).item() == pytest.approx(amax)   # amax_cur recorded
    k = _pow2_exp(amax, fmax)
    assert int(site[2].item()) == 127 - k
    expect = (x.float() * 2.0 ** k).clamp(-fmax, fmax).to(tdt)
    assert torch.equal(q.view(torch.uint8), expect.view(torch.uint8))
    # dequant is exact
    y = P.fp8_dequant(q, site)
    assert torch.equal(y.float(), expect.float() * 2.0 ** -k)


def test_roll_window():
    P = _native.ops()
    sites = torch.zeros(3, 4, dtype=torch.int32, device=DEV)
    f = sites.view(torch.float32)
    f[0, 1] = 2.0    # cur
    f[0, 3] = 5.0    # last step
    f[1, 0] = 7.0    # ref kept when nothing was seen
    P.fp8_roll(sites)
    torch.cuda.synchronize()
    assert f[0, 0].item() == 5.0 and f[0, 3].item() == 2.0 and f[0, 1].item() == 0.0
    assert f[1, 0].item() == 7.0


def _deq(q, site):
    return _native.ops().fp8_dequant(q, site).float()


FP8_CASES = [
    # name, N, C1, C2, H, Cout, k, s, p, act_in, transposed
    ("enc_c64_nonfastk", 2, 64, 0, 32, 128, 4, 2, 1, None, False),
    ("enc_c128_fastk", 2, 128, 0, 16, 256, 4, 2, 1, None, False),
    ("patch_s1_c256", 2, 256, 0, 10, 512, 4, 1, 1, None, False),
    ("convT_concat_relu", 2, 128, 128, 8, 128, 4, 2, 1, "relu", True),
    ("convT_concat64_relu", 2, 64, 64, 16, 64, 4, 2, 1, "relu", True),
    ("convT_inner_c512", 2, 512, 0, 2, 512, 4, 2, 1, None, True),
    ("enc_concat64", 2, 64, 64, 16, 128, 4, 2, 1, None, False),
    ("convT_c64_relu", 2, 64, 0, 16, 64, 4, 2, 1, "relu", True),
    ("convT_concat64_norelu", 2, 64, 64, 16, 64, 4, 2, 1, None, True),
    ("convT_concat64_cout128", 2, 64, 64, 16, 128, 4, 2, 1, "relu", True),
    ("enc_concat64_relu_cout64", 2, 64, 64, 16, 64, 3, 1, 1, "relu", False),
    # 64-wide grids with 128-channel multiples: the class-shared halo kernel (conv_s2t.hip F8)
    ("s2t_convT_concat_relu", 4, 128, 128, 64, 64, 4, 2, 1, "relu", True),
    ("s2t_convT_c128_cout128", 4, 128, 0, 64, 128, 4, 2, 1, None, True),
    ("s2t_dgrad_c64_cout128", 4, 64, 0, 128, 128, 4, 2, 1, None, False),
    # >= 256 output tiles and 128-channel multiples: the 32x32x64 f8f6f4 tiles (conv_fwd_m32.hip
    # F8 = 1 forward / 2 input gradient, round 6) -- conv (MODE 0 fwd, MODE 1 dgrad), ConvT on a
    # virtual concat with input ReLU (MODE 1 fwd, MODE 0 dgrad), and a Cout that is not a tile
    # multiple
    # (Cout 65..128: the fp8 m32 route; wider layers stay on the glds 256 x 256 fp8 tile)
    ("m32_enc_c128", 64, 128, 0, 64, 128, 4, 2, 1, None, False),
    ("m32_convT_concat_relu", 64, 128, 128, 32, 128, 4, 2, 1, "relu", True),
    ("m32_enc_c256_cout96", 64, 256, 0, 64, 96, 4, 2, 1, None, False),
    ("m32_convT_c128", 64, 128, 0, 32, 128, 4, 2, 1, None, True),
]


@pytest.mark.parametrize("case", FP8_CASES, ids=[c[0] for c in FP8_CASES])
def test_fp8_conv_fwd_dgrad_match_dequantised_oracle(case):
    name, N, C1, C2, H, Cout, k, s, p, act_in, transposed = case
    x1 = rand_img(N, C1, H, H, seed=1)
    # the two concat halves get very different ranges: per-source scales must hold
    x2 = rand_img(N, C2, H, H, scale=40.0, seed=2) if C2 else None
    Cin = C1 + C2
    g = torch.Generator(device=DEV).manual_seed(5)
    if transposed:
        w = torch.randn(Cin, Cout, k, k, device=DEV, generator=g) * (1.0 / (Cin * k * k) ** 0.5)
    else:
        w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) * (1.0 / (Cin * k * k) ** 0.5)
    w.requires_grad_(True)
    xin1 = x1.detach().clone().requires_grad_(True)
    xin2 = x2.detach().clone().requires_grad_(True) if x2 is not None else None
    xin = (xin1, xin2) if xin2 is not None else xin1
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        if transposed:
            y = ops.conv_transpose2d(xin, w, None, s, p, act_in=act_in)
        else:
            y = ops.conv2d(xin, w, None, s, p, act_in=act_in)
        gy = rand_img(*y.shape, scale=1e-3, seed=3)     # gradient-sized values: e5m2 + scaling
        y.backward(gy)
        torch.cuda.synchronize()
    if name.startswith("m32_"):
        names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
        # e4m3 forward and e5m2 input gradient on the 32x32x64 tiles where the route takes them:
        # 128-channel multiples in, 65..128 channels out (the input gradient reads dY = Cout
        # channels and writes Cin)
        dgrad_m32 = Cout % 128 == 0 and 64 < Cin <= 128
        for f in ((1, 2) if dgrad_m32 else (1,)):
            # (template arguments BN, MODE, RELU, EXT, F8, BM)
            assert any("conv_fwd_m32_kernel<128" in k and f", {f}, 256>(" in k for k in names), (f, sorted(set(names)))
    if name.startswith("s2t_"):
        names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
        want = "conv_s2t_kernel<64, true, false, 1>" if act_in == "relu" else (
            "conv_s2t_kernel<64, false, false, 1>" if transposed else "conv_s2t_kernel<64, false, false, 2>")
        assert any(want in k for k in names), (want, sorted(set(names)))

    # the fp8 operands exactly as the kernels saw them
    kk = f8.obj_key(w)
    pool = f8._pool(torch.device(DEV, torch.cuda.current_device()))
    sx1 = pool.sites[pool.index[(kk, "x", 1)]]
    q1 = next(q for (x_, q) in f8._qcache.values() if x_.data_ptr() == xin1.data_ptr())
    xd1 = _deq(q1, sx1)
    if x2 is not None:
        sx2 = pool.sites[pool.index[(kk, "x", 2)]]
        q2 = next(q for (x_, q) in f8._qcache.values() if x_.data_ptr() == xin2.data_ptr())
        xd2 = _deq(q2, sx2)
        xd = torch.cat([xd1, xd2], 1)
    else:
        xd = xd1
    swap = 1 if transposed else 0
    assert (swap, Cout, Cin, "fp8") in w._p2p_cache, list(w._p2p_cache.keys())
    w8, sw = w._p2p_cache[(swap, Cout, Cin, "fp8")][2]
    wd = _deq(w8, sw)   # [Cout][kh][kw][Cin] GEMM image of the fwd weight
    if transposed:
        # image 1 of a ConvT weight [Cin][Cout][kh][kw] is [Cout][kh][kw][Cin]
        wref = wd.view(Cout, k, k, Cin).permute(3, 0, 1, 2).contiguous()
    else:
        wref = wd.view(Cout, k, k, Cin).permute(0, 3, 1, 2).contiguous()
    xr = F.relu(xd) if act_in == "relu" else xd
    if transposed:
        yr = F.conv_transpose2d(xr, wref, None, s, p)
    else:
        yr = F.conv2d(xr, wref, None, s, p)
    e = rel_err(y, yr)
    if e >= 1e-2:
        d = (y.float() - yr).abs()
        bad = (d > 1e-2 * yr.abs().max()).nonzero()
        print(name, "bad count", bad.shape[0], "of", d.numel(), "first", bad[:8].tolist())
        print("channels with errors", sorted(set(bad[:, 1].tolist()))[:40])
        print("rows with errors", sorted(set(bad[:, 2].tolist()))[:40])
    assert e < 1e-2, f"{name}: fwd rel err {e}"

    # dgrad: e5m2 gradient x e4m3 weight (image of the dgrad layout) vs the same in fp32
    sg = pool.sites[pool.index[(kk, "gy", 1)]]
    gq = next(q for (x_, q) in f8._qcache.values() if x_.data_ptr() == gy.data_ptr())
    gyd = _deq(gq, sg)
    xr_leaf = xr.detach().clone().requires_grad_(True)
    yr2 = F.conv_transpose2d(xr_leaf, wref, None, s, p) if transposed else F.conv2d(xr_leaf, wref, None, s, p)
    yr2.backward(gyd)
    gref = xr_leaf.grad
    xb = torch.cat([x1, x2], 1) if x2 is not None else x1
    if act_in == "relu":
        gref = gref * (xb.float() > 0)      # the kernel gates with the bf16 input's sign
    gx = torch.cat([xin1.grad, xin2.grad], 1) if xin2 is not None else xin1.grad
    e = rel_err(gx, gref)
    # the dgrad weight image holds the same values (same amax -> same scale)
    assert e < 2e-2, f"{name}: dgrad rel err {e}"


def test_unet_step_fp8_close_to_bf16():
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    dev = torch.device(DEV)
    res = {}
    for prec in ("bf16", "fp8"):
        f8.set_precision(prec)
        torch.manual_seed(0)
        G = define_G(netG="unet_256", gpu_id=dev, verbose=False)
        D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
        step = Pix2PixStep(G, D)
        g = torch.Generator(device=DEV).manual_seed(1)
        A = bf(torch.rand(4, 3, 256, 256, device=dev, generator=g) * 2 - 1)
        B = bf(torch.rand(4, 3, 256, 256, device=dev, generator=g) * 2 - 1)
        vals = []
        for _ in range(3):
            losses = step.step(A, B)
            vals.append({k: float(v) for k, v in losses.items()})
        torch.cuda.synchronize()
        res[prec] = vals
    for k in res["bf16"][0]:
        a, b = res["bf16"][0][k], res["fp8"][0][k]
        assert math.isfinite(b), (k, b)
        assert abs(a - b) <= 0.05 * abs(a) + 0.02, (k, a, b)
    assert all(math.isfinite(v) for d in res["fp8"] for v in d.values())


def test_unet_step_fp8_captures():
    """The fp8 step is capturable in one hipGraph: every scale site (weights included) is
    registered by the eager warmup, so the capture asks for none (the weight-pair sites were
    once keyed by per-call ``detach()`` views -- a new site every step -- and bench.py's fp8
    line fell back to eager with a CaptureError)."""
    from p2p_pytorch_amd.engine.graph import CapturedStep
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    dev = torch.device(DEV)
    torch.manual_seed(0)
    G = define_G(netG="unet_256", gpu_id=dev, verbose=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
    step = Pix2PixStep(G, D)
    g = torch.Generator(device=DEV).manual_seed(1)
    A = bf(torch.rand(2, 3, 256, 256, device=dev, generator=g) * 2 - 1)
    B = bf(torch.rand(2, 3, 256, 256, device=dev, generator=g) * 2 - 1)
    p0 = next(G.parameters())
    w0 = p0.detach().clone()
    cap = CapturedStep(step.step, A, B, warmup=2)
    for _ in range(2):
        out = cap()
    torch.cuda.synchronize()
    vals = {k: float(v) for k, v in out.items()}
    assert all(math.isfinite(v) for v in vals.values()), vals
    assert not torch.equal(w0, p0.detach())   # the replays stepped the optimizer


def _expect_fp8(y, site, fmt):
    k = 127 - int(site[2].item())
    tdt, fmax = (torch.float8_e4m3fn, 448.0) if fmt == 0 else (torch.float8_e5m2, 57344.0)
    return (y.float() * 2.0 ** k).clamp(-fmax, fmax).to(tdt).view(torch.uint8)


@pytest.mark.parametrize("producer", ["norm", "conv_epilogue"])
def test_fused_shadows_equal_standalone_quantisation(producer):
    """Producer-fused fp8 shadows (norm apply / norm backward / conv epilogue) hold exactly
    fp8(value * 2^k) of the bf16 tensor they shadow, k from the site's delayed amax."""
    xl = rand_img(2, 64, 16, 16, seed=4).requires_grad_(True)
    g = torch.Generator(device=DEV).manual_seed(6)
    w = (torch.randn(64, 64, 3, 3, device=DEV, generator=g) * 0.05).requires_grad_(True)
    key = 777001
    for it in range(2):          # step 0 bootstraps the sites, step 1 uses the fused path
        hip.begin_step()
        # a non-leaf input: the gradient the norm backward returns reaches its hook as is
        # (a leaf's AccumulateGrad would clone it)
        x = xl * 1.0
        grads = []
        x.register_hook(grads.append)
        if producer == "norm":
            y = ops.instance_norm(x, act="lrelu", qkey=key)
        else:
            y = ops.conv2d(x, w, None, 1, 1, act_out="lrelu")
        ent = f8._shadows.get((y.data_ptr(), tuple(y.shape), y._version))
        assert ent is not None, "no shadow stashed"
        q, site = ent[1], ent[2]
        torch.cuda.synchronize()
        assert torch.equal(q.view(torch.uint8), _expect_fp8(y, site, 0)), f"fwd shadow, step {it}"
        if producer == "norm":
            gy = rand_img(*y.shape, scale=1e-3, seed=7)
            y.backward(gy)
            dx = grads[0]
            ent = f8._shadows.get((dx.data_ptr(), tuple(dx.shape), dx._version))
            assert ent is not None, "no dx shadow"
            torch.cuda.synchronize()
            assert torch.equal(ent[1].view(torch.uint8), _expect_fp8(dx, ent[2], 1)), f"dx shadow, step {it}"


def _deq(q, site):
    """fp8 tensor x its power-of-two scale -> exact fp32."""
    return q.float() * 2.0 ** (int(site[2].item()) - 127)


@pytest.mark.parametrize("case", ["conv_s2_relu", "convT_concat", "conv_s1_wide", "conv_c64", "convT_c64out"])
def test_fp8_wgrad_matches_dequantised_oracle(case):
    """fp8 weight gradient (e5m2 dY x e4m3 X on the scaled f8f6f4 MFMA, both operands read
    k-transposed with ds_read_b64_tr_b8) against an fp32 weight gradient of the DEQUANTISED
    operands: the products are exact in fp32, so the bound only absorbs summation order."""
    P = _native.ops()
    if case == "conv_s2_relu":      # U-Net e3-like: 128 -> 256, 4x4 s2 p1, input ReLU
        N, C1, C2, H, Cout, k, s, p, act, tr = 8, 128, 0, 32, 256, 4, 2, 1, 1, False
    elif case == "conv_s1_wide":    # PatchGAN c4-like: 256 -> 512, 4x4 s1 p1
        N, C1, C2, H, Cout, k, s, p, act, tr = 4, 256, 0, 17, 512, 4, 1, 1, 0, False
    elif case == "conv_c64":        # U-Net e2-like: 64 -> 128 (a 64-channel im2col side)
        N, C1, C2, H, Cout, k, s, p, act, tr = 4, 64, 0, 64, 128, 4, 2, 1, 0, False
    elif case == "convT_c64out":    # U-Net d2-like ConvT: (128 | 128) -> 64 (64-channel dY side)
        N, C1, C2, H, Cout, k, s, p, act, tr = 4, 128, 128, 32, 64, 4, 2, 1, 1, True
    else:                           # U-Net decoder ConvT on a skip concat: (128 | 128) -> 128
        N, C1, C2, H, Cout, k, s, p, act, tr = 8, 128, 128, 16, 128, 4, 2, 1, 1, True
    x1 = rand_img(N, C1, H, H, seed=61)
    x2 = rand_img(N, C2, H, H, seed=62) if C2 else None
    OH = (H - 1) * s - 2 * p + k if tr else (H + 2 * p - k) // s + 1
    gy = rand_img(N, Cout, OH, OH, scale=0.01, seed=63)
    sites = [torch.zeros(4, dtype=torch.int32, device=DEV) for _ in range(3)]
    qs = []
    for t, site, fmt in ((x1, sites[0], 0), (x2, sites[1], 0), (gy, sites[2], 1)):
        if t is None:
            qs.append(None)
            continue
        P.fp8_amax(t, site, 0)
        qs.append(P.fp8_quant(t, site, fmt, 0))
    x1q, x2q, gq = qs
    xd = _deq(x1q, sites[0])
    if x2q is not None:
        xd = torch.cat((xd, _deq(x2q, sites[1])), 1)
    xa = F.relu(xd) if act else xd
    gd = _deq(gq, sites[2])
    if tr:
        w = torch.zeros(C1 + C2, Cout, k, k, device=DEV, requires_grad=True)
        F.conv_transpose2d(xa, w, None, s, p).backward(gd)
        gw = torch.empty(C1 + C2, Cout, k, k, device=DEV)
        ok = P.conv_wgrad(x1q, x2q, act, gq, None, 0, k, k, s, p, 0, 1, gw, 1.0, 0, 0,
                          sites[0], sites[2], 0, 1, sites[1] if x2q is not None else None, None)
    else:
        w = torch.zeros(Cout, C1 + C2, k, k, device=DEV, requires_grad=True)
        F.conv2d(xa, w, None, s, p).backward(gd)
        gw = torch.empty(Cout, C1 + C2, k, k, device=DEV)
        ok = P.conv_wgrad(gq, None, 0, x1q, x2q, act, k, k, s, p, 0, 1, gw, 1.0, 0, 0,
                          sites[2], sites[0], 1, 0, None, sites[1] if x2q is not None else None)
    assert ok, "fp8 wgrad kernel did not take the geometry"
    assert rel_err(gw, w.grad) < 1e-4, rel_err(gw, w.grad)


def test_fp8_s2t_ext_dgrad_chain_matches_implicit_gemm(monkeypatch):
    """conv s2 -> IN + lrelu -> conv s2 (U-Net encoder / PatchGAN) in fp8: the second conv's
    input gradient runs on the fp8 halo kernel with the act' gate and the norm-backward
    partials in its extended epilogue (conv_s2t_kernel<64, false, true, 2>); the same chain
    with P2P_NO_S2T=1 (the implicit-GEMM fp8 tile) must agree up to fp8 scale / summation
    order noise -- an indexing error (tap, chunk, source scale) is an O(1) difference."""
    from torch.profiler import ProfilerActivity, profile
    x = rand_img(4, 64, 256, 256, seed=9)
    g = torch.Generator(device=DEV).manual_seed(11)
    w1 = torch.randn(64, 64, 4, 4, device=DEV, generator=g) * 0.03
    w2 = torch.randn(128, 64, 4, 4, device=DEV, generator=g) * 0.03

    def run():
        hip.begin_step()
        hx, hw1, hw2 = (t.detach().clone().requires_grad_(True) for t in (x, w1, w2))
        h = ops.instance_norm(ops.conv2d(hx, hw1, None, 2, 1, stats=True), act="lrelu")
        z = ops.conv2d(h, hw2, None, 2, 1)
        loss = (z.float() * torch.linspace(-1, 1, z.numel(), device=DEV).view_as(z)).sum()
        loss.backward()
        torch.cuda.synchronize()
        return hx.grad, hw1.grad, hw2.grad

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        run()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert any("conv_s2t_kernel<64, false, true, 2>" in k for k in names), sorted(set(names))
    outs = [run() for _ in range(2)]          # the second with settled fp8 scales
    monkeypatch.setenv("P2P_NO_S2T", "1")
    outs0 = [run() for _ in range(2)]
    monkeypatch.delenv("P2P_NO_S2T")
    errs = [rel_err(a, b) for a, b in zip(outs[1], outs0[1])]
    print("fp8 s2t vs implicit GEMM:", errs)
    assert all(e < 0.05 for e in errs), errs
