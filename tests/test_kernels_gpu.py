"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

The HIP side runs bf16 activations (fp32 accumulate, fp32 master weights); the oracle runs
the identical math in fp32 on the *same bf16-rounded inputs*, so the tolerance only has
to absorb bf16 output rounding and accumulation order.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from p2p_pytorch_amd import _native
from p2p_pytorch_amd import ops
from p2p_pytorch_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_backend():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    yield


def _record(tag, rows):
    """Append measured (name, err_native, err_eager_bf16) rows to gpurun_out/bounds.jsonl
    (tolerance calibration evidence; no-op when the directory is absent)."""
    import json
    import os
    if os.path.isdir("gpurun_out"):
        with open("gpurun_out/bounds.jsonl", "a") as f:
            f.write(json.dumps({"test": tag, "rows": rows}) + "\n")


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def bf(x):
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def rand_img(n, c, h, w, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return bf(torch.randn(n, c, h, w, device=DEV, generator=g) * scale)


def _leaf(x):
    return x.detach().clone().requires_grad_(True)


CONV_CASES = [
    # (name, N, C1, C2, H, Cout, k, s, p, act_in, act_out, bias)
    ("enc_s2", 2, 64, 0, 32, 128, 4, 2, 1, "lrelu", None, True),
    ("first_c3", 2, 3, 0, 32, 64, 4, 2, 1, None, None, True),
    ("d_input_concat3+3", 2, 3, 3, 32, 64, 4, 2, 1, None, None, True),
    ("patch_s1", 2, 256, 0, 10, 512, 4, 1, 1, "lrelu", None, True),
    ("patch_out_c1", 2, 512, 0, 9, 1, 4, 1, 1, "lrelu", None, True),
    ("bottleneck_splitk", 2, 512, 0, 4, 512, 4, 2, 1, "lrelu", None, True),
    ("one_by_one", 2, 64, 0, 16, 128, 1, 1, 0, "lrelu", None, True),
    ("concat_64+64", 2, 64, 64, 16, 64, 3, 1, 1, "relu", None, False),
    # 8-channel input, 128 outputs, 4x4: the 128x128 glds wgrad tile (Kq = 128)
    ("c8_r128_wgrad128", 4, 8, 0, 64, 128, 4, 2, 1, None, None, True),
    ("c8_r128_relu_in", 4, 8, 0, 64, 128, 4, 2, 1, "relu", None, True),
]


@pytest.mark.parametrize("case", CONV_CASES, ids=[c[0] for c in CONV_CASES])
def test_conv2d_fwd_bwd(case):
    name, N, C1, C2, H, Cout, k, s, p, act_in, act_out, use_bias = case
    torch.manual_seed(0)
    x1 = rand_img(N, C1, H, H, seed=1)
    x2 = rand_img(N, C2, H, H, seed=2) if C2 else None
    Cin = C1 + C2
    w = (torch.randn(Cout, Cin, k, k, device=DEV) * (1.0 / (Cin * k * k) ** 0.5))
    b = torch.randn(Cout, device=DEV) * 0.1 if use_bias else None
    # HIP
    hx1, hw = _leaf(x1), _leaf(w)
    hx2 = _leaf(x2) if x2 is not None else None
    hb = _leaf(b) if b is not None else None
    xin = (hx1, hx2) if hx2 is not None else hx1
    y = ops.conv2d(xin, hw, hb, s, p, act_in=act_in, act_out=act_out)
    gy = rand_img(*y.shape, seed=3)
    y.backward(gy)
    # fp32 oracle on the same bf16 inputs
    rx1, rw = _leaf(x1.float()), _leaf(w)
    rx2 = _leaf(x2.float()) if x2 is not None else None
    rb = _leaf(b) if b is not None else None
    rin = (rx1, rx2) if rx2 is not None else rx1
    # the HIP path computes with bf16 weights: round the oracle's weight the same way
    ry = ref.conv2d(rin, rw.to(torch.bfloat16).float(), rb, s, p, act_in=act_in, act_out=act_out)
    ry.backward(gy.float())
    assert y.shape == ry.shape
    assert rel_err(y, ry) < 2e-2, name
    assert rel_err(hx1.grad, rx1.grad) < 3e-2, name
    if x2 is not None:
        assert rel_err(hx2.grad, rx2.grad) < 3e-2, name
    assert rel_err(hw.grad, rw.grad) < 3e-2, name
    if b is not None:
        assert rel_err(hb.grad, rb.grad) < 3e-2, name


CONVT_CASES = [
    # (name, N, C1, C2, H, Cout, act_in, act_out, bias)
    ("dec_concat", 2, 64, 64, 16, 32, "relu", None, True),
    ("innermost_1x1", 4, 512, 0, 1, 512, "relu", None, True),
    ("dec_2x2_concat", 2, 512, 512, 2, 512, "relu", None, True),
    ("head_tanh_c3", 2, 64, 64, 32, 3, "relu", "tanh", True),
]


@pytest.mark.parametrize("case", CONVT_CASES, ids=[c[0] for c in CONVT_CASES])
def test_conv_transpose2d_fwd_bwd(case):
    name, N, C1, C2, H, Cout, act_in, act_out, use_bias = case
    x1 = rand_img(N, C1, H, H, seed=4)
    x2 = rand_img(N, C2, H, H, seed=5) if C2 else None
    Cin = C1 + C2
    w = torch.randn(Cin, Cout, 4, 4, device=DEV) * (1.0 / (Cin * 4) ** 0.5)
    b = torch.randn(Cout, device=DEV) * 0.1 if use_bias else None
    hx1, hw = _leaf(x1), _leaf(w)
    hx2 = _leaf(x2) if x2 is not None else None
    hb = _leaf(b) if b is not None else None
    y = ops.conv_transpose2d((hx1, hx2) if hx2 is not None else hx1, hw, hb, 2, 1, act_in, act_out)
    gy = rand_img(*y.shape, seed=6)
    y.backward(gy)
    rx1, rw = _leaf(x1.float()), _leaf(w)
    rx2 = _leaf(x2.float()) if x2 is not None else None
    rb = _leaf(b) if b is not None else None
    ry = ref.conv_transpose2d((rx1, rx2) if rx2 is not None else rx1,
                              rw.to(torch.bfloat16).float(), rb, 2, 1, act_in, act_out)
    ry.backward(gy.float())
    assert y.shape == ry.shape == (N, Cout, 2 * H, 2 * H)
    assert rel_err(y, ry) < 2e-2, name
    assert rel_err(hx1.grad, rx1.grad) < 3e-2, name
    if x2 is not None:
        assert rel_err(hx2.grad, rx2.grad) < 3e-2, name
    assert rel_err(hw.grad, rw.grad) < 3e-2, name
    if b is not None:
        assert rel_err(hb.grad, rb.grad) < 3e-2, name


REFLECT_CASES = [
    # (name, N, Cin, H, Cout, k, s, pad_mode, up, act_in)  -- family-R ConvLayer shapes
    ("res3x3", 2, 64, 16, 64, 3, 1, "reflect", 1, None),
    ("head9x9_c12", 2, 12, 24, 32, 9, 1, "reflect", 1, None),
    ("down3x3_s2", 2, 32, 20, 64, 3, 2, "reflect", 1, "relu"),
    ("c5x5_c3", 2, 3, 16, 64, 5, 1, "reflect", 1, None),
    ("up2_3x3", 2, 64, 8, 32, 3, 1, "reflect", 2, None),
    ("up2_zeros", 2, 32, 12, 64, 3, 1, "zeros", 2, None),
    ("tail9x9_c3", 2, 32, 16, 3, 9, 1, "reflect", 1, None),
]


@pytest.mark.parametrize("case", REFLECT_CASES, ids=[c[0] for c in REFLECT_CASES])
def test_conv_reflect_upsample_fwd_bwd(case):
    name, N, Cin, H, Cout, k, s, pad_mode, up, act_in = case
    x = rand_img(N, Cin, H, H, seed=7)
    w = torch.randn(Cout, Cin, k, k, device=DEV) * (1.0 / (Cin * k * k) ** 0.5)
    b = torch.randn(Cout, device=DEV) * 0.1
    hx, hw, hb = _leaf(x), _leaf(w), _leaf(b)
    y = ops.conv2d(hx, hw, hb, s, k // 2, pad_mode=pad_mode, upsample=up, act_in=act_in)
    gy = rand_img(*y.shape, seed=8)
    y.backward(gy)
    rx, rw, rb = _leaf(x.float()), _leaf(w), _leaf(b)
    ry = ref.conv2d(rx, rw.to(torch.bfloat16).float(), rb, s, k // 2, pad_mode=pad_mode,
                    upsample=up, act_in=act_in)
    ry.backward(gy.float())
    assert y.shape == ry.shape
    assert rel_err(y, ry) < 2e-2, name
    assert rel_err(hx.grad, rx.grad) < 3e-2, name
    assert rel_err(hw.grad, rw.grad) < 3e-2, name
    assert rel_err(hb.grad, rb.grad) < 3e-2, name


FOLD_CASES = [
    # (N, Cin, H, W, k, s, act_in): the reflect-pad dgrad folded in the conv epilogue + frame band
    (2, 128, 16, 16, 3, 1, "relu"),      # residual-block conv (256x128 EXT tile, ReLU gate)
    (2, 64, 20, 18, 3, 2, "lrelu"),      # G.conv2 / conv3 (stride 2: four parity classes)
    (2, 64, 12, 14, 5, 1, None),         # pad 2: two-pixel frame and bands
    (2, 12, 24, 20, 9, 1, None),         # pad 4, 16-channel gradient (register-staged tile)
    (1, 32, 6, 6, 3, 1, "relu"),         # smallest band geometry H = W = 2p + 4
]


@pytest.mark.parametrize("case", FOLD_CASES, ids=[f"c{c[1]}_h{c[2]}_k{c[4]}_s{c[5]}" for c in FOLD_CASES])
def test_reflect_dgrad_epilogue_fold_matches_pad_fold(case, monkeypatch):
    """The epilogue fold (interior pixels stored gated by the dgrad, frame mirrored by fold_band)
    equals the padded-grid dgrad + pad_fold pass: bitwise off the bands, within one bf16
    rounding on them (there the interior value is rounded before the frame adds in)."""
    from p2p_pytorch_amd.ops import hip
    N, Cin, H, W, k, s, act_in = case
    x = rand_img(N, Cin, H, W, seed=21)
    w = torch.randn(Cin * 2, Cin, k, k, device=DEV) * (1.0 / (Cin * k * k) ** 0.5)

    p = k // 2
    gy = rand_img(N, 2 * Cin, (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1, seed=22)

    def dgrad(fold_epi):
        monkeypatch.setattr(hip, "_FOLD_EPI", fold_epi)
        hx = _leaf(x)
        ops.conv2d(hx, w, None, s, p, pad_mode="reflect", act_in=act_in).backward(gy)
        return hx.grad.float()

    ge, gl = dgrad(True), dgrad(False)
    band = torch.zeros(H, W, dtype=torch.bool, device=DEV)
    for r in list(range(1, p + 1)) + list(range(H - 1 - p, H - 1)):
        band[r, :] = True
    for c in list(range(1, p + 1)) + list(range(W - 1 - p, W - 1)):
        band[:, c] = True
    off = ~band
    assert torch.equal(ge[:, :, off], gl[:, :, off])
    tol = 2.0 ** -7 * gl.abs().max().item()
    assert (ge - gl).abs().max().item() <= tol
    rx = _leaf(x.float())
    ref.conv2d(rx, w.to(torch.bfloat16).float(), None, s, p, pad_mode="reflect",
               act_in=act_in).backward(gy.float())
    assert rel_err(ge, rx.grad) < 3e-2


UPFOLD_CASES = [
    # (N, Cin, Cout, H, W, act_in): G.deconv3 / deconv2 (nearest x2 + reflect 1 + 3x3)
    (2, 128, 64, 16, 16, None),
    (2, 64, 32, 12, 20, "relu"),
    (1, 32, 64, 5, 7, None),
]


@pytest.mark.parametrize("case", UPFOLD_CASES, ids=[f"c{c[1]}o{c[2]}_h{c[3]}w{c[4]}" for c in UPFOLD_CASES])
def test_up2_reflect_dgrad_as_strided_conv(case, monkeypatch):
    """The nearest-x2 + reflect-1 3x3 conv's input gradient as ONE 4x4 stride-2 conv over dY
    (phase-summed taps, edge-replicate fold in the epilogue) against the fp32 oracle and the
    upsampled-grid dgrad + pad_fold path."""
    from p2p_pytorch_amd.ops import hip
    N, Cin, Cout, H, W, act_in = case
    x = rand_img(N, Cin, H, W, seed=31)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV) * (1.0 / (Cin * 9) ** 0.5)
    gy = rand_img(N, Cout, 2 * H, 2 * W, seed=32)

    def dgrad(up_fold):
        monkeypatch.setattr(hip, "_UP_FOLD", up_fold)
        hx = _leaf(x)
        ops.conv2d(hx, w, None, 1, 1, pad_mode="reflect", upsample=2, act_in=act_in).backward(gy)
        return hx.grad.float()

    gf, gp = dgrad(True), dgrad(False)
    rx = _leaf(x.float())
    ref.conv2d(rx, w.to(torch.bfloat16).float(), None, 1, 1, pad_mode="reflect", upsample=2,
               act_in=act_in).backward(gy.float())
    assert rel_err(gf, rx.grad) < 3e-2
    assert rel_err(gf, gp) < 3e-2


def test_conv_wgrad_large_m():
    # many pixels per weight -> many split-K slabs; checks the deterministic slab reduce
    x = rand_img(8, 64, 64, 64, seed=8)
    w = torch.randn(128, 64, 4, 4, device=DEV) * 0.02
    hw = _leaf(w)
    y = ops.conv2d(x, hw, None, 2, 1, act_in="lrelu")
    gy = rand_img(*y.shape, seed=9)
    y.backward(gy)
    g1 = hw.grad.clone()
    hw.grad = None
    y = ops.conv2d(x, hw, None, 2, 1, act_in="lrelu")
    y.backward(gy)
    assert torch.equal(g1, hw.grad), "wgrad must be bitwise reproducible"
    rw = _leaf(w)
    ry = ref.conv2d(x.float(), rw.to(torch.bfloat16).float(), None, 2, 1, act_in="lrelu")
    ry.backward(gy.float())
    assert rel_err(hw.grad, rw.grad) < 2e-2


# (N, Cin, Cout, H, k, pad_mode): family-R residual 3x3 (reflect, tens of splits), the U-Net
# 4x4 s1-equivalent shape, a 9x9 head (T = 81 taps, the LDS tile's limit), odd channel count
@pytest.mark.parametrize("N,Cin,Cout,H,k,pad_mode", [(16, 128, 128, 64, 3, "reflect"),
                                                     (8, 64, 128, 64, 4, "zeros"),
                                                     (4, 32, 32, 128, 9, "reflect"),
                                                     (16, 40, 24, 32, 3, "zeros")])
def test_wgrad_split_reduce_kernels_bitwise(N, Cin, Cout, H, k, pad_mode):
    """The coalesced split-K reduce (per-thread split walk in a fixed order, G partial sums):
    two runs give bitwise equal weight gradients, both within bf16 tolerance of the fp32
    oracle.  (The round-4 scattered-store kernel it was A/B-ed against bitwise is gone with
    its P2P_WRED_OLD knob; it only remains for kernels with more than 81 taps.)"""
    x = rand_img(N, Cin, H, H, seed=21)
    w = torch.randn(Cout, Cin, k, k, device=DEV) * (1.0 / (Cin * k * k) ** 0.5)
    stride, pad = (1, k // 2) if k % 2 else (2, 1)

    def run():
        hw = _leaf(w)
        y = ops.conv2d(x, hw, None, stride, pad, pad_mode)
        y.backward(gy)
        return hw.grad

    with torch.no_grad():
        shape = ops.conv2d(x, w, None, stride, pad, pad_mode).shape
    gy = rand_img(*shape, seed=22)
    g_new = run()
    g_again = run()
    assert torch.equal(g_new, g_again), (g_new - g_again).abs().max().item()
    rw = _leaf(w)
    xr = F.pad(x.float(), (pad,) * 4, mode="reflect") if pad_mode == "reflect" else x.float()
    F.conv2d(xr, rw.to(torch.bfloat16).float(), None, stride,
             0 if pad_mode == "reflect" else pad).backward(gy.float())
    assert rel_err(g_new, rw.grad) < 2e-2


@pytest.mark.parametrize("N,C,H", [(2, 64, 32), (4, 512, 2), (2, 128, 64), (3, 256, 5)])
def test_instance_norm(N, C, H):
    x = rand_img(N, C, H, H, scale=3.0, seed=10)
    x = bf(x.float() + 2.0)  # non-zero mean
    hx = _leaf(x)
    y = ops.instance_norm(hx)
    gy = rand_img(N, C, H, H, seed=11)
    y.backward(gy)
    rx = _leaf(x.float())
    ry = F.instance_norm(rx, eps=1e-5)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 2e-2
    if H * H > 1:
        assert rel_err(hx.grad, rx.grad) < 3e-2


@pytest.mark.parametrize("act", ["lrelu", "relu"])
def test_conv_instance_norm_act_chain(act):
    """conv(+bias) -> IN with fused act: the act' gate and the conv bias gradient are fused
    into the norm backward (bias grad handed to the conv through the colsum stash)."""
    x = rand_img(2, 64, 16, 16, seed=20)
    w = torch.randn(128, 64, 4, 4, device=DEV) * 0.03
    b = torch.randn(128, device=DEV) * 0.1
    hx, hw, hb = _leaf(x), _leaf(w), _leaf(b)
    y = ops.instance_norm(ops.conv2d(hx, hw, hb, 2, 1), act=act)
    gy = rand_img(*y.shape, seed=21)
    y.backward(gy)
    rx, rw, rb = _leaf(x.float()), _leaf(w), _leaf(b)
    # the HIP path stores the conv output in bf16 before the norm: round the oracle's conv
    # output the same way (straight-through), so both evaluate the ReLU gate on the same
    # pre-activation instead of flipping gates within bf16 rounding of 0
    rc = ref.conv2d(rx, rw.to(torch.bfloat16).float(), rb, 2, 1)
    rc = rc + (rc.to(torch.bfloat16).float() - rc).detach()
    ry = ref.apply_act(F.instance_norm(rc), act)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 3e-2
    assert rel_err(hx.grad, rx.grad) < 4e-2
    assert rel_err(hw.grad, rw.grad) < 4e-2
    # bias before an instance norm has an exactly-zero true gradient (sum_p dx_norm = 0):
    # the HIP path returns that exact zero; fp32 autograd returns rounding noise around it
    assert torch.count_nonzero(hb.grad) == 0
    assert rb.grad.abs().max() < 1e-3


def test_batch_norm_train_and_eval():
    N, C, H = 4, 64, 16
    x = bf(torch.randn(N, C, H, H, device=DEV) * 2 + 1)
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV) * 0.1
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm2, rv2 = rm.clone(), rv.clone()
    hx, hg, hb = _leaf(x), _leaf(g), _leaf(b)
    y = ops.batch_norm(hx, rm, rv, hg, hb, True, 0.1, 1e-5)
    gy = rand_img(N, C, H, H, seed=12)
    y.backward(gy)
    rx, rg, rb = _leaf(x.float()), _leaf(g), _leaf(b)
    ry = F.batch_norm(rx, rm2, rv2, rg, rb, True, 0.1, 1e-5)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 2e-2
    assert rel_err(hx.grad, rx.grad) < 3e-2
    assert rel_err(hg.grad, rg.grad) < 2e-2
    assert rel_err(hb.grad, rb.grad) < 2e-2
    assert rel_err(rm, rm2) < 1e-3 and rel_err(rv, rv2) < 1e-3
    ye = ops.batch_norm(x, rm, rv, g, b, False, 0.1, 1e-5)
    rye = F.batch_norm(x.float(), rm2, rv2, g, b, False, 0.1, 1e-5)
    assert rel_err(ye, rye) < 2e-2


@pytest.mark.parametrize("act", [None, "lrelu", "prelu"])
def test_batch_norm_eval_backward(act):
    """Eval-mode (frozen running statistics) BN backward on the HIP norm passes: dx =
    rstd * gamma * gate(dy), d(gamma), d(beta) and the shared PReLU slope gradient."""
    N, C, H = 4, 64, 16
    x = bf(torch.randn(N, C, H, H, device=DEV) * 2 + 0.5)
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV) * 0.3
    rm = torch.randn(C, device=DEV) * 0.5
    rv = torch.rand(C, device=DEV) + 0.5
    w = torch.full((1,), 0.25, device=DEV)
    hx, hg, hb, hw = _leaf(x), _leaf(g), _leaf(b), _leaf(w)
    kw = {"prelu_weight": hw} if act == "prelu" else ({"act": act} if act else {})
    y = ops.batch_norm(hx, rm.clone(), rv.clone(), hg, hb, False, 0.1, 1e-5, **kw)
    gy = rand_img(N, C, H, H, seed=41)
    y.backward(gy)
    rx, rg, rb, rw = _leaf(x.float()), _leaf(g), _leaf(b), _leaf(w)
    ry = F.batch_norm(rx, rm.clone(), rv.clone(), rg, rb, False, 0.1, 1e-5)
    if act == "prelu":
        ry = F.prelu(ry, rw)
    elif act == "lrelu":
        ry = F.leaky_relu(ry, 0.2)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 2e-2
    assert rel_err(hx.grad, rx.grad) < 2e-2
    assert rel_err(hg.grad, rg.grad) < 2e-2 and rel_err(hb.grad, rb.grad) < 2e-2
    if act == "prelu":
        assert rel_err(hw.grad, rw.grad) < 1e-2


@pytest.mark.parametrize("act,training", [("relu", True), ("lrelu", True), ("relu", False)])
def test_batch_norm_residual_join(act, training):
    """y = act(BN(x) + r) in the BN apply pass (family-R residual join): output, dx, dr,
    d(gamma), d(beta) and the running statistics vs fp32 F.batch_norm + add + act; the
    deferred form parks dr for the conv reading r (skip_grad="take"), which adds it."""
    from p2p_pytorch_amd.ops import hip
    N, C, H = 4, 128, 16
    x = bf(torch.randn(N, C, H, H, device=DEV) * 2 + 0.3)
    r = bf(torch.randn(N, C, H, H, device=DEV))
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV) * 0.3
    rm, rv = torch.randn(C, device=DEV) * 0.2, torch.rand(C, device=DEV) + 0.5
    gy = rand_img(N, C, H, H, seed=51)
    hx, hr, hg, hb = _leaf(x), _leaf(r), _leaf(g), _leaf(b)
    hrm, hrv = rm.clone(), rv.clone()
    y = ops.batch_norm(hx, hrm, hrv, hg, hb, training, 0.1, 1e-5, act=act, residual=hr)
    y.backward(gy)
    rx, rr, rg, rb = _leaf(x.float()), _leaf(r.float()), _leaf(g), _leaf(b)
    rrm, rrv = rm.clone(), rv.clone()
    z = F.batch_norm(rx, rrm, rrv, rg, rb, training, 0.1, 1e-5) + rr
    ry = F.relu(z) if act == "relu" else F.leaky_relu(z, 0.2)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 2e-2
    assert rel_err(hx.grad, rx.grad) < 3e-2
    assert rel_err(hr.grad, rr.grad) < 1e-2
    assert rel_err(hg.grad, rg.grad) < 2e-2 and rel_err(hb.grad, rb.grad) < 2e-2
    if training:
        assert rel_err(hrm, rrm) < 1e-3 and rel_err(hrv, rrv) < 1e-3
    # deferred: the residual's gradient is parked under r's storage for its other consumer
    hx2, hr2 = _leaf(x), _leaf(r)
    y2 = ops.batch_norm(hx2, rm.clone(), rv.clone(), g, b, training, 0.1, 1e-5, act=act,
                        residual=hr2, defer_residual=True)
    y2.backward(gy)
    assert hr2.grad is None
    parked = hip._DEFERRED.pop(hr2.data_ptr())
    hip.assert_no_deferred()
    assert torch.equal(parked, hr.grad)
    assert torch.equal(hx2.grad, hx.grad)


@pytest.mark.parametrize("C", [32, 64, 3])
def test_batch_norm_fused_prelu(C):
    """BN + shared-slope PReLU in one apply pass; backward gate and slope gradient reduced in
    the norm's partial-sum pass (family R's G / C sites) vs fp32 F.batch_norm + F.prelu."""
    N, H = 4, 16
    x = bf(torch.randn(N, C, H, H, device=DEV) * 2 + 0.3)
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV) * 0.3
    w = torch.full((1,), 0.25, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    hx, hg, hb, hw = _leaf(x), _leaf(g), _leaf(b), _leaf(w)
    y = ops.batch_norm(hx, rm.clone(), rv.clone(), hg, hb, True, 0.1, 1e-5, prelu_weight=hw)
    gy = rand_img(N, C, H, H, seed=31)
    y.backward(gy)
    rx, rg, rb, rw = _leaf(x.float()), _leaf(g), _leaf(b), _leaf(w)
    ry = F.prelu(F.batch_norm(rx, rm.clone(), rv.clone(), rg, rb, True, 0.1, 1e-5), rw)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 2e-2
    assert rel_err(hx.grad, rx.grad) < 3e-2
    assert rel_err(hg.grad, rg.grad) < 2e-2 and rel_err(hb.grad, rb.grad) < 2e-2
    assert rel_err(hw.grad, rw.grad) < 1e-2


@pytest.mark.parametrize("name", ["relu", "lrelu", "tanh", "sigmoid"])
def test_act(name):
    x = rand_img(2, 16, 8, 8, seed=13)
    hx = _leaf(x)
    y = ops.act(hx, name)
    gy = rand_img(2, 16, 8, 8, seed=14)
    y.backward(gy)
    rx = _leaf(x.float())
    ry = ref.apply_act(rx, name)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 1e-2
    assert rel_err(hx.grad, rx.grad) < 2e-2


@pytest.mark.parametrize("name", ["relu", "lrelu"])
def test_add_act(name):
    """act(a + b) fused (residual joins of family R) vs fp32; grads reach both inputs."""
    a, b = rand_img(2, 32, 8, 8, seed=21), rand_img(2, 32, 8, 8, seed=22)
    ha, hb = _leaf(a), _leaf(b)
    y = ops.add_act(ha, hb, name)
    gy = rand_img(2, 32, 8, 8, seed=23)
    y.backward(gy)
    ra, rb = _leaf(a.float()), _leaf(b.float())
    ry = ref.apply_act(ra + rb, name)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 1e-2
    assert rel_err(ha.grad, ra.grad) < 2e-2 and rel_err(hb.grad, rb.grad) < 2e-2


def test_dropout_mask_and_grad():
    from p2p_pytorch_amd.ops import hip
    x = bf(torch.ones(4, 64, 16, 16, device=DEV))
    hx = _leaf(x)
    y = hip.dropout(hx, 0.5, salt=7)
    frac = (y.float() == 0).float().mean().item()
    assert 0.45 < frac < 0.55
    assert torch.all((y.float() == 0) | (y.float() == 2.0))
    y.backward(torch.ones_like(y))
    assert torch.equal(hx.grad.float(), y.float()), "backward must reuse the forward mask"
    y2 = hip.dropout(x, 0.5, salt=7)
    assert torch.equal(y, y2)
    hip.advance_rng()
    y3 = hip.dropout(x, 0.5, salt=7)
    assert not torch.equal(y, y3), "advance_rng must draw a new mask"


@pytest.mark.parametrize("shape", [(4, 1, 30, 30), (3, 1, 7, 9), (64, 64, 32, 32)])
@pytest.mark.parametrize("kind", ["bce_logits", "mse", "l1", "mse_pair", "bce"])
def test_losses(kind, shape):
    """vectorised (16-B) loss kernels incl. a numel % 8 tail and a multi-block reduction"""
    a = rand_img(*shape, seed=15)
    b = rand_img(*shape, seed=16)
    ha = _leaf(a)
    ra = _leaf(a.float())
    if kind == "bce_logits":
        v, r = ops.bce_logits_const(ha, 1.0), ref.bce_logits_const(ra, 1.0)
    elif kind == "mse":
        v, r = ops.mse_const(ha, 0.0), ref.mse_const(ra, 0.0)
    elif kind == "l1":
        v, r = ops.l1(ha, b), ref.l1(ra, b.float())
    elif kind == "mse_pair":
        v, r = ops.mse(ha, b), ref.mse(ra, b.float())
    else:
        ha2 = _leaf(bf(torch.sigmoid(a.float())))
        ra2 = _leaf(ha2.detach().float())
        v, r = ops.bce_const(ha2, 0.0), ref.bce_const(ra2, 0.0)
        ha, ra = ha2, ra2
    assert v.dtype == torch.float32 and v.dim() == 0
    assert abs(v.item() - r.item()) <= 1e-3 * max(1.0, abs(r.item()))
    (v * 3.0).backward()
    (r * 3.0).backward()
    assert rel_err(ha.grad, ra.grad) < 2e-2


def test_weight_prep_multi_matches_single():
    """Multi-tensor weight cast (one launch) == per-tensor cast == bf16(permuted fp32)."""
    P = torch.ops.p2p
    torch.manual_seed(0)
    shapes = [(64, 3, 4, 4), (128, 64, 4, 4), (6, 512, 4, 4), (64, 64, 3, 3), (3, 64, 7, 7),
              (512, 256, 1, 1)]
    ws, sw, xp, yp, refs = [], [], [], [], []
    for (a, b, kh, kw) in shapes:
        w = torch.randn(a, b, kh, kw, device=DEV)
        for swap in (0, 1):
            X, Y = (b, a) if swap else (a, b)
            Xp, Yp = (X + 7) // 8 * 8 + (8 if swap else 0), (Y + 7) // 8 * 8
            ws.append(w)
            sw.append(swap)
            xp.append(Xp)
            yp.append(Yp)
            img = torch.zeros(Xp, kh, kw, Yp, device=DEV)
            src = w.permute(1, 2, 3, 0) if swap else w.permute(0, 2, 3, 1)
            img[:X, :, :, :Y] = src
            refs.append(img.to(torch.bfloat16))
    outs = P.weight_prep_multi(ws, sw, xp, yp)
    for o, r, w, s_, x_, y_ in zip(outs, refs, ws, sw, xp, yp):
        assert torch.equal(o, r)
        assert torch.equal(P.weight_prep(w, s_, x_, y_, None), r)
    # one-pass pair form (T <= 16): both images of each weight
    sel = [i for i in range(0, len(ws), 2) if ws[i].shape[2] * ws[i].shape[3] <= 16]
    pairs = P.weight_prep_pairs([ws[i] for i in sel], [xp[i] for i in sel], [yp[i] for i in sel])
    for j, i in enumerate(sel):
        assert torch.equal(pairs[2 * j], refs[i])
        # image 1 of the pair has exactly the X/Y extents of image 0 swapped
        r1 = torch.zeros(yp[i], *ws[i].shape[2:], xp[i], device=DEV)
        r1[:ws[i].shape[1], :, :, :ws[i].shape[0]] = ws[i].permute(1, 2, 3, 0)
        assert torch.equal(pairs[2 * j + 1], r1.to(torch.bfloat16))


def test_fused_adam_matches_torch():
    from p2p_pytorch_amd.engine.optim import FusedAdam
    torch.manual_seed(0)
    ps = [torch.randn(n, device=DEV) for n in (7, 4096, 10000, 64 * 3 * 4 * 4)]
    qs = [p.clone() for p in ps]
    ps = [torch.nn.Parameter(p) for p in ps]
    qs = [torch.nn.Parameter(q) for q in qs]
    o1 = FusedAdam(ps, lr=2e-4, betas=(0.5, 0.999))
    o2 = torch.optim.Adam(qs, lr=2e-4, betas=(0.5, 0.999))
    for it in range(5):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad = g.clone()
            q.grad = g.clone()
        o1.step()
        o2.step()
    for p, q in zip(ps, qs):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-6)


def test_unet_patchgan_step_matches_oracle():
    """Small U-Net + PatchGAN forward/backward: HIP bf16 path vs the fp32 PyTorch oracle.

    bf16 error compounds through a deep U-Net (instance norms over 2x2 maps amplify it),
    so the bound is relative to stock PyTorch bf16 autocast on the same inputs: the HIP
    path must be no less accurate than the eager bf16 baseline, per parameter.
    """
    from p2p_pytorch_amd.models import define_D, define_G
    torch.manual_seed(0)
    G = define_G(netG="unet_64", gpu_id=DEV, verbose=False, use_dropout=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=DEV, verbose=False)
    A = bf(torch.rand(2, 3, 64, 64, device=DEV) * 2 - 1)
    B = bf(torch.rand(2, 3, 64, 64, device=DEV) * 2 - 1)

    def run(backend, dtype=None):
        _native.set_backend(backend)
        G.zero_grad(set_to_none=True)
        D.zero_grad(set_to_none=True)
        try:
            ctx = torch.autocast("cuda", dtype) if dtype else torch.autocast("cuda", enabled=False)
            a, b = (A, B) if backend == "native" else (A.float(), B.float())
            with ctx:
                fake = G(a)
                pred = D((a, fake) if backend == "native" else torch.cat((a, fake.to(a.dtype)), 1))
                loss = ops.bce_logits_const(pred, 1.0) + 100 * ops.l1(fake, b)
            loss.backward()
        finally:
            _native.set_backend("native")
        grads = {n: p.grad.detach().float().clone() for n, p in G.named_parameters()}
        return loss.detach().float(), fake.detach().float(), grads

    l32, f32, g32 = run("torch")
    l16, f16, g16 = run("torch", torch.bfloat16)
    lh, fh, gh = run("native")
    assert rel_err(fh, f32) < 5e-2
    assert abs(lh.item() - l32.item()) < 2e-2 * abs(l32.item())
    worse, rows = [], []
    for n in g32:
        assert torch.isfinite(gh[n]).all(), n
        eh, ee = rel_err(gh[n], g32[n]), rel_err(g16[n], g32[n])
        rows.append((n, eh, ee))
        # measured worst (eh - 1.5 ee) = -0.002 over the 24 tensors (gpurun_out/bounds.jsonl)
        if eh > 1.5 * ee + 0.01:
            worse.append((n, eh, ee))
    _record("unet_patchgan_grads", rows)
    assert not worse, worse


@pytest.mark.parametrize("gate", [None, "lrelu"])
def test_skip_grad_fusion_op_level(gate):
    """A U-Net skip x read by the next encoder conv ("take") and the decoder ConvT's
    virtual concat ("defer", its backward runs first): x's ONE gradient write (ConvT's
    part parked, added in the encoder dgrad epilogue) vs the fp32 oracle's sum."""
    from p2p_pytorch_amd.ops import hip
    x = rand_img(2, 64, 16, 16, seed=31)
    w_e = torch.randn(128, 64, 4, 4, device=DEV) * (1.0 / (64 * 16) ** 0.5)
    w_i = torch.randn(128, 64, 4, 4, device=DEV) * (1.0 / (128 * 4) ** 0.5)
    w_o = torch.randn(128, 32, 4, 4, device=DEV) * (1.0 / (128 * 4) ** 0.5)
    gy = rand_img(2, 32, 32, 32, seed=32)

    def net(conv, convT, xx, we, wi, wo, fused):
        kw = {"skip_grad": "take", "grad_gate": gate} if fused else {}
        h = conv(xx, we, None, 2, 1, **kw)                       # encoder: 16 -> 8
        u = convT(h, wi, None, 2, 1, "relu")                      # inner decoder: 8 -> 16
        kw = {"skip_grad": "defer"} if fused else {}
        return convT((xx, u), wo, None, 2, 1, "relu", **kw)      # decoder on cat(skip, u)

    def hip_run(fused):
        hx = _leaf(x)
        hw = [_leaf(w) for w in (w_e, w_i, w_o)]
        y = net(ops.conv2d, ops.conv_transpose2d, hx, *hw, fused)
        y.backward(gy)
        hip.assert_no_deferred()
        return y, hx, hw

    y, hx, hw = hip_run(True)
    _, ux, uw = hip_run(False)   # unfused: autograd adds the two parts
    rx = _leaf(x.float())
    rw = [_leaf(w) for w in (w_e, w_i, w_o)]
    rb = [w.to(torch.bfloat16).float() for w in rw]
    ry = net(lambda xx, w, b, s, p, **k: ref.conv2d(xx, w, b, s, p),
             ref.conv_transpose2d, rx, *rb, False)
    # grad_gate: x is the stored lrelu(pre) of its producer and the gradient is w.r.t. pre
    ry.backward(gy.float())
    gref = rx.grad
    if gate == "lrelu":
        gref = gref * torch.where(x.float() > 0, 1.0, 0.2)
    if gate == "lrelu":   # unfused run has no gate: apply it the same way
        ux.grad = ux.grad * torch.where(x > 0, 1.0, 0.2).to(ux.grad.dtype)
    # three chained bf16 convs: judge the fused skip gradient against the unfused one's
    # distance from the fp32 oracle (the fusion may only reorder roundings)
    assert rel_err(y, ry) < 2e-2
    assert rel_err(hx.grad, gref) < 1.5 * rel_err(ux.grad, gref) + 1e-2
    for h, u, r in zip(hw, uw, rw):
        assert rel_err(h.grad, r.grad) < 1.5 * rel_err(u.grad, r.grad) + 1e-2


def test_unet_skip_grad_wiring():
    """Model level: every U-Net skip is wired defer/take, one backward consumes every
    parked gradient, and the gradients stay finite."""
    from p2p_pytorch_amd.models import define_G
    from p2p_pytorch_amd.ops import hip
    torch.manual_seed(0)
    G = define_G(netG="unet_128", gpu_id=DEV, verbose=False, use_dropout=False)
    convs = [m for m in G.modules() if hasattr(m, "skip_grad")]
    assert sum(m.skip_grad == "defer" for m in convs) == G.num_downs - 1
    assert sum(m.skip_grad == "take" for m in convs) == G.num_downs - 1
    A = bf(torch.rand(2, 3, 128, 128, device=DEV) * 2 - 1)
    G(A).float().square().mean().backward()
    hip.assert_no_deferred()
    for n, p in G.named_parameters():
        assert torch.isfinite(p.grad).all(), n


def test_pack_pairs_matches_cat_input():
    """The fused D batch packed in place (pack_pairs) is the same conv input as the
    batch-cat of the two (a, b) pairs: in deterministic mode (ordered split-K) the logits
    and every weight gradient are bitwise identical."""
    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd.models import define_D
    from p2p_pytorch_amd.ops import hip
    torch.manual_seed(0)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=DEV, verbose=False)
    a1, b1, a2, b2 = (bf(torch.rand(2, 3, 64, 64, device=DEV) * 2 - 1) for _ in range(4))

    def run(x):
        D.zero_grad(set_to_none=True)
        y = D(x)
        y.float().square().mean().backward()
        return y.detach().float(), {n: p.grad.detach().float().clone() for n, p in D.named_parameters()}

    p2p.set_deterministic(True)
    try:
        yp, gp = run(hip.pack_pairs([(a1, b1), (a2, b2)]))
        yc, gc = run((torch.cat((a1, a2)), torch.cat((b1, b2))))
    finally:
        p2p.set_deterministic(False)
    assert torch.equal(yp, yc)
    for n in gc:
        assert torch.equal(gp[n], gc[n]), (n, rel_err(gp[n], gc[n]))


# ---------------------------------------------------------------- family-R fringe ops
def _grad_pair(fn_h, fn_r, x, gy_seed=21):
    """HIP op on the GPU vs the same op in fp32 on the CPU (the oracle must not depend on
    the GPU library path: MIOpen's pooling backward is not the PyTorch definition)."""
    hx = _leaf(x)
    rx = _leaf(x.float().cpu())
    yh = fn_h(hx)
    yr = fn_r(rx)
    if yh.dim() == 0:
        yh.backward(torch.tensor(1.7, device=DEV))
        yr.backward(torch.tensor(1.7))
    else:
        gy = rand_img(*yh.shape, seed=gy_seed)
        yh.backward(gy)
        yr.backward(gy.float().cpu())
    return yh.cpu(), yr, hx.grad.cpu(), rx.grad


def test_prelu_shared_slope():
    x = rand_img(2, 32, 16, 16, seed=11)
    wh = torch.nn.Parameter(torch.tensor([0.25], device=DEV))
    wr = torch.nn.Parameter(torch.tensor([0.25]))
    yh, yr, gh, gr = _grad_pair(lambda t: ops.prelu(t, wh), lambda t: F.prelu(t, wr), x)
    assert rel_err(yh, yr) < 1e-2 and rel_err(gh, gr) < 1e-2
    assert abs(wh.grad.item() - wr.grad.item()) <= 2e-2 * abs(wr.grad.item()) + 1e-3
    assert wh.grad.shape == wh.shape


def test_tv_loss():
    x = rand_img(2, 3, 20, 24, seed=12)
    yh, yr, gh, gr = _grad_pair(ops.tv, ref.tv, x)
    assert abs(yh.item() - yr.item()) <= 1e-3 * abs(yr.item())
    assert rel_err(gh, gr) < 1e-2


def test_quantize_3bit():
    x = rand_img(2, 3, 16, 16, seed=13)
    y = ops.quantize(x, 3)
    r = ref.quantize(x.float(), 3)
    assert rel_err(y, r) < 1e-2


def test_quantize_unshuffle_feeds_the_head_conv():
    """The quantiser's second output is pixel_unshuffle(quantize(x), 2), channel-padded with
    zeros and tagged as a packed conv input; the expander's 9x9 head (nearest x2, reflect 4)
    reading it equals the same conv over the plain unshuffle (no unshuffle / pad pass)."""
    from p2p_pytorch_amd.ops import hip
    hip.begin_step()
    x = bf(torch.rand(2, 3, 64, 48, device=DEV))
    y = ops.quantize(x, 3, unshuffle=2)
    assert torch.equal(y.float(), ops.quantize(x, 3).float())
    u = ops.pixel_unshuffle(y, 2, conv_input=True)
    assert u.shape == (2, 16, 32, 24) and getattr(u, "_p2p_packed", None) == (12, 0)
    assert ops.pixel_unshuffle(y.detach(), 2, conv_input=True) is u   # G(compressed.detach())
    ru = F.pixel_unshuffle(y.float(), 2)
    assert torch.equal(u[:, :12].float(), ru) and not u[:, 12:].float().any()
    w = _leaf(torch.randn(32, 12, 9, 9, device=DEV) * 0.05)
    b = _leaf(torch.randn(32, device=DEV) * 0.1)
    z = ops.conv2d(u, w, b, 1, 4, "reflect", 2)
    plain = ops.pixel_unshuffle(y, 2)          # the unfused route (12 channels, pad pass)
    zr = ops.conv2d(plain, w, b, 1, 4, "reflect", 2)
    assert z.shape == zr.shape == (2, 32, 64, 48)
    assert torch.equal(z.float(), zr.float())
    hip.begin_step()
    assert ops.pixel_unshuffle(y, 2, conv_input=True).shape == (2, 12, 32, 24)   # stash per step


@pytest.mark.parametrize("C,H,W", [(3, 32, 32), (6, 33, 20), (8, 7, 9)])
def test_avg_pool3_s2(C, H, W):
    x = rand_img(2, C, H, W, seed=14)
    yh, yr, gh, gr = _grad_pair(ops.avg_pool3_s2, ref.avg_pool3_s2, x)
    assert yh.shape == yr.shape
    assert rel_err(yh, yr) < 1e-2 and rel_err(gh, gr) < 1e-2


HALO_CASES = [
    # (N, Cin, H, W, Cout, pad_mode, up, k): family R's full-resolution layers on the
    # halo-tile kernels (csrc/halo_kxk.hip forward / flipped-tap dgrad, halo_wgrad.hip)
    (2, 32, 40, 36, 3, "reflect", 1, 9),     # G.deconv1 (+ its dgrad: 8-ch gy, flipped taps)
    (2, 12, 20, 18, 32, "reflect", 2, 9),    # G.conv1 on the unshuffled image, nearest x2
    (2, 16, 33, 35, 16, "zeros", 1, 9),      # partial tiles, zero pad
    (2, 64, 20, 18, 32, "reflect", 2, 3),    # G.deconv2 (64 -> 32, x2), wgrad 3x3 / 64 ch
    (2, 3, 34, 30, 64, "zeros", 1, 3),       # VGG conv1_1: its 64 -> 8 dgrad (flipped taps)
]


@pytest.mark.parametrize("case", HALO_CASES)
def test_halo_k9_conv(case, monkeypatch):
    """Stride-1 conv forward + input / weight gradients on the halo paths vs fp32 (and vs
    the implicit-GEMM fallback, P2P_NO_HALO=1)."""
    N, C, H, W, Co, mode, up, k = case
    g = torch.Generator(device=DEV).manual_seed(3)
    x = rand_img(N, C, H, W, seed=41)
    w = (torch.randn(Co, C, k, k, device=DEV, generator=g) * (0.4 / k)).to(torch.bfloat16).float()
    b = torch.randn(Co, device=DEV, generator=g) * 0.1
    gy_shape = (N, Co, H * up, W * up)
    gy = rand_img(*gy_shape, seed=42)

    def run():
        hx, hw, hb = _leaf(x), _leaf(w), _leaf(b)
        y = ops.conv2d(hx, hw, hb, 1, k // 2, mode, up)
        y.backward(gy)
        return y.float(), hx.grad.float(), hw.grad.float(), hb.grad.float()

    yh, gxh, gwh, gbh = run()
    monkeypatch.setenv("P2P_NO_HALO", "1")
    yf, gxf, gwf, gbf = run()
    monkeypatch.delenv("P2P_NO_HALO")
    rx, rw, rb = _leaf(x.float()), _leaf(w), _leaf(b)
    ry = ref.conv2d(rx, rw, rb, 1, k // 2, mode, up)
    ry.backward(gy.float())
    assert yh.shape == ry.shape
    assert rel_err(yh, ry) < 1e-2, rel_err(yh, ry)
    assert rel_err(yh, yf) < 1e-2
    assert rel_err(gxh, rx.grad) < 2e-2 and rel_err(gxh, gxf) < 2e-2
    assert rel_err(gwh, rw.grad) < 2e-2 and rel_err(gbh, rb.grad) < 2e-2


@pytest.mark.parametrize("shape", [(2, 64, 16, 16), (2, 12, 9, 7)])
def test_max_pool2_ties_route_to_first(shape):
    # 64 ch: 8-channel vector kernels; 12 ch / odd sizes: the scalar fallback
    x = bf(torch.relu(torch.randn(*shape, device=DEV)))  # many exact-zero ties
    yh, yr, gh, gr = _grad_pair(ops.max_pool2, lambda t: F.max_pool2d(t, 2, 2), x)
    assert torch.equal(yh.float(), yr)
    assert rel_err(gh, gr) < 1e-2
    assert torch.equal(gh != 0, gr != 0)


def test_l2_normalize_channels():
    x = rand_img(2, 12, 16, 16, seed=15)
    yh, yr, gh, gr = _grad_pair(ops.l2_normalize_channels, ref.l2_normalize_channels, x)
    assert rel_err(yh, yr) < 1e-2 and rel_err(gh, gr) < 2e-2


def test_l2_normalize_channels_residual():
    x, r0 = rand_img(2, 3, 16, 16, seed=24), rand_img(2, 3, 16, 16, seed=25)
    hx, hr = _leaf(x), _leaf(r0)
    y = ops.l2_normalize_channels(hx, residual=hr)
    gy = rand_img(2, 3, 16, 16, seed=26)
    y.backward(gy)
    rx, rr = _leaf(x.float()), _leaf(r0.float())
    ry = ref.l2_normalize_channels(rx) + rr
    ry.backward(gy.float())
    assert rel_err(y, ry) < 1e-2
    assert rel_err(hx.grad, rx.grad) < 2e-2 and rel_err(hr.grad, rr.grad) < 1e-2


@pytest.mark.parametrize("shape", [(2, 12, 16, 16), (3, 12, 9, 7), (2, 48, 8, 4)])
def test_l2_normalize_pixel_shuffle_fused(shape):
    """CompressionNetwork tail: PixelShuffle(2) -> l2-normalise + residual in ONE pass (the
    shuffle is the kernel's addressing; its backward writes the un-shuffled gradient) against
    the fp32 oracle F.pixel_shuffle -> normalize -> + res."""
    n, c, h, w = shape
    x, r0 = rand_img(*shape, seed=27), rand_img(n, c // 4, 2 * h, 2 * w, seed=28)
    hx, hr = _leaf(x), _leaf(r0)
    y = ops.l2_normalize_channels(hx, residual=hr, shuffle=2)
    gy = rand_img(n, c // 4, 2 * h, 2 * w, seed=29)
    y.backward(gy)
    rx, rr = _leaf(x.float()), _leaf(r0.float())
    ry = ref.l2_normalize_channels(F.pixel_shuffle(rx, 2)) + rr
    ry.backward(gy.float())
    assert y.shape == ry.shape
    assert rel_err(y, ry) < 1e-2
    assert rel_err(hx.grad, rx.grad) < 2e-2 and rel_err(hr.grad, rr.grad) < 1e-2


@pytest.mark.parametrize("r", [2])
def test_pixel_shuffle_roundtrip(r):
    x = rand_img(2, 12, 8, 6, seed=16)
    yh, yr, gh, gr = _grad_pair(lambda t: ops.pixel_shuffle(t, r),
                                lambda t: F.pixel_shuffle(t, r), x)
    assert torch.equal(yh.float(), yr) and torch.equal(gh.float(), gr)
    x = rand_img(2, 3, 8, 6, seed=17)
    yh, yr, gh, gr = _grad_pair(lambda t: ops.pixel_unshuffle(t, r),
                                lambda t: F.pixel_unshuffle(t, r), x)
    assert torch.equal(yh.float(), yr) and torch.equal(gh.float(), gr)


def test_family_r_networks_match_oracle():
    """Compression network C + ExpandNetwork G + multiscale SN PatchGAN forward/backward on
    the HIP path vs the fp32 oracle (bound relative to eager bf16 autocast, per parameter)."""
    from p2p_pytorch_amd.models.factory import define_C, define_D, define_G
    torch.manual_seed(0)
    C = define_C(gpu_id=DEV, verbose=False)
    G = define_G(gpu_id=DEV, verbose=False)
    D = define_D(6, 64, gpu_id=DEV, verbose=False)
    # 4 x 64^2: the residual trunk normalises over 4*16*16 = 1024 samples per channel (at
    # 2 x 32^2 it was 128 and the bf16 eager error of the early BN affines was already 40-50 %)
    B = bf(torch.rand(4, 3, 64, 64, device=DEV) * 2 - 1)

    def run(backend, dtype=None):
        _native.set_backend(backend)
        for m in (C, G, D):
            m.zero_grad(set_to_none=True)
        try:
            ctx = torch.autocast("cuda", dtype) if dtype else torch.autocast("cuda", enabled=False)
            b = B if backend == "native" else B.float()
            with ctx:
                comp = C(b)
                fake = G(comp)
                pred = D(torch.cat((comp, fake.to(comp.dtype)), 1))
                loss = sum(ops.mse_const(p[-1], 1.0) for p in pred) + 10 * ops.l1(fake, b) + \
                    ops.tv(fake)
            loss.backward()
        finally:
            _native.set_backend("native")
        grads = {n: p.grad.detach().float().clone() for n, p in G.named_parameters()
                 if p.grad is not None}
        return loss.detach().float(), fake.detach().float(), grads

    l32, f32, g32 = run("torch")
    l16, f16, g16 = run("torch", torch.bfloat16)
    lh, fh, gh = run("native")
    assert torch.isfinite(lh) and abs(lh.item() - l32.item()) < 5e-2 * abs(l32.item())
    assert rel_err(fh, f32) < 1.5 * rel_err(f16, f32) + 0.05
    # biases of convs feeding a batch norm have a true gradient of exactly 0 (sum of a
    # normalised group's dx): relative error is meaningless there, so an absolute floor
    # scaled to the network's gradients applies as well
    gscale = max(g.abs().max().item() for g in g32.values())
    worse, rows = [], []
    for n in g32:
        assert torch.isfinite(gh[n]).all(), n
        eh, ee = rel_err(gh[n], g32[n]), rel_err(g16[n], g32[n])
        rows.append((n, eh, ee, (gh[n] - g32[n]).abs().max().item() / gscale))
        # the 9-block BN trunk is ill-conditioned: eager bf16 alone is 30-50 % off on the early
        # BN affines and the error moves +-50 % run to run (atomic-order nondeterminism in both
        # stacks).  Measured over 11 repeats: per-tensor eh / ee up to 2.47 (in1_d.bias, eh - ee
        # <= 0.24), median 0.89-1.03 (native is as accurate as eager).  A wrong kernel shows up
        # as eh ~ 1; so per tensor max(2.5x eager, eager + 0.3), and the median <= 1.25
        # (3-element tensors -- the output BN(3) affine -- are sums that nearly cancel: their
        # error is the bf16 storage noise of the whole image, bound by ee + 0.5 only)
        slack = 0.5 if g32[n].numel() <= 4 else 0.3
        if eh > max(2.5 * ee, ee + slack) + 0.02 and (gh[n] - g32[n]).abs().max().item() > 1e-3 * gscale:
            worse.append((n, eh, ee))
    _record("family_r_grads", rows)
    assert not worse, worse
    ratios = sorted(eh / max(ee, 1e-3) for _, eh, ee, _ in rows)
    assert ratios[len(ratios) // 2] <= 1.25, ratios[len(ratios) // 2]


@pytest.mark.parametrize("kind,N,C,H,Cout", [("conv", 16, 64, 128, 128), ("convT", 16, 128, 32, 256),
                                             ("conv_s1", 2, 256, 17, 512)])
@pytest.mark.parametrize("norm", ["instance", "batch"])
def test_conv_epilogue_norm_stats(kind, N, C, H, Cout, norm):
    """Norm statistics emitted by the conv epilogue == the norm's own statistics pass."""
    from p2p_pytorch_amd.ops import hip
    x = rand_img(N, C, H, H, seed=31)
    if kind == "convT":
        w = torch.randn(C, Cout, 4, 4, device=DEV) * 0.05
        f = lambda st: ops.conv_transpose2d(x, w, None, 2, 1, "relu", None, stats=st)  # noqa: E731
    else:
        w = torch.randn(Cout, C, 4, 4, device=DEV) * 0.05
        s = 1 if kind == "conv_s1" else 2
        f = lambda st: ops.conv2d(x, w, None, s, 1, stats=st)  # noqa: E731
    outs = []
    for st in (False, True):
        hip.begin_step()
        y = f(st)
        if st and kind != "conv_s1":
            assert len(hip._stats_stash) == 1, "epilogue statistics expected for this shape"
        if norm == "instance":
            z = ops.instance_norm(y, act="lrelu")
        else:
            rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
            z = ops.batch_norm(y, rm, rv, torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV),
                               True, act="relu")
        outs.append(z.float())
        assert not hip._stats_stash
    assert rel_err(outs[1], outs[0]) < 1e-2


@pytest.mark.parametrize("h,wd", [(128, 1024), (512, 4096), (3, 70)])
def test_spectral_norm_power_iteration(h, wd):
    """csrc/sn.hip vs the reference's power iteration (networks.py:537-549) in fp32."""
    from p2p_pytorch_amd.ops import hip
    g = torch.Generator(device=DEV).manual_seed(9)
    W = (torch.randn(h, wd, device=DEV, generator=g) * 0.05).requires_grad_(True)
    u0 = torch.randn(h, device=DEV, generator=g)
    v0 = torch.randn(wd, device=DEV, generator=g)
    u0, v0 = u0 / (u0.norm() + 1e-12), v0 / (v0.norm() + 1e-12)
    u, v = u0.clone(), v0.clone()
    sig = hip.spectral_sigma(W, u, v, 1)
    (sig * 3.0).backward()
    # oracle
    vr = W.detach().t().mv(u0)
    vr = vr / (vr.norm() + 1e-12)
    ur = W.detach().mv(vr)
    ur = ur / (ur.norm() + 1e-12)
    sr = torch.dot(ur, W.detach().mv(vr))
    torch.cuda.synchronize()
    assert torch.allclose(v, vr, rtol=1e-4, atol=1e-6)
    assert torch.allclose(u, ur, rtol=1e-4, atol=1e-6)
    assert abs(sig.item() - sr.item()) <= 1e-5 * abs(sr.item())
    assert torch.allclose(W.grad, 3.0 * torch.outer(ur, vr), rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("dtype,cl,ref_compat,hw", [
    (torch.bfloat16, True, True, (37, 70)),
    (torch.float32, False, True, (256, 256)),
    (torch.float32, True, False, (7, 129)),
])
def test_image_metrics_kernel(dtype, cl, ref_compat, hw):
    """csrc/metrics.hip (one pass PSNR + SSIM) vs the float64 tensor oracle on the CPU."""
    from p2p_pytorch_amd.engine import metrics
    H, W = hw
    g = torch.Generator(device=DEV).manual_seed(11)
    a = torch.rand(3, 3, H, W, device=DEV, generator=g) * 2.2 - 1.1
    b = (a + 0.1 * torch.randn(3, 3, H, W, device=DEV, generator=g)).clamp(-1, 1)
    b[2] = a[2]                                  # identical image: PSNR inf, SSIM 1
    a, b = a.to(dtype), b.to(dtype)
    if cl:
        a = a.contiguous(memory_format=torch.channels_last)
    p, s = metrics.image_metrics(b, a, ref_compat)
    rp = metrics._psnr_torch(a.cpu(), b.cpu(), ref_compat)
    rs = metrics._ssim_torch(b.cpu(), a.cpu(), ref_compat)
    assert torch.isinf(p[2]) and torch.isinf(rp[2])
    assert torch.allclose(p[:2].cpu(), rp[:2], rtol=0, atol=1e-4), (p, rp)
    assert torch.allclose(s.cpu().double(), rs.double(), rtol=0, atol=1e-6), (s, rs)
    assert abs(s[2].item() - 1.0) < 1e-12


@pytest.mark.parametrize("cin,cout,k,s", [(64, 128, 4, 2), (256, 512, 4, 1)])
def test_spectral_norm_conv_epilogue_scale(cin, cout, k, s):
    """SpectralNorm conv with 1/sigma applied in the conv epilogues (SNConvFn, no W/sigma
    tensor) vs the reference formulation conv(x, w / sigma) in fp32: output, input gradient
    and the weight_bar gradient (both the direct and the sigma path)."""
    from p2p_pytorch_amd.models.compress_gan import SpectralNorm
    torch.manual_seed(5)
    conv = torch.nn.Conv2d(cin, cout, k, stride=s, padding=2)
    sn = SpectralNorm(conv).to(DEV)
    sn_ref = copy.deepcopy(sn)
    x = rand_img(2, cin, 18, 18, seed=51)
    hx = _leaf(x)
    y = sn(hx)
    gy = rand_img(*y.shape, seed=52)
    y.backward(gy)
    _native.set_backend("torch")
    try:
        rx = _leaf(x.float())
        ry = sn_ref(rx)
        ry.backward(gy.float())
    finally:
        _native.set_backend("native")
    assert y.shape == ry.shape
    assert rel_err(y, ry) < 2e-2
    assert rel_err(hx.grad, rx.grad) < 3e-2
    gw, rgw = sn.module.weight_bar.grad, sn_ref.module.weight_bar.grad
    assert rel_err(gw, rgw) < 3e-2, rel_err(gw, rgw)
    # u / v advanced identically (one power iteration each)
    assert torch.allclose(sn.module.weight_u, sn_ref.module.weight_u, rtol=1e-3, atol=1e-5)


def test_l1_gated_lrelu_gradient():
    """ops.l1(a, b, gate_a="lrelu"): value = mean|a - b|, grad_a = sign(a - b) * lrelu'(a) / n
    (the D features' LeakyReLU derivative carried by the feature-matching loss)."""
    a = rand_img(2, 64, 9, 7, seed=61)
    b = rand_img(2, 64, 9, 7, seed=62)
    ha = _leaf(a)
    v = ops.l1(ha, b, gate_a="lrelu")
    (v * 2.0).backward()
    af, bf_ = a.float(), b.float()
    ref_v = (af - bf_).abs().mean()
    ref_g = 2.0 * torch.sign(af - bf_) * torch.where(af > 0, 1.0, 0.2) / af.numel()
    assert abs(v.item() - ref_v.item()) <= 1e-3 * abs(ref_v.item())
    assert rel_err(ha.grad, ref_g) < 1e-2


def test_guard_flag_kernel():
    """The NaN / Inf guard on the HIP path: flag and counter from one kernel."""
    from p2p_pytorch_amd.utils.guards import nonfinite
    one, nan, inf = (torch.tensor(v, device=DEV) for v in (1.0, float("nan"), float("-inf")))
    cnt = torch.zeros((), device=DEV)
    assert float(nonfinite(one, one * 2, counter=cnt)) == 0.0 and float(cnt) == 0.0
    assert float(nonfinite(one, nan, counter=cnt)) == 1.0 and float(cnt) == 1.0
    assert float(nonfinite(inf, counter=cnt)) == 1.0 and float(cnt) == 2.0
    assert float(nonfinite(torch.tensor(3.0e38, device=DEV))) == 0.0


@pytest.mark.parametrize("R,C", [(5, 64), (3000, 136), (40000, 64)])
def test_rowsum_and_scalar_helpers(R, C):
    """The step-bookkeeping kernels (csrc/elementwise.hip small-tensor helpers): rowsum (the
    norm-partial column sums, both the one-pass and the split path) against an fp64 sum;
    lincomb / lincomb_ / lincomb_n / scale_n / i64_add_ against the arithmetic they replace."""
    P = _native.ops()
    g = torch.Generator(device=DEV).manual_seed(3)
    ws = torch.randn(R, C, device=DEV, generator=g)
    out = P.rowsum(ws)
    ref_ = ws.double().sum(0)
    assert torch.allclose(out.double(), ref_, rtol=1e-5, atol=1e-3 * (R ** 0.5) * 1e-2)
    assert torch.equal(out, P.rowsum(ws))        # fixed order: bitwise repeatable
    a = torch.randn(7, device=DEV, generator=g)
    b = torch.randn(7, device=DEV, generator=g)
    assert torch.allclose(P.lincomb(a, b, 0.5, -2.0, 1.0), 0.5 * a - 2.0 * b + 1.0)
    t = a.clone()
    P.lincomb_(t, b, 1.0, -1.0, 1.0)
    assert torch.allclose(t, a - b + 1.0)
    ts = [torch.randn((), device=DEV, generator=g) for _ in range(5)]
    ws5 = [0.5, 1.0, -3.0, 0.25, 2.0]
    assert torch.allclose(P.lincomb_n(ts, ws5), sum(w * x for w, x in zip(ws5, ts)))
    gs = P.scale_n(torch.tensor(1.5, device=DEV), ws5)
    assert torch.allclose(gs, 1.5 * torch.tensor(ws5, device=DEV))
    c = torch.tensor([41], dtype=torch.int64, device=DEV)
    P.i64_add_(c, 1)
    assert c.item() == 42


def test_bounds_counters_positive_control():
    """P2P_BOUNDS_ASSERT build (csrc/bounds.h): a deliberately out-of-range check is counted,
    reported with its site id and reset; the normal build reports the counters disabled."""
    scratch = torch.zeros(1, device=DEV, dtype=torch.int32)
    torch.ops.p2p.oob_counts(True)
    torch.ops.p2p.oob_selftest(scratch)
    on, count, site, idx, limit = torch.ops.p2p.oob_counts(True)
    if on:
        assert (count, site, idx, limit) == (1, 99, 1, 1)
        assert int(scratch.item()) == 0            # the access was skipped
        assert torch.ops.p2p.oob_counts(True)[1] == 0
    else:
        assert count == 0 and int(scratch.item()) == 1


@pytest.mark.parametrize("N,Cin,H", [(4, 512, 31), (3, 64, 17), (2, 256, 8)])
def test_logits_conv_input_gradient_kernel(N, Cin, H, monkeypatch):
    """The input gradient of a 4x4 stride-1 conv with ONE output channel (the PatchGAN logits,
    csrc/dgrad_c1.hip) against the fp32 oracle and against the implicit-GEMM route it replaces
    (P2P_C1_DGRAD=0, read per call); the profiler must show the kernel ran."""
    from torch.profiler import ProfilerActivity, profile
    x = rand_img(N, Cin, H, H, seed=41)
    g = torch.Generator(device=DEV).manual_seed(42)
    w = torch.randn(1, Cin, 4, 4, device=DEV, generator=g) * (1.0 / (Cin * 16) ** 0.5)
    b = torch.randn(1, device=DEV, generator=g) * 0.1

    def run():
        hx, hw, hb = _leaf(x), _leaf(w), _leaf(b)
        y = ops.conv2d(hx, hw, hb, 1, 1)
        gy = rand_img(*y.shape, seed=43)
        y.backward(gy)
        torch.cuda.synchronize()
        return hx.grad, hw.grad, gy

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        gx, gw, gy = run()
    assert any("dgrad_c1_kernel" in e.name for e in prof.events()), "dgrad_c1_kernel never ran"
    monkeypatch.setenv("P2P_C1_DGRAD", "0")
    gx0, gw0, _ = run()
    rx, rw = _leaf(x.float()), _leaf(w)
    F.conv2d(rx, rw.to(torch.bfloat16).float(), b, 1, 1).backward(gy.float())
    assert rel_err(gx, rx.grad) < 2e-2, rel_err(gx, rx.grad)
    assert rel_err(gx, gx0) < 1e-2, rel_err(gx, gx0)
    assert rel_err(gw, gw0) < 1e-3
