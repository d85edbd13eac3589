"""The 32x32x16-MFMA conv tiles (csrc/conv_fwd_m32.hip) against the fp32 oracle.

Each case forces a 256-row tile (``P2P_CONV_VARIANT=g5``: 256 x 256, ``g4``: 256 x 128) on
shapes whose GEMM M and N are NOT tile multiples, and covers every instantiation the
dispatcher routes there: conv forward (MODE 0), transposed-conv forward and stride-2 input
gradients (MODE 1 parity classes), the virtual concat of two inputs, reflect padding, the
EXT epilogue of a gated input gradient (act' from the saved input), bias + output
activation.  The HIP result must match an fp32 PyTorch conv on the same bf16 inputs, and
the profiler must show that ``conv_fwd_m32_kernel`` actually ran.  The same case with the
tiles switched off (``torch.ops.p2p.set_m32(0)``: the round-4 16x16x32 kernels) must agree
with it to bf16 rounding.
"""
import os

import pytest
import torch

from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_backend():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    yield


def bf(x):
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def rand_img(n, c, h, w, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return bf(torch.randn(n, c, h, w, device=DEV, generator=g))


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _leaf(x):
    return None if x is None else x.detach().clone().requires_grad_(True)


CASES = [
    # (name, variant, kind, N, C1, C2, H, Cout, k, s, p, pad_mode, act_in, act_out)
    # sized so that the forward and the input gradient both reach >= 256 tiles (smaller
    # grids take split-K, which stays on the 16x16 kernels)
    ("conv_s1_256x256", "g5", "conv", 8, 256, 0, 65, 320, 4, 1, 1, "zeros", None, "lrelu"),
    ("conv_s2_concat_256x256", "g5", "conv", 8, 128, 128, 128, 288, 4, 2, 1, "zeros", None, None),
    ("conv_s2_relu_gate_256x128", "g4", "conv", 8, 128, 64, 128, 192, 4, 2, 1, "zeros", "relu", None),
    ("conv_reflect3x3_256x128", "g4", "conv", 8, 128, 0, 64, 136, 3, 1, 1, "reflect", None, None),
    ("convT_concat_256x256", "g5", "convT", 16, 256, 256, 32, 200, 4, 2, 1, "zeros", None, None),
    ("convT_relu_256x128", "g4", "convT", 32, 256, 0, 32, 192, 4, 2, 1, "zeros", "relu", None),
    # weight gradients on the 256 x 256 32x32x16 tile (R, Kq multiples of 128, >= 256):
    # conv (R = Cout), transposed conv on a virtual concat (R = Cin halves of 256), reflect
    # 3x3 (Kq = 9 x 256), and a ReLU'd operand
    ("wgrad_conv_s2_r512", "g5", "conv", 32, 256, 0, 64, 512, 4, 2, 1, "zeros", None, None),
    ("wgrad_convT_concat", "g5", "convT", 16, 256, 256, 32, 256, 4, 2, 1, "zeros", None, None),
    ("wgrad_reflect3x3_r256", "g5", "conv", 32, 256, 0, 48, 256, 3, 1, 1, "reflect", None, None),
    ("wgrad_conv_relu_r256", "g5", "conv", 64, 256, 0, 64, 256, 4, 2, 1, "zeros", "relu", None),
    # the 128 x 256 weight-gradient tile (R = 128, round 6): family R's residual 3x3 and the
    # U-Net e2 / PatchGAN c2 shape (64 -> 128, 4x4 s2)
    ("wgrad_reflect3x3_r128", "g5", "conv", 32, 128, 0, 64, 128, 3, 1, 1, "reflect", None, None),
    ("wgrad_conv_s2_r128_c64", "g4", "conv", 32, 64, 0, 128, 128, 4, 2, 1, "zeros", None, None),
]
WGRAD_M32 = {c[0] for c in CASES if c[0].startswith("wgrad_")}


def _run(case, m32, extra_env=None):
    name, var, kind, N, C1, C2, H, Cout, k, s, p, pad_mode, act_in, act_out = case
    x1 = rand_img(N, C1, H, H, seed=1)
    x2 = rand_img(N, C2, H, H, seed=2) if C2 else None
    Cin = C1 + C2
    g = torch.Generator(device=DEV).manual_seed(3)
    if kind == "conv":
        w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) / (Cin * k * k) ** 0.5
    else:
        w = torch.randn(Cin, Cout, k, k, device=DEV, generator=g) / (Cin * 4) ** 0.5
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    hx1, hx2, hw, hb = _leaf(x1), _leaf(x2), _leaf(w), _leaf(b)
    xin = (hx1, hx2) if x2 is not None else hx1
    prev = torch.ops.p2p.set_m32(1 if m32 else 0)
    # the tile under test, and none of the special-geometry kernels that would take some of
    # these layers first (stride-2 halo kernel, 3x3 / 9x9 halo kernels)
    env = {"P2P_CONV_VARIANT": var, "P2P_NO_S2T": "1", "P2P_NO_HALO": "1", **(extra_env or {})}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            if kind == "conv":
                y = ops.conv2d(xin, hw, hb, s, p, pad_mode, 1, act_in=act_in, act_out=act_out)
            else:
                y = ops.conv_transpose2d(xin, hw, hb, s, p, act_in, act_out)
            gy = rand_img(*y.shape, seed=4)
            y.backward(gy)
            torch.cuda.synchronize()
    finally:
        torch.ops.p2p.set_m32(prev)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    names = [e.name for e in prof.events() if "conv_fwd_m32_kernel" in e.name]
    if name in WGRAD_M32 and m32:
        assert any("conv_wgrad_m32_kernel" in e.name for e in prof.events()), f"{name}: wgrad m32 never ran"
    return (y, hx1.grad, None if x2 is None else hx2.grad, hw.grad, hb.grad), (x1, x2, w, b, gy), names


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_m32_conv_matches_fp32_oracle(case):
    name, var, kind, N, C1, C2, H, Cout, k, s, p, pad_mode, act_in, act_out = case
    (y, gx1, gx2, gw, gb), (x1, x2, w, b, gy), names = _run(case, True)
    assert names, f"{name}: conv_fwd_m32_kernel never ran"
    rx1, rx2, rw, rb = _leaf(x1.float()), _leaf(None if x2 is None else x2.float()), _leaf(w), _leaf(b)
    rin = (rx1, rx2) if rx2 is not None else rx1
    wq = rw.to(torch.bfloat16).float()   # the HIP path computes with bf16 weight images
    if kind == "conv":
        ry = ref.conv2d(rin, wq, rb, s, p, pad_mode, 1, act_in=act_in, act_out=act_out)
    else:
        ry = ref.conv_transpose2d(rin, wq, rb, s, p, act_in, act_out)
    ry.backward(gy.float())
    assert y.shape == ry.shape
    assert rel_err(y, ry) < 2e-2, (name, "y", rel_err(y, ry))
    assert rel_err(gx1, rx1.grad) < 3e-2, (name, "dx1", rel_err(gx1, rx1.grad))
    if x2 is not None:
        assert rel_err(gx2, rx2.grad) < 3e-2, (name, "dx2", rel_err(gx2, rx2.grad))
    assert rel_err(gw, rw.grad) < 3e-2, (name, "dw")
    assert rel_err(gb, rb.grad) < 3e-2, (name, "db")


AB_CASES = CASES[:3] + [c for c in CASES if c[0] in WGRAD_M32][:2] + [c for c in CASES if c[0].endswith("_r128")][:1]


@pytest.mark.parametrize("case", AB_CASES, ids=[c[0] for c in AB_CASES])
def test_m32_matches_16x16_tiles(case):
    out_a, _, names = _run(case, True)
    out_b, _, names_b = _run(case, False)
    assert names and not names_b
    for ta, tb in zip(out_a, out_b):
        if ta is not None:
            assert rel_err(ta, tb) < 1.5e-2


# The 512 x 128 tile (round 6): bf16 layers with 65-128 output channels whose parity classes
# are multiples of 512 pixels.  Pinned with P2P_M32_BM (read per call; the production route
# takes it from 1024 blocks up).  Cases: conv on a virtual concat with Cout not a tile multiple,
# a ReLU'd input whose input gradient carries the act' gate (EXT, MODE 1), and the ConvT with
# input ReLU (MODE 1 RELU) -- e2 / PatchGAN c2 / d-layer shapes at 32x32 and 64x64.
# (>= 256 tiles of 256 rows, as above: smaller grids take split-K)
CASES_512 = [
    ("conv_s2_concat_512x128", "g4", "conv", 16, 64, 64, 128, 96, 4, 2, 1, "zeros", None, "lrelu"),
    ("conv_s2_relu_gate_512x128", "g4", "conv", 16, 128, 0, 128, 128, 4, 2, 1, "zeros", "relu", None),
    ("convT_relu_512x128", "g4", "convT", 16, 256, 0, 64, 128, 4, 2, 1, "zeros", "relu", None),
]


@pytest.mark.parametrize("case", CASES_512, ids=[c[0] for c in CASES_512])
def test_m32_512_rows_bitwise_vs_256(case):
    """Per output element the 512-row tile runs the 256-row tile's MFMA chain (same K tiles,
    same 32x32x16 blocks, same epilogue rounding): forward and input gradients bitwise equal,
    and the 512-row instances must actually have run (forward and the MODE-1 gradient)."""
    out_a, _, names = _run(case, True, {"P2P_M32_BM": "512"})
    out_b, _, names_b = _run(case, True, {"P2P_M32_BM": "256"})
    assert any(n.rstrip(")").split("(")[0].endswith(", 512>") for n in names), sorted(set(names))
    assert not any(", 512>" in n for n in names_b), sorted(set(names_b))
    if case[12] == "relu" and case[2] == "conv":   # gated input gradient: the EXT instance
        assert any("conv_fwd_m32_kernel<128, 1, false, true, 0, 512>" in n for n in names), sorted(set(names))
    for ta, tb in zip(out_a, out_b):
        if ta is not None:
            assert torch.equal(ta, tb), (case[0], (ta.float() - tb.float()).abs().max().item())


def test_m32_512_rows_oracle():
    """The first 512-row case against the fp32 oracle (bias, lrelu output, concat)."""
    case = CASES_512[0]
    name, var, kind, N, C1, C2, H, Cout, k, s, p, pad_mode, act_in, act_out = case
    (y, gx1, gx2, gw, gb), (x1, x2, w, b, gy), names = _run(case, True, {"P2P_M32_BM": "512"})
    assert any(", 512>" in n for n in names)
    rx1, rx2, rw, rb = _leaf(x1.float()), _leaf(x2.float()), _leaf(w), _leaf(b)
    ry = ref.conv2d((rx1, rx2), rw.to(torch.bfloat16).float(), rb, s, p, pad_mode, 1, act_in=act_in,
                    act_out=act_out)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 2e-2
    assert rel_err(gx1, rx1.grad) < 3e-2 and rel_err(gx2, rx2.grad) < 3e-2


def test_m32_512_rows_full_step_fused_norms(monkeypatch):
    """Fused norm statistics and norm-backward partials are chunked per BM rows (host and
    kernel share one predicate, p2p_conv_m32_rows): two pix2pix steps (batch-norm U-Net,
    instance-norm PatchGAN) with the 512-row tiles pinned match the 256-row run's losses.
    Batch 16: the Cout-128 layers (e2, c2, their input gradients) reach the 256 tiles below
    which split-K takes them."""
    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    from p2p_pytorch_amd.ops import hip

    def run(bm):
        monkeypatch.setenv("P2P_M32_BM", bm)
        hip.reset_rng(0)
        torch.manual_seed(0)
        G = define_G(netG="unet_256", gpu_id=DEV, verbose=False)
        D = define_D(6, 64, norm="instance", netD="basic", gpu_id=DEV, verbose=False)
        st = Pix2PixStep(G, D)
        a = rand_img(16, 3, 256, 256, seed=31)
        b = rand_img(16, 3, 256, 256, seed=32)
        p2p.set_deterministic(True)
        try:
            with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
                losses = [st.step(a, b), st.step(a, b)]
                torch.cuda.synchronize()
        finally:
            p2p.set_deterministic(False)
        names = {e.name for e in prof.events() if "conv_fwd_m32_kernel" in e.name}
        return [{k: float(v) for k, v in l.items()} for l in losses], names

    l512, n512 = run("512")
    l256, n256 = run("256")
    assert any(", 512>" in n for n in n512), sorted(n512)
    assert not any(", 512>" in n for n in n256)
    for a, b in zip(l512, l256):
        for k in a:
            assert abs(a[k] - b[k]) <= 2e-3 * max(1.0, abs(b[k])), (k, a[k], b[k])


# The 512 x 64 tile (round 6): 33-64 output channels (the glds 128 x 64 tile otherwise) --
# family R's 64-channel 3x3 layers, VGG conv1_x / conv2_1's neighbours; forced onto the GEMM
# route with variant g2 (no halo / s2t kernels), >= 256 tiles of 128 rows (no split-K)
CASES_64 = [
    ("conv3x3_c64_relu_out_512x64", "g2", "conv", 16, 64, 0, 64, 64, 3, 1, 1, "zeros", None, "relu"),
    ("conv3x3_reflect_relu_in_cout48", "g2", "conv", 16, 128, 0, 64, 48, 3, 1, 1, "reflect", "relu", None),
    ("convT_c64_512x64", "g2", "convT", 16, 128, 0, 32, 64, 4, 2, 1, "zeros", None, None),
]


@pytest.mark.parametrize("case", CASES_64, ids=[c[0] for c in CASES_64])
def test_m32_512x64_matches_oracle_and_glds(case, monkeypatch):
    name, var, kind, N, C1, C2, H, Cout, k, s, p, pad_mode, act_in, act_out = case
    # (pinned: these grids have 128-256 blocks of 512 rows, below the route's one-per-CU bar)
    (y, gx1, gx2, gw, gb), (x1, x2, w, b, gy), names = _run(case, True, {"P2P_M32_BM": "512"})
    assert any("conv_fwd_m32_kernel<64, " in n and ", 512>" in n for n in names), sorted(set(names))
    rx1, rw, rb = _leaf(x1.float()), _leaf(w), _leaf(b)
    wq = rw.to(torch.bfloat16).float()
    if kind == "conv":
        ry = ref.conv2d(rx1, wq, rb, s, p, pad_mode, 1, act_in=act_in, act_out=act_out)
    else:
        ry = ref.conv_transpose2d(rx1, wq, rb, s, p, act_in, act_out)
    ry.backward(gy.float())
    assert rel_err(y, ry) < 2e-2, (name, "y", rel_err(y, ry))
    assert rel_err(gx1, rx1.grad) < 3e-2, (name, "dx", rel_err(gx1, rx1.grad))
    assert rel_err(gw, rw.grad) < 3e-2, (name, "dw")
    out_b, _, names_b = _run(case, True, {"P2P_M32_BM": "512", "P2P_M32_C64": "0"})
    assert not any("conv_fwd_m32_kernel<64, " in n for n in names_b)
    assert rel_err(y, out_b[0]) < 1.5e-2 and rel_err(gx1, out_b[1]) < 1.5e-2
