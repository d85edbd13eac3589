"""Shape fuzzing of the HIP conv family (hypothesis).

Random geometries -- batch, channel counts (incl. packed 3/6-channel images, odd multiples
of 8, virtual concats), kernel 1..5, stride 1..2, padding, zero / reflect pad, nearest
upsample, input / output activations, transposed convs -- each checked forward AND
backward (dX, dW, db) against the fp32 PyTorch oracle on the same bf16 inputs.  The
examples are derandomised (fixed database-free sequence) so a failure reproduces.
"""
import os
import zlib

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
SETTINGS = settings(max_examples=int(os.environ.get("P2P_FUZZ_EXAMPLES", "40")), deadline=None,
                    derandomize=True, database=None,
                    suppress_health_check=list(HealthCheck))


@pytest.fixture(autouse=True, scope="module")
def _native_backend():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    yield


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def close_sum(a, b, terms, rtol=4e-2):
    """Reductions (dW, db) over few, cancelling terms: relative error alone is meaningless
    (the bf16 rounding of each of the `terms` summands is ~2^-8), so allow an absolute floor
    of 2^-7 * sqrt(terms) on unit-scale data."""
    a, b = a.float(), b.float()
    return (a - b).abs().max().item() <= rtol * b.abs().max().item() + 2.0 ** -7 * terms ** 0.5


def bf(x):
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


CH = st.sampled_from([3, 6, 8, 16, 24, 32, 40, 64, 72, 128, 256])


@st.composite
def conv_case(draw):
    k = draw(st.integers(1, 5))
    s = draw(st.integers(1, 2))
    reflect = draw(st.booleans()) and k > 1
    p = draw(st.integers(0, k // 2)) if reflect else draw(st.integers(0, min(2, k)))
    up = draw(st.sampled_from([1, 1, 2]))
    H = draw(st.integers(max(k, p + 1, 3), 20))
    concat = draw(st.booleans()) and not reflect and up == 1
    C1 = draw(CH)
    C2 = draw(CH) if concat else 0
    Cout = draw(st.sampled_from([1, 3, 8, 16, 32, 48, 64, 128, 256]))
    N = draw(st.integers(1, 3))
    act_in = draw(st.sampled_from([None, "relu"]))
    act_out = draw(st.sampled_from([None, "relu", "lrelu", "tanh"]))
    return N, C1, C2, H, Cout, k, s, p, reflect, up, act_in, act_out


@SETTINGS
@given(conv_case())
def test_fuzz_conv2d(case):
    N, C1, C2, H, Cout, k, s, p, reflect, up, act_in, act_out = case
    if (H * up + 2 * p - k) // s + 1 < 1:
        return
    g = torch.Generator(device=DEV).manual_seed(zlib.crc32(repr(case).encode()))
    x1 = bf(torch.randn(N, C1, H, H, device=DEV, generator=g))
    x2 = bf(torch.randn(N, C2, H, H, device=DEV, generator=g)) if C2 else None
    Cin = C1 + C2
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) * (1.0 / (Cin * k * k) ** 0.5)
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    hx1 = x1.clone().requires_grad_(True)
    hx2 = x2.clone().requires_grad_(True) if x2 is not None else None
    hw, hb = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    pm = "reflect" if reflect else "zeros"
    y = ops.conv2d((hx1, hx2) if hx2 is not None else hx1, hw, hb, s, p, pad_mode=pm, upsample=up,
                   act_in=act_in, act_out=act_out)
    gy = bf(torch.randn(*y.shape, device=DEV, generator=g))
    y.backward(gy)
    rx1 = x1.float().requires_grad_(True)
    rx2 = x2.float().requires_grad_(True) if x2 is not None else None
    rw, rb = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    # piecewise-linear output activations: the oracle back-propagates through the HIP
    # output's own gate -- an output within bf16 rounding of 0 may legitimately land on the
    # other side of the kink, which would flag the whole k x k input window it touches
    kink = act_out in ("relu", "lrelu")
    ry = ref.conv2d((rx1, rx2) if rx2 is not None else rx1, rw.to(torch.bfloat16).float(), rb, s, p,
                    pad_mode=pm, upsample=up, act_in=act_in, act_out=None if kink else act_out)
    if kink:
        gate = torch.where(y.detach().float() > 0, 1.0, 0.0 if act_out == "relu" else 0.2)
        ry.backward(gy.float() * gate)
        ry = ref.apply_act(ry.detach(), act_out)
    else:
        ry.backward(gy.float())
    assert y.shape == ry.shape, case
    assert rel_err(y, ry) < 2.5e-2, ("fwd", case)
    assert rel_err(hx1.grad, rx1.grad) < 4e-2, ("dx1", case)
    if x2 is not None:
        assert rel_err(hx2.grad, rx2.grad) < 4e-2, ("dx2", case)
    P = y.shape[0] * y.shape[2] * y.shape[3]
    assert close_sum(hw.grad, rw.grad, P), ("dw", case)
    assert close_sum(hb.grad, rb.grad, P), ("db", case)


@st.composite
def convt_case(draw):
    concat = draw(st.booleans())
    C1 = draw(CH)
    C2 = draw(CH) if concat else 0
    Cout = draw(st.sampled_from([3, 8, 16, 32, 64, 128, 256]))
    H = draw(st.integers(1, 12))
    N = draw(st.integers(1, 3))
    act_in = draw(st.sampled_from([None, "relu"]))
    act_out = draw(st.sampled_from([None, "tanh"]))
    return N, C1, C2, H, Cout, act_in, act_out


@SETTINGS
@given(convt_case())
def test_fuzz_conv_transpose2d(case):
    N, C1, C2, H, Cout, act_in, act_out = case
    g = torch.Generator(device=DEV).manual_seed(zlib.crc32(repr(case).encode()))
    x1 = bf(torch.randn(N, C1, H, H, device=DEV, generator=g))
    x2 = bf(torch.randn(N, C2, H, H, device=DEV, generator=g)) if C2 else None
    Cin = C1 + C2
    w = torch.randn(Cin, Cout, 4, 4, device=DEV, generator=g) * (1.0 / (Cin * 4) ** 0.5)
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    hx1 = x1.clone().requires_grad_(True)
    hx2 = x2.clone().requires_grad_(True) if x2 is not None else None
    hw, hb = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = ops.conv_transpose2d((hx1, hx2) if hx2 is not None else hx1, hw, hb, 2, 1, act_in, act_out)
    gy = bf(torch.randn(*y.shape, device=DEV, generator=g))
    y.backward(gy)
    rx1 = x1.float().requires_grad_(True)
    rx2 = x2.float().requires_grad_(True) if x2 is not None else None
    rw, rb = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ry = ref.conv_transpose2d((rx1, rx2) if rx2 is not None else rx1, rw.to(torch.bfloat16).float(), rb, 2,
                              1, act_in, act_out)
    ry.backward(gy.float())
    assert y.shape == ry.shape == (N, Cout, 2 * H, 2 * H), case
    assert rel_err(y, ry) < 2.5e-2, ("fwd", case)
    assert rel_err(hx1.grad, rx1.grad) < 4e-2, ("dx1", case)
    if x2 is not None:
        assert rel_err(hx2.grad, rx2.grad) < 4e-2, ("dx2", case)
    P = N * H * H
    assert close_sum(hw.grad, rw.grad, P), ("dw", case)
    assert close_sum(hb.grad, rb.grad, 4 * P), ("db", case)
