"""Shape fuzzing of the HIP instance / batch norm (fwd, dX, dgamma / dbeta, running stats)
against torch.nn.functional in fp32 on the same bf16 inputs -- random N, C (incl. odd
counts that go through the identity-channel padding), spatial sizes from 1x1 up, fused
ReLU / LeakyReLU, affine or not.  Derandomised, like tests/test_conv_fuzz_gpu.py."""
import os
import zlib

import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
SETTINGS = settings(max_examples=int(os.environ.get("P2P_FUZZ_EXAMPLES", "40")), deadline=None,
                    derandomize=True, database=None, suppress_health_check=list(HealthCheck))


@pytest.fixture(autouse=True, scope="module")
def _native_backend():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    yield


def bf(x):
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def close(a, b, rtol, terms=1):
    a, b = a.float().cpu(), b.float().cpu()
    return (a - b).abs().max().item() <= rtol * b.abs().max().item() + 2.0 ** -7 * terms ** 0.5


@st.composite
def norm_case(draw):
    kind = draw(st.sampled_from(["instance", "batch"]))
    N = draw(st.integers(1, 4))
    C = draw(st.sampled_from([3, 8, 16, 24, 64, 128, 200, 512]))
    H = draw(st.integers(2 if kind == "instance" else 1, 40))
    W = draw(st.integers(2 if kind == "instance" else 1, 40))
    act = draw(st.sampled_from([None, "relu", "lrelu"]))
    affine = kind == "batch" or draw(st.booleans())
    return kind, N, C, H, W, act, affine


@SETTINGS
@given(norm_case())
def test_fuzz_norm(case):
    kind, N, C, H, W, act, affine = case
    if kind == "batch" and N * H * W < 2:
        return
    g = torch.Generator(device=DEV).manual_seed(zlib.crc32(repr(case).encode()))
    x = bf(torch.randn(N, C, H, W, device=DEV, generator=g) * 2 + 1)
    gamma = (torch.rand(C, device=DEV, generator=g) + 0.5) if affine else None
    beta = (torch.randn(C, device=DEV, generator=g) * 0.1) if affine else None
    gy = bf(torch.randn(N, C, H, W, device=DEV, generator=g))
    hx = x.clone().requires_grad_(True)
    hg = gamma.clone().requires_grad_(True) if affine else None
    hb = beta.clone().requires_grad_(True) if affine else None
    # oracle on the CPU (MIOpen's own fp32 batch norm segfaults on some of these shapes), in
    # NCHW-contiguous layout (the CPU instance_norm backward is wrong for channels_last, N=1)
    rx = x.float().cpu().contiguous().requires_grad_(True)
    rg = gamma.cpu().requires_grad_(True) if affine else None
    rb = beta.cpu().requires_grad_(True) if affine else None
    if kind == "instance":
        y = ops.instance_norm(hx, 1e-5, act, hg, hb)
        z = F.instance_norm(rx, weight=rg, bias=rb, eps=1e-5)
    else:
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        rm2, rv2 = rm.cpu(), rv.cpu()
        y = ops.batch_norm(hx, rm, rv, hg, hb, True, 0.1, 1e-5, act)
        z = F.batch_norm(rx, rm2, rv2, rg, rb, True, 0.1, 1e-5)
    y.backward(gy)
    # the ReLU / LReLU kink through the HIP output's own gate (bf16 rounding near 0)
    if act in ("relu", "lrelu"):
        gate = torch.where(y.detach().float() > 0, 1.0, 0.0 if act == "relu" else 0.2)
        z.backward((gy.float() * gate).cpu().contiguous())
        ry = ref.apply_act(z.detach(), act)
    else:
        z.backward(gy.float().cpu().contiguous())
        ry = z
    group = H * W if kind == "instance" else N * H * W
    assert close(y, ry, 2e-2), ("fwd", case)
    assert close(hx.grad, rx.grad, 4e-2, 4), ("dx", case)
    if affine:
        assert close(hg.grad, rg.grad, 3e-2, N * H * W), ("dgamma", case)
        assert close(hb.grad, rb.grad, 3e-2, N * H * W), ("dbeta", case)
    if kind == "batch":
        assert close(rm, rm2, 1e-3) and close(rv, rv2, 1e-3, group), ("running stats", case)
