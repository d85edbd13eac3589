"""Norm-backward partial sums fused into the consumer conv's dgrad epilogue (conv_dev.h nb_*).

The fused path must compute the same input / parameter gradients as the norm's own partial
pass (only the fp32 summation order of the per-channel sums differs), and it must actually
run for the layer shapes it targets: encoder conv -> IN(lrelu) -> strided conv (MODE-1
dgrad), decoder ConvT(cat(skip, relu(IN(.)))) (second half of a split MODE-0 dgrad), and
batch norm + ReLU / shared-slope PReLU, affine, also under a reflect-pad or nearest-x2 fold
(family R: interior pixels in the epilogue, the band's change in fold_band).  Checked op-level against the unfused path and the fp32
oracle, and at model level on the U-Net-256 generator.  Batches are sized so the dgrads
run without split-K (the fusion needs whole tiles; split-K layers keep the partial pass).
"""
import pytest
import torch

from p2p_pytorch_amd import _native, ops
from p2p_pytorch_amd.ops import hip
from p2p_pytorch_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_backend():
    _native.set_backend("native")
    assert _native.load(), _native.load_error()
    yield


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def bf(x):
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _rand(*shape, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, device=DEV, generator=g) * scale


class _Count:
    def __init__(self, monkeypatch):
        self.hits = 0
        orig = hip._take_nbp

        def take(g):
            p = orig(g)
            self.hits += p is not None
            return p
        monkeypatch.setattr(hip, "_take_nbp", take)


def _run(monkeypatch, fused, fn):
    monkeypatch.setattr(hip, "_NB_FUSE", fused)
    hip.begin_step()
    out = fn()
    assert not hip._nbp_stash, "every parked partial must be taken by its norm"
    return out


def test_nb_encoder_instance_lrelu(monkeypatch):
    x = bf(_rand(64, 64, 64, 64, seed=1))
    w1 = _rand(128, 64, 4, 4, seed=2, scale=(1 / 1024) ** 0.5)
    w2 = _rand(256, 128, 4, 4, seed=3, scale=(1 / 2048) ** 0.5)
    gy = bf(_rand(64, 256, 16, 16, seed=4))

    def fn():
        hx, hw1, hw2 = x.clone().requires_grad_(True), w1.clone().requires_grad_(True), w2.clone().requires_grad_(True)
        h = ops.conv2d(hx, hw1, None, 2, 1, stats=True)
        z = ops.instance_norm(h, act="lrelu")
        y = ops.conv2d(z, hw2, None, 2, 1)
        y.backward(gy)
        return hx.grad.float(), hw1.grad.float(), hw2.grad.float()

    cnt = _Count(monkeypatch)
    fused = _run(monkeypatch, True, fn)
    assert cnt.hits == 1, "the fused partials were not used"
    plain = _run(monkeypatch, False, fn)
    assert cnt.hits == 1
    for a, b in zip(fused, plain):
        assert rel_err(a, b) < 1e-2
    # fp32 oracle on the same bf16 inputs
    rx = x.float().requires_grad_(True)
    h = ref.conv2d(rx, w1.to(torch.bfloat16).float(), None, 2, 1)
    z = ref.instance_norm(h, 1e-5, "lrelu")
    ref.conv2d(z, w2.to(torch.bfloat16).float(), None, 2, 1).backward(gy.float())
    # the fusion only reorders fp32 sums: as close to the oracle as the unfused bf16 path
    assert rel_err(fused[0], rx.grad) <= 1.1 * rel_err(plain[0], rx.grad) + 1e-3


def test_nb_decoder_split_half_relu(monkeypatch):
    """ConvT(cat(skip, u)) with u = relu(IN(ConvT(.))): the up half (second output half of
    the MODE-0 dgrad, no ReLU' gate of its own) carries the norm's partials."""
    skip = bf(_rand(64, 64, 32, 32, seed=11))
    v = bf(_rand(64, 128, 16, 16, seed=12))
    wi = _rand(128, 64, 4, 4, seed=13, scale=(1 / 512) ** 0.5)
    wo = _rand(128, 32, 4, 4, seed=14, scale=(1 / 512) ** 0.5)
    gy = bf(_rand(64, 32, 64, 64, seed=15))

    def fn():
        hv, hwi, hwo = v.clone().requires_grad_(True), wi.clone().requires_grad_(True), wo.clone().requires_grad_(True)
        u = ops.instance_norm(ops.conv_transpose2d(hv, hwi, None, 2, 1, "relu", None, stats=True), act="relu")
        y = ops.conv_transpose2d((skip, u), hwo, None, 2, 1, "relu", None, gate_x2=False)
        y.backward(gy)
        return hv.grad.float(), hwi.grad.float(), hwo.grad.float()

    cnt = _Count(monkeypatch)
    fused = _run(monkeypatch, True, fn)
    assert cnt.hits == 1, "the fused partials were not used"
    plain = _run(monkeypatch, False, fn)
    for a, b in zip(fused, plain):
        assert rel_err(a, b) < 1e-2


@pytest.mark.parametrize("affine", [False, True])
def test_nb_batch_norm_relu(monkeypatch, affine):
    """Batch norm + ReLU, plain and affine (round 5: affine batch norms fuse too)."""
    x = bf(_rand(64, 64, 64, 64, seed=21))
    w1 = _rand(128, 64, 4, 4, seed=22, scale=(1 / 1024) ** 0.5)
    w2 = _rand(128, 128, 4, 4, seed=23, scale=(1 / 2048) ** 0.5)
    gam = 1 + _rand(128, seed=24, scale=0.1)
    bet = _rand(128, seed=25, scale=0.1)
    gy = bf(_rand(64, 128, 16, 16, seed=26))

    def fn():
        hx = x.clone().requires_grad_(True)
        hg = gam.clone().requires_grad_(True) if affine else None
        hb = bet.clone().requires_grad_(True) if affine else None
        rm, rv = torch.zeros(128, device=DEV), torch.ones(128, device=DEV)
        h = ops.conv2d(hx, w1, None, 2, 1, stats=True)
        z = ops.batch_norm(h, rm, rv, hg, hb, True, act="relu")
        ops.conv2d(z, w2, None, 2, 1).backward(gy)
        return (hx.grad.float(),) + ((hg.grad.float(), hb.grad.float()) if affine else ())

    cnt = _Count(monkeypatch)
    fused = _run(monkeypatch, True, fn)
    assert cnt.hits == 1
    plain = _run(monkeypatch, False, fn)
    for a, b in zip(fused, plain):
        assert rel_err(a, b) < 1e-2


def test_nb_unet256_generator_grads(monkeypatch):
    """Model level: U-Net-256 generator gradients with and without the fusion, each against
    the fp32 eager oracle (8 chained bf16 layers amplify any reordering of the sums, so the
    two bf16 runs are compared by their distance from fp32, per parameter)."""
    from p2p_pytorch_amd.models import define_G
    torch.manual_seed(0)
    G = define_G(netG="unet_256", gpu_id=DEV, verbose=False, use_dropout=False)
    A = bf(torch.rand(16, 3, 256, 256, device=DEV) * 2 - 1)

    def fn():
        G.zero_grad(set_to_none=True)
        G(A).float().square().mean().backward()
        hip.assert_no_deferred()
        return {n: p.grad.detach().float().clone() for n, p in G.named_parameters()}

    cnt = _Count(monkeypatch)
    fused = _run(monkeypatch, True, fn)
    assert cnt.hits >= 3, cnt.hits   # e2 / e3 consumers, u2 (u1: the image-layer halo kernel)
    plain = _run(monkeypatch, False, fn)
    _native.set_backend("torch")
    try:
        G.zero_grad(set_to_none=True)
        G(A.float()).square().mean().backward()
        oracle = {n: p.grad.detach().float().clone() for n, p in G.named_parameters()}
        G.zero_grad(set_to_none=True)      # stock kernels under bf16 autocast: the dtype's error
        with torch.autocast("cuda", dtype=torch.bfloat16):
            G(A.float()).float().square().mean().backward()
        eager = {n: p.grad.detach().float().clone() for n, p in G.named_parameters()}
    finally:
        _native.set_backend("native")
    def rel_l2(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    for n in fused:
        ef, ep = rel_err(fused[n], oracle[n]), rel_err(plain[n], oracle[n])
        ee = rel_err(eager[n], oracle[n])
        assert ef <= 1.5 * ep + 0.01, (n, ef, ep)
        if ee > 0.25:
            # the innermost instance norms (2x2 / 4x4 planes) leave these gradients without
            # bf16-resolvable signal -- the fp64 oracle study puts EVERY bf16 path 34-192 %
            # (max-norm) off there (profiles/diag_inner_grad_r4.txt): where even eager bf16 is
            # > 25 % off, the native path is held to 3x its relative-L2 error instead
            el2, pl2 = rel_l2(eager[n], oracle[n]), rel_l2(plain[n], oracle[n])
            assert pl2 <= 3 * el2 + 0.01, (n, pl2, el2)
            continue
        # and absolutely: the unfused native path within twice the eager bf16 error
        assert ep <= 2 * ee + 0.01, (n, ep, ee)


def test_fused_bias_colsum(monkeypatch):
    """A biased conv whose LeakyReLU' is applied by its consumer's dgrad (out_gated /
    grad_gate, the U-Net's outermost conv / the PatchGAN's first conv): the consumer's dgrad
    epilogue emits the gradient's column sums, which become the producer's bias gradient."""
    x = bf(_rand(64, 32, 64, 64, seed=31))
    w1 = _rand(64, 32, 4, 4, seed=32, scale=(1 / 512) ** 0.5)
    b1 = _rand(64, seed=33, scale=0.1)
    w2 = _rand(128, 64, 4, 4, seed=34, scale=(1 / 1024) ** 0.5)
    gy = bf(_rand(64, 128, 16, 16, seed=35))
    taken = []
    orig = hip._take_colsum

    def take(g):
        r = orig(g)
        taken.append(r is not None)
        return r
    monkeypatch.setattr(hip, "_take_colsum", take)

    def fn():
        hw1, hb1 = w1.clone().requires_grad_(True), b1.clone().requires_grad_(True)
        h = ops.conv2d(x, hw1, hb1, 2, 1, act_out="lrelu", out_gated=True)
        ops.conv2d(h, w2, None, 2, 1, grad_gate="lrelu").backward(gy)
        return hw1.grad.float(), hb1.grad.float()

    taken.clear()
    fused = _run(monkeypatch, True, fn)
    assert taken == [True], taken
    taken.clear()
    plain = _run(monkeypatch, False, fn)
    assert taken == [False], taken
    assert rel_err(fused[0], plain[0]) < 1e-2
    assert rel_err(fused[1], plain[1]) < 1e-2
