"""Training-convergence evidence for the native paths.

Every other numerics test compares ONE step.  Here the same pix2pix model (U-Net-128 + 70x70
PatchGAN, GAN + 100 * L1, Adam 2e-4 / 0.5, batch 16 at 128x128) is trained from the same
initial weights for ``STEPS`` steps on a learnable synthetic task -- B is a fixed 3x3 colour
mix + blur of A, with A smooth random images -- three ways:

  * stock PyTorch fp32 eager (``set_backend('torch')``, no autocast): the reference numerics;
  * the native HIP path in bf16 (the headline path);
  * the native HIP path with fp8 convs (BASELINE config 5).

Each path is trained from three initialisations (SEEDS) and compared by its mean over them:
a 300-step GAN run amplifies any numeric difference, and single runs of the identical fp32
configuration ended at L1 0.0219 / 0.0267 / 0.0298 and PSNR 35.6 / 34.6 / 33.2 dB on three
MI355X runs (MIOpen picks its algorithms per run; gpurun_out/r4l, r4m, r4m2 -- the fp32 runs
here use cudnn.deterministic), while one native bf16 / fp8 run gave 0.0306 / 33.5 dB and
0.0294 / 32.5 dB.  Asserted per native path (seed means): the train L1 (mean of the last 20
steps) fell to <= 20 % of the first 10 steps'; it ends within 20 % of the fp32 mean; no update
was skipped by the NaN guard; and the held-out PSNR (the reference's per-epoch validation
metric, train.py:450-502, computed on the device by engine/metrics.py; averaged over the last
five evaluations, every 10 steps) is at most 2 dB below the fp32 mean and 15 dB above the
untrained generator's.  Dropout is off
(``use_dropout=False``) so the runs see the same network function (their dropout RNG streams
differ by backend).
"""
import pytest
import torch
import torch.nn.functional as F

import p2p_pytorch_amd as p2p
from p2p_pytorch_amd.ops import fp8 as _fp8

pytestmark = pytest.mark.gpu

STEPS = 300
BATCH = 16
SIZE = 128
NTRAIN = 64
NTEST = 16


def _task(seed=0):
    """Smooth random A in [-1, 1] (bilinear-upsampled 16x16 noise) and B = clamp(mix(A))."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(seed)
    n = NTRAIN + NTEST
    low = torch.rand(n, 3, 16, 16, device=dev, generator=g) * 2 - 1
    a = F.interpolate(low, size=(SIZE, SIZE), mode="bilinear", align_corners=False).clamp(-1, 1)
    mix = torch.tensor([[0.2, 0.7, 0.1], [0.6, -0.3, 0.5], [-0.4, 0.3, 0.8]], device=dev)
    w = torch.zeros(3, 3, 3, 3, device=dev)
    blur = torch.tensor([[1., 2., 1.], [2., 4., 2.], [1., 2., 1.]], device=dev) / 16.0
    for o in range(3):
        for i in range(3):
            w[o, i] = mix[o, i] * blur
    b = F.conv2d(a, w, padding=1).clamp(-1, 1)
    return a[:NTRAIN], b[:NTRAIN], a[NTRAIN:], b[NTRAIN:]


def _init_state(seed=1234):
    from p2p_pytorch_amd.models import define_D, define_G
    torch.manual_seed(seed)
    G = define_G(netG="unet_128", gpu_id="cuda", use_dropout=False, verbose=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id="cuda", verbose=False)
    return ({k: v.detach().clone() for k, v in G.state_dict().items()},
            {k: v.detach().clone() for k, v in D.state_dict().items()})


def _train(backend, precision, init, task):
    from p2p_pytorch_amd.engine.metrics import psnr
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    p2p.set_backend(backend)
    _fp8.set_precision(precision)
    try:
        G = define_G(netG="unet_128", gpu_id="cuda", use_dropout=False, verbose=False)
        D = define_D(6, 64, norm="instance", netD="basic", gpu_id="cuda", verbose=False)
        G.load_state_dict(init[0])
        D.load_state_dict(init[1])
        step = Pix2PixStep(G, D, lr=2e-4, beta1=0.5, lambda_L1=100.0)
        a_tr, b_tr, a_te, b_te = task
        dt = torch.float32 if backend == "torch" else torch.bfloat16

        def prep(x):
            return x.to(dt).contiguous(memory_format=torch.channels_last)

        def held_out_psnr():
            with torch.no_grad():
                out = G(prep(a_te)).float()
            # per-image PSNR on [-1, 1] -> [0, 1] levels, averaged like the reference's epoch mean
            return float(psnr(b_te.float(), out, ref_compat=False).float().mean())

        p0 = held_out_psnr()
        l1, tail = [], []
        for s in range(STEPS):
            i = (s * BATCH) % NTRAIN
            losses = step.step(prep(a_tr[i:i + BATCH]), prep(b_tr[i:i + BATCH]))
            l1.append(losses["G_L1"])
            if s + 1 > STEPS - PSNR_TAIL * PSNR_EVERY and (s + 1) % PSNR_EVERY == 0:
                tail.append(held_out_psnr())
        l1 = [float(v) / 100.0 for v in l1]
        p1 = sum(tail) / len(tail)
        skipped = float(step.skipped) if step.skipped is not None else 0.0
        return {"l1_first": sum(l1[:10]) / 10, "l1_last": sum(l1[-20:]) / 20, "psnr0": p0, "psnr": p1,
                "skipped": skipped, "finite": all(v == v for v in l1)}
    finally:
        _fp8.set_precision("bf16")
        p2p.set_backend("native")


SEEDS = (1234, 1235, 1236)
# held-out PSNR: the mean of the evaluations after the last PSNR_TAIL x PSNR_EVERY steps, not
# the single final one -- the GAN term makes the generator oscillate by a dB or more from one
# evaluation to the next (round 6: one fp32 run ended at 35.4 / 35.2 / 35.5 dB, the next native
# bf16 one at 32.9 / 33.0 / 35.4, gpurun_out/r6p), and a single end point turned that noise into
# the asserted difference
PSNR_EVERY = 10
PSNR_TAIL = 5


@pytest.fixture(scope="module")
def runs():
    """Every path trained from the same SEEDS initialisations; per path the mean over seeds."""
    task = _task()
    inits = [_init_state(sd) for sd in SEEDS]
    cudnn = (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        per = {"fp32": [_train("torch", "bf16", i, task) for i in inits]}
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = cudnn
    per["bf16"] = [_train("native", "bf16", i, task) for i in inits]
    per["fp8"] = [_train("native", "fp8", i, task) for i in inits]
    out = {}
    for k, rs in per.items():
        out[k] = {f: sum(r[f] for r in rs) / len(rs) for f in ("l1_first", "l1_last", "psnr0", "psnr", "skipped")}
        out[k]["finite"] = all(r["finite"] for r in rs)
        out[k]["per_seed"] = [(round(r["l1_last"], 5), round(r["psnr"], 2)) for r in rs]
    print("convergence:", out)
    return out


@pytest.mark.parametrize("path", ["bf16", "fp8"])
def test_native_training_converges_like_fp32(runs, path):
    ref, r = runs["fp32"], runs[path]
    assert ref["finite"] and r["finite"]
    assert ref["l1_last"] <= 0.2 * ref["l1_first"], ref          # the task is learnable
    assert r["skipped"] == 0.0, r
    assert r["l1_last"] <= 0.2 * r["l1_first"], r
    assert abs(r["l1_last"] - ref["l1_last"]) <= 0.2 * ref["l1_last"], (r, ref)
    assert r["psnr"] > r["psnr0"] + 15.0, r
    # (3-seed means of the tail PSNR; fp32-vs-fp32 single runs spanned 2.4 dB, round 4)
    assert r["psnr"] >= ref["psnr"] - 2.0, (r, ref)
