"""hipGraph replay of the reference-family step (/root/reference/train.py:291-414) == eager.

Round 4 broke the family-R capture without a test noticing: the nearest-x2 dgrad's weight
image was built from a host tensor (``torch.tensor`` + ``einsum``) inside the captured
backward, capture raised and ``bench.py --family ref`` silently ran eager.  The image is now
a device kernel (``torch.ops.p2p.up2_dgrad_image``); this test pins the capture itself:

  (a) the step captures (``CapturedStep`` raises ``CaptureError`` otherwise), and
  (b) with ``set_deterministic(True)`` K replays give bitwise the parameters, buffers
      (BatchNorm running stats, spectral-norm u / v) and losses of K eager steps from the
      same init and data, so ``bench.py`` times exactly the eager step's work;
  (c) the phase-summed 4x4 image equals the einsum definition it replaced.
"""
import pytest
import torch

import p2p_pytorch_amd as p2p
from p2p_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu

STEPS = 3


def _build():
    from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
    from p2p_pytorch_amd.models import VGGLoss, define_C, define_D, define_G
    dev = torch.device("cuda")
    hip.reset_rng(0)
    torch.manual_seed(7)
    G = define_G(gpu_id=dev, verbose=False)
    D = define_D(6, 64, gpu_id=dev, verbose=False)
    C = define_C(gpu_id=dev, verbose=False)
    vgg = VGGLoss().to(dev)
    step = CompressGANStep(G, D, C, vgg=vgg, c_phase_backward=True)
    return step, (G, D, C)


def _data():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    return [[(torch.rand(2, 3, 64, 64, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
             .contiguous(memory_format=torch.channels_last) for _ in range(2)]
            for _ in range(STEPS)]


def _state(nets):
    ts = []
    for m in nets:
        ts += [p.detach().reshape(-1).float() for p in m.parameters()]
        ts += [b.detach().reshape(-1).float() for b in m.buffers() if b.dtype.is_floating_point]
    return torch.cat(ts)


@pytest.fixture()
def deterministic():
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    yield
    p2p.set_deterministic(False)


def test_family_r_graph_replay_equals_eager(deterministic):
    from p2p_pytorch_amd.engine.graph import CapturedStep
    step, nets = _build()
    for a, b in _data():
        le = step.step(a, b)
    torch.cuda.synchronize()
    se, le = _state(nets), {k: v.item() for k, v in le.items()}

    step, nets = _build()
    data = _data()
    cap = CapturedStep(step.step, *data[0], warmup=2)     # raises CaptureError on failure
    for a, b in data:
        lg = cap(a, b)
    torch.cuda.synchronize()
    sg, lg = _state(nets), {k: v.item() for k, v in lg.items()}
    assert le == lg
    assert torch.equal(se, sg), (se - sg).abs().max().item()


def test_up2_dgrad_image_matches_einsum():
    p2p.set_backend("native")
    torch.manual_seed(3)
    w = torch.randn(40, 24, 3, 3, device="cuda")
    m = torch.tensor(((0, 0, 1), (0, 1, 1), (1, 1, 0), (1, 0, 0)), dtype=torch.float32, device="cuda")
    wd = torch.einsum("ak,oikl,bl->ioab", m, w, m).contiguous()       # [Cin][Cout][4][4]
    ref = torch.zeros(32, 4, 4, 48, device="cuda")
    ref[:24, :, :, :40] = wd.permute(0, 2, 3, 1)
    got = torch.ops.p2p.up2_dgrad_image(w, 32, 48).float()
    assert torch.equal(got, ref.to(torch.bfloat16).float())
