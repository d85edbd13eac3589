"""CapturedStep's warmup rollback (engine/graph.py ``_Snapshot``) on the CPU path: after
two real training steps, restoring the snapshot returns every parameter, buffer and
optimizer moment to its pre-warmup value (the graph then replays step 1 exactly)."""
import torch


def test_snapshot_restores_pre_warmup_state():
    from p2p_pytorch_amd.engine.graph import _Snapshot
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    torch.manual_seed(0)
    G = define_G(netG="unet_4", ngf=8, gpu_id="cpu", verbose=False)
    D = define_D(6, 8, norm="batch", netD="basic", gpu_id="cpu", verbose=False)
    step = Pix2PixStep(G, D)
    a = torch.rand(2, 3, 32, 32) * 2 - 1
    b = torch.rand(2, 3, 32, 32) * 2 - 1
    step.step(a, b)          # optimizer state exists (torch Adam on CPU creates it lazily)
    before = [t.detach().clone() for t in step.state_tensors()]
    snap = _Snapshot(step)
    for _ in range(2):
        step.step(a, b)
    after = list(step.state_tensors())
    assert any(not torch.equal(x, y) for x, y in zip(before, after))
    snap.restore()
    for x, y in zip(before, step.state_tensors()):
        assert torch.equal(x, y)
    # BatchNorm D: the 2B fused D batch must be off (statistics over fake and real)
    assert not step.d_per_sample
