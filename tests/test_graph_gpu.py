"""hipGraph replay == eager training, and the RCCL reducer path under capture.

``bench.py`` times graph replays, so the replay must do exactly the work of the eager
step.  With ``set_deterministic(True)`` (ordered split-K reductions):

  (a) K replays of ``CapturedStep`` from a fresh model give bitwise the parameters of K
      eager steps from the same init and data -- the capture's warmup steps are rolled
      back (engine/graph.py) and every per-step input (Adam step / lr, dropout seed,
      weight images) advances on the device;
  (b) the same with the data-parallel reducers attached on a world-size-1 RCCL process
      group and ``force_comm=True``: the bucket all-reduces are real RCCL collectives,
      captured into the graph, and the result is still bitwise the plain eager step --
      with the conv weight gradients written straight into the buckets by the kernels
      (direct gradients, on the side stream; counted) and with them through autograd.
"""
import pytest
import torch
import torch.distributed as dist

import p2p_pytorch_amd as p2p
from p2p_pytorch_amd.ops import hip

pytestmark = pytest.mark.gpu

STEPS = 3


def _build(reducers=False, direct=True, comm_dtype=None):
    from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
    from p2p_pytorch_amd.models import define_D, define_G
    from p2p_pytorch_amd.parallel import GradReducer
    dev = torch.device("cuda")
    hip.reset_rng(0)
    torch.manual_seed(0)
    G = define_G(netG="unet_64", gpu_id=dev, verbose=False)       # 6 levels, dropout on
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id=dev, verbose=False)
    rg = rd = None
    if reducers:
        rg = GradReducer(G, bucket_mb=4.0, force_comm=True, direct=direct, comm_dtype=comm_dtype)
        rd = GradReducer(D, bucket_mb=4.0, force_comm=True, direct=direct, comm_dtype=comm_dtype)
        assert len(rg.buckets) > 1
        # the world-8 op at world 1: RCCL averages inside the collective
        assert rg._avg and rd._avg and rg._op() == dist.ReduceOp.AVG
    return Pix2PixStep(G, D, reducer_g=rg, reducer_d=rd), G, D


def _data():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    out = []
    for _ in range(STEPS):
        ab = [(torch.rand(2, 3, 64, 64, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
              .contiguous(memory_format=torch.channels_last) for _ in range(2)]
        out.append(ab)
    return out


def _params(G, D):
    return torch.cat([p.detach().reshape(-1) for p in list(G.parameters()) + list(D.parameters())])


def _eager(reducers=False, direct=True, comm_dtype=None):
    step, G, D = _build(reducers, direct, comm_dtype)
    for a, b in _data():
        losses = step.step(a, b)
    torch.cuda.synchronize()
    return _params(G, D), {k: v.item() for k, v in losses.items()}


def _graph(reducers=False, direct=True, comm_dtype=None):
    from p2p_pytorch_amd.engine.graph import CapturedStep
    step, G, D = _build(reducers, direct, comm_dtype)
    data = _data()
    cap = CapturedStep(step.step, *data[0], warmup=2)
    if reducers:
        # the recorded collectives run on the capture's own fresh group (engine/graph.py)
        assert step.reducer_g.pg is not None and step.reducer_g.pg is step.reducer_d.pg
    for a, b in data:
        losses = cap(a, b)
    torch.cuda.synchronize()
    return _params(G, D), {k: v.item() for k, v in losses.items()}


@pytest.fixture()
def deterministic():
    p2p.set_backend("native")
    p2p.set_deterministic(True)
    yield
    p2p.set_deterministic(False)


def test_graph_replay_equals_eager_steps(deterministic):
    pe, le = _eager()
    pg, lg = _graph()
    assert le == lg
    assert torch.equal(pe, pg), (pe - pg).abs().max().item()


def test_rccl_reducers_under_capture_equal_eager(deterministic):
    from p2p_pytorch_amd.parallel import dist as pdist
    pdist.init_single(torch.device("cuda", torch.cuda.current_device()))
    from p2p_pytorch_amd.parallel import GradReducer
    ndirect = [0]
    orig = GradReducer.direct_done

    def counted(self, p, stream=None):
        ndirect[0] += 1
        return orig(self, p, stream)

    GradReducer.direct_done = counted
    try:
        assert dist.get_backend() == "nccl"
        pe, le = _eager(reducers=False)
        pr, lr = _eager(reducers=True)          # eager with real RCCL collectives
        n_eager = ndirect[0]
        pa, la = _eager(reducers=True, direct=False)   # gradients through autograd
        pg, lg = _graph(reducers=True)          # the same, captured into one hipGraph
    finally:
        GradReducer.direct_done = orig
        dist.destroy_process_group()
    assert n_eager > 0, "no conv weight gradient took the direct path"
    assert le == lr == la == lg
    assert torch.equal(pe, pr), (pe - pr).abs().max().item()
    assert torch.equal(pe, pa), (pe - pa).abs().max().item()
    assert torch.equal(pe, pg), (pe - pg).abs().max().item()


def test_rccl_bf16_comm_avg_under_capture(deterministic):
    """``--comm_dtype bf16``: buckets narrowed to bf16, ``ReduceOp.AVG`` on RCCL (world 1:
    the identity average, rounded through bf16), captured == eager bitwise."""
    from p2p_pytorch_amd.parallel import dist as pdist
    pdist.init_single(torch.device("cuda", torch.cuda.current_device()))
    try:
        pe, le = _eager(reducers=True, comm_dtype=torch.bfloat16)
        pg, lg = _graph(reducers=True, comm_dtype=torch.bfloat16)
        pf, _ = _eager(reducers=True)
    finally:
        pdist.destroy()
    assert le == lg
    assert torch.equal(pe, pg), (pe - pg).abs().max().item()
    assert not torch.equal(pe, pf), "bf16 comm buffers changed nothing: not exercised"
