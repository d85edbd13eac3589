"""Data parallelism under the reference-family step (gloo, world 2 and 4, CPU).

The reference step back-propagates the G loss through D and discards those D gradients
(/root/reference/train.py:384-389).  Under data parallelism that backward must not launch
D all-reduces, and every D backward that IS kept must be reduced exactly once.  Checked
over several steps (the round-1 reducer desynchronised D from step 2 on):

  * every D bucket is launched exactly once per step (the G backward launches none);
  * the reduced D gradient equals the mean over ranks of the local (pre-reduction) ones;
  * G, D and C parameters stay bitwise identical across ranks after every step;
  * the ready-order re-bucketing agrees across ranks (same bucket layout).
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_ddp_cpu import _free_port

STEPS = 3


def _flat(mod):
    return torch.cat([p.detach().reshape(-1) for p in mod.parameters()])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
        from p2p_pytorch_amd.models import VGGLoss, define_C, define_D, define_G
        from p2p_pytorch_amd.parallel import GradReducer
        from p2p_pytorch_amd.parallel import dist as pdist
        pdist.init_from_env()
        torch.manual_seed(100 + rank)                 # deliberately different per rank ...
        G = define_G(gpu_id="cpu", verbose=False)
        D = define_D(6, 16, gpu_id="cpu", verbose=False)
        C = define_C(gpu_id="cpu", verbose=False)
        for m in (G, D, C):
            pdist.broadcast_module(m)                 # ... fixed by the rank-0 broadcast
        torch.manual_seed(7)
        vgg = VGGLoss()                               # frozen: identical by seed
        red_g = GradReducer(G, bucket_mb=2.0)
        red_d = GradReducer(D, bucket_mb=0.25)
        assert len(red_d.buckets) > 1
        launches, local = [], {}
        orig = red_d._launch

        def spy(b):
            launches.append(b.index)
            local[b.index] = b.flat.detach().clone() / red_d.scale   # grads arrive pre-scaled
            orig(b)

        red_d._launch = spy
        step = CompressGANStep(G, D, C, vgg=vgg, reducer_g=red_g, reducer_d=red_d)
        g = torch.Generator().manual_seed(321)
        report = []
        for it in range(STEPS):
            A = torch.rand(world, 3, 32, 32, generator=g) * 2 - 1
            B = torch.rand(world, 3, 32, 32, generator=g) * 2 - 1
            launches.clear()
            local.clear()
            d_before = _flat(D).clone()
            out = step.step(A[rank:rank + 1], B[rank:rank + 1])
            assert not torch.equal(d_before, _flat(D)), "D did not train"
            assert all(float(b.flat.abs().max()) > 0 for b in red_d.buckets), "zero D grads"
            assert all(torch.isfinite(v).all() for v in out.values())
            assert sorted(launches) == list(range(len(red_d.buckets))), (it, launches)
            # reduced == mean of the local gradients
            worst = 0.0
            for b in red_d.buckets:
                gl = [torch.zeros_like(local[b.index]) for _ in range(world)]
                dist.all_gather(gl, local[b.index])
                mean = torch.stack(gl).mean(0)
                worst = max(worst, float((b.flat - mean).abs().max() /
                                         (mean.abs().max() + 1e-12)))
            same = True
            for m in (G, D, C):
                f = _flat(m)
                gathered = [torch.zeros_like(f) for _ in range(world)]
                dist.all_gather(gathered, f)
                same = same and all(torch.equal(gathered[0], t) for t in gathered)
            report.append((worst, same, [len(b.params) for b in red_d.buckets]))
        q.put((rank, report))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_family_r_dp_keeps_ranks_in_sync(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    layouts = set()
    for rank, rep in res:
        assert not isinstance(rep, str), rep
        for it, (worst, same, layout) in enumerate(rep):
            assert worst < 1e-6, f"rank {rank} step {it}: reduced D grad != shard mean ({worst})"
            assert same, f"rank {rank} step {it}: parameters diverged across ranks"
        layouts.add(tuple(rep[-1][2]))
    assert len(layouts) == 1, layouts
