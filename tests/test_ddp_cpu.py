"""Data-parallel plumbing on CPU: gloo process group, world_size 2 (and 4).

Checks the bucketed GradReducer: after one pix2pix step on per-rank shards, every rank
holds the gradient of the *global* batch (mean over ranks == single-process gradient on
the concatenated batch), parameters stay bitwise identical across ranks after Adam, and
broadcast_module synchronises a mismatched init.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build(seed):
    from p2p_pytorch_amd.models import define_D, define_G
    torch.manual_seed(seed)
    G = define_G(netG="unet_4", ngf=8, gpu_id="cpu", verbose=False, use_dropout=False)
    D = define_D(6, 8, norm="instance", netD="basic", gpu_id="cpu", verbose=False)
    return G, D


def _data(world):
    g = torch.Generator().manual_seed(123)
    A = torch.rand(2 * world, 3, 32, 32, generator=g) * 2 - 1
    B = torch.rand(2 * world, 3, 32, 32, generator=g) * 2 - 1
    return A, B


def _grads_single(world):
    from p2p_pytorch_amd.models import GANLoss
    from p2p_pytorch_amd.ops import l1
    G, D = _build(100)             # rank 0's init, which the broadcast propagates
    A, B = _data(world)
    crit = GANLoss(gan_mode="vanilla")
    fake = G(A)
    loss = crit(D(torch.cat((A, fake), 1)), True) + 100 * l1(fake, B)
    loss.backward()
    return {n: p.grad.clone() for n, p in G.named_parameters()}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from p2p_pytorch_amd.models import GANLoss
        from p2p_pytorch_amd.ops import l1
        from p2p_pytorch_amd.parallel import GradReducer
        from p2p_pytorch_amd.parallel import dist as pdist
        pdist.init_from_env()
        G, D = _build(100 + rank)          # deliberately different init per rank ...
        pdist.broadcast_module(G)          # ... fixed by the rank-0 broadcast
        pdist.broadcast_module(D)
        red = GradReducer(G, bucket_mb=0.05)  # tiny buckets -> several in flight
        assert len(red.buckets) > 1
        A, B = _data(world)
        a, b = A[2 * rank:2 * rank + 2], B[2 * rank:2 * rank + 2]
        crit = GANLoss(gan_mode="vanilla")
        red.zero_grad()
        fake = G(a)
        loss = crit(D(torch.cat((a, fake), 1)), True) + 100 * l1(fake, b)
        loss.backward()
        red.finish()
        grads = {n: p.grad.detach().numpy().copy() for n, p in G.named_parameters()}
        # second backward of the same batch: zero_grad() now re-buckets in the recorded
        # grad-ready order (last-ready bucket capped) -- the reduced grads must not change
        nb0 = [len(b.params) for b in red.buckets]
        red.zero_grad()
        assert red._ready_order is None, "rebucket did not run"
        fake = G(a)
        loss = crit(D(torch.cat((a, fake), 1)), True) + 100 * l1(fake, b)
        loss.backward()
        red.finish()
        for n, p in G.named_parameters():
            lo = red._param_bucket[p].flat.data_ptr()
            assert lo <= p.grad.data_ptr() < lo + red._param_bucket[p].flat.numel() * 4, n
            # (a different bucket layout changes the ring's per-element summation order)
            assert torch.allclose(p.grad, torch.from_numpy(grads[n]), rtol=1e-5, atol=1e-7), \
                ("rebucketed grad", n, nb0)
        opt = torch.optim.Adam(G.parameters(), lr=1e-3)
        opt.step()
        flat = torch.cat([p.detach().reshape(-1) for p in G.parameters()])
        gathered = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(gathered, flat)
        same = all(torch.equal(gathered[0], t) for t in gathered)
        q.put((rank, grads if rank == 0 else None, same))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e), False))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_grad_reducer_matches_global_batch(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    for rank, payload, same in res:
        assert not isinstance(payload, str), payload
        assert same, f"rank {rank}: parameters diverged after the step"
    ref = _grads_single(world)
    got = res[0][1]
    for n, g in ref.items():
        assert torch.allclose(torch.from_numpy(got[n]), g, atol=1e-6, rtol=1e-4), n
