"""Data-parallel hardening on CPU (gloo): the paths a multi-GPU run takes that the basic
reducer tests do not.

  * ``comm_dtype=torch.bfloat16``: buckets (gradients pre-scaled by 1/world) cast into a bf16 wire buffer,
    all-reduced, widened back -- the reduced gradient is within a bf16 bound of the fp32
    mean of the rank-local gradients, and parameters stay bitwise identical across ranks.
  * ``enable_timing()`` + ``comm_stats()``: every bucket is counted, busy / exposed times
    are non-negative and the overlap fraction lies in [0, 1].
  * ``--train_c`` under DP: C's gradients are reduced (``reducer_c``), C stays identical
    across ranks.
  * The step watchdog exits 124 while its rank is blocked inside a collective whose peer
    never arrives (the abort of the process group must not block the exit).
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_ddp_cpu import _build, _data, _free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(world, target, timeout=600):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=timeout) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    for _, payload in res:
        assert not isinstance(payload, str), payload
    return [p for _, p in res]


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)


def _pix2pix_backward(G, D, a, b):
    from p2p_pytorch_amd.models import GANLoss
    from p2p_pytorch_amd.ops import l1
    fake = G(a)
    loss = GANLoss(gan_mode="vanilla")(D(torch.cat((a, fake), 1)), True) + 100 * l1(fake, b)
    loss.backward()


def _bf16_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from p2p_pytorch_amd.parallel import GradReducer
        from p2p_pytorch_amd.parallel import dist as pdist
        pdist.init_from_env()
        G, D = _build(100 + rank)
        pdist.broadcast_module(G)
        pdist.broadcast_module(D)
        red = GradReducer(G, bucket_mb=0.05, comm_dtype=torch.bfloat16)
        assert all(b.cbuf is not None and b.cbuf.dtype == torch.bfloat16 for b in red.buckets)
        local = {}
        orig = red._launch

        def spy(b):
            # the rank-local fp32 gradient (buckets hold it pre-scaled by 1/world since round 4)
            local[b.index] = b.flat.detach().clone() / red.scale
            orig(b)

        red._launch = spy
        A, B = _data(world)
        red.zero_grad()
        _pix2pix_backward(G, D, A[2 * rank:2 * rank + 2], B[2 * rank:2 * rank + 2])
        red.finish()
        worst = 0.0
        for b in red.buckets:
            gl = [torch.zeros_like(local[b.index]) for _ in range(world)]
            dist.all_gather(gl, local[b.index])
            mean = torch.stack(gl).mean(0)
            # each term is rounded to bf16 once (x/world is exact for power-of-two worlds),
            # and the ring sums world-1 times in bf16: bound by world * 2^-8 of sum |x_r|/world
            bound = world * 2.0 ** -8 * torch.stack(gl).abs().mean(0) + 1e-30
            worst = max(worst, float(((b.flat - mean).abs() / bound).max()))
        opt = torch.optim.Adam(G.parameters(), lr=1e-3)
        opt.step()
        flat = torch.cat([p.detach().reshape(-1) for p in G.parameters()])
        gathered = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(gathered, flat)
        same = all(torch.equal(gathered[0], t) for t in gathered)
        q.put((rank, (worst, same)))
    except Exception:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bf16_comm_within_bound_and_ranks_identical(world):
    for worst, same in _run(world, _bf16_worker):
        assert worst <= 1.0, f"bf16-reduced grad off the fp32 mean by {worst:.2f}x the bound"
        assert same, "parameters diverged across ranks after a bf16-comm step"


def _timing_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from p2p_pytorch_amd.parallel import GradReducer
        from p2p_pytorch_amd.parallel import dist as pdist
        pdist.init_from_env()
        G, D = _build(100)
        red = GradReducer(G, bucket_mb=0.05).enable_timing()
        assert red.comm_stats() == {}                    # nothing timed yet
        A, B = _data(world)
        stats = []
        for _ in range(2):                               # second backward: re-bucketed layout
            red.zero_grad()
            _pix2pix_backward(G, D, A[2 * rank:2 * rank + 2], B[2 * rank:2 * rank + 2])
            red.finish()
            stats.append((red.comm_stats(), len(red.buckets)))
        q.put((rank, stats))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_comm_timing_stats():
    for stats in _run(2, _timing_worker):
        for st, nb in stats:
            assert st["buckets"] == nb > 1, st
            assert st["comm_ms"] > 0.0 and st["exposed_ms"] >= 0.0, st
            assert 0.0 <= st["overlap"] <= 1.0, st
            assert st["exposed_ms"] <= st["comm_ms"] + 1e-6, st


def _train_c_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from p2p_pytorch_amd.engine.compress_gan import CompressGANStep
        from p2p_pytorch_amd.models import VGGLoss, define_C, define_D, define_G
        from p2p_pytorch_amd.parallel import GradReducer
        from p2p_pytorch_amd.parallel import dist as pdist
        pdist.init_from_env()
        torch.manual_seed(100 + rank)
        G = define_G(gpu_id="cpu", verbose=False)
        D = define_D(6, 16, gpu_id="cpu", verbose=False)
        C = define_C(gpu_id="cpu", verbose=False)
        for m in (G, D, C):
            pdist.broadcast_module(m)
        torch.manual_seed(7)
        red_c = GradReducer(C, bucket_mb=0.05)
        launched = []
        orig = red_c._launch
        red_c._launch = lambda b: (launched.append(b.index), orig(b))
        step = CompressGANStep(G, D, C, vgg=VGGLoss(), train_c=True,
                               reducer_g=GradReducer(G, bucket_mb=2.0),
                               reducer_d=GradReducer(D, bucket_mb=2.0), reducer_c=red_c)
        g = torch.Generator().manual_seed(321)
        report = []
        for _ in range(2):
            A = torch.rand(world, 3, 32, 32, generator=g) * 2 - 1
            B = torch.rand(world, 3, 32, 32, generator=g) * 2 - 1
            c0 = torch.cat([p.detach().reshape(-1) for p in C.parameters()]).clone()
            launched.clear()
            step.step(A[rank:rank + 1], B[rank:rank + 1])
            c1 = torch.cat([p.detach().reshape(-1) for p in C.parameters()])
            gathered = [torch.zeros_like(c1) for _ in range(world)]
            dist.all_gather(gathered, c1)
            report.append((not torch.equal(c0, c1), all(torch.equal(gathered[0], t) for t in gathered),
                           sorted(launched) == list(range(len(red_c.buckets)))))
        q.put((rank, report))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_train_c_reduces_c_gradients():
    for report in _run(2, _train_c_worker):
        for trained, same, all_launched in report:
            assert trained, "C did not train with train_c"
            assert all_launched, "not every C bucket was all-reduced exactly once"
            assert same, "C diverged across ranks under data parallelism"


_HANG = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    from p2p_pytorch_amd.utils import StepWatchdog
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo", rank=rank, world_size=2)
    if rank == 0:
        StepWatchdog(timeout_s=2.0, abort_grace_s=2.0).start()
        t = torch.ones(4)
        dist.all_reduce(t)          # rank 1 never joins: blocks until the watchdog fires
        print("collective returned", flush=True)
        sys.exit(3)
    time.sleep(120)                 # the stalled peer
""")


def test_watchdog_exits_while_blocked_in_collective():
    port = _free_port()
    code = _HANG.format(root=ROOT)
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2")
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    try:
        t0 = time.monotonic()
        out, err = procs[0].communicate(timeout=90)
        dt = time.monotonic() - t0
        assert procs[0].returncode == 124, (procs[0].returncode, out, err[-2000:])
        assert b"watchdog" in err
        assert dt < 60, dt
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait(timeout=30)
