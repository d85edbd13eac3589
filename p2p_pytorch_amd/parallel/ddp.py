"""Bucketed gradient all-reduce overlapped with backward (RCCL over xGMI).

Why not ``DistributedDataParallel``: one pix2pix step runs D three times and G once,
with two optimizers and D frozen in the G phase; the
reference-family step even back-propagates the G loss through D and then throws those D
gradients away (/root/reference/train.py:384-389).  DDP's forward-coupled hooks mis-fire
on that pattern; here every network has its own reducer and the trainer says explicitly
when a backward starts (``zero_grad``), when one must not be reduced (``paused``) and when
one is complete (``finish``).

Mechanism
  * Parameters are packed into flat fp32 buckets of ``bucket_mb`` -- first in reverse
    registration order, then (after the first backward) in the order their grads actually
    became ready, with the last-ready bucket capped at ``tail_mb`` (its all-reduce is the
    one backward cannot hide).  Rank 0's recorded order is broadcast, so every rank builds
    the same layout even when autograd's ready order differs between ranks.  Each
    ``p.grad`` is a *view* into its bucket, so autograd accumulates straight into
    communication memory -- no gather/scatter copies.
  * ``register_post_accumulate_grad_hook`` counts ready params; the moment a bucket is
    complete its ``all_reduce`` is enqueued (async).  RCCL runs it on its own HIP stream,
    ordered after the producing kernels by an event, so it overlaps the rest of backward.
  * Per-backward state (pending counts, in-flight work) is reset by ``zero_grad`` -- which
    first joins any collective still in flight, so zeroing never races a reduction -- and by
    ``finish``.  A gradient that arrives for a bucket already sent raises instead of being
    silently half-reduced.
  * ``paused()``: a backward whose gradients will be discarded (the reference's D grads
    from the G loss, the C-phase backward) launches no collective.
  * Averaging (round 5): on RCCL the bucket all-reduce is
    ``ReduceOp.AVG`` (ncclAvg: the division happens inside the collective) at every world
    size, force_comm world 1 included (round 6), so no gradient
    is ever rescaled on the compute stream -- the round-4 reducer issued one ``mul_(1/world)``
    per parameter in its hook (~130 extra launches per step at world 8).  Process groups
    without AVG (gloo: the CPU / one-GPU rehearsal backend) sum and scale each BUCKET once in
    ``finish``.
  * ``comm_dtype=torch.bfloat16``: the bucket is copied into a bf16 comm buffer, averaged in
    bf16 (half the xGMI bytes) and widened back into the fp32 grads by ``finish``.
  * ``finish()`` enqueues any incomplete bucket (params that got no grad contribute
    zeros) and makes the compute stream wait on every collective (no host sync).  Nothing in ``_on_grad`` / ``finish`` synchronises the host, so a step with
    reducers can be captured into one hipGraph (RCCL collectives are graph-capturable).
  * ``force_comm=True`` issues the collectives even at world size 1 (exercises the RCCL
    and capture path on a single GPU).
  * ``enable_timing()`` (logging only): collectives are issued from a side stream
    bracketed by HIP events (CPU / gloo groups: host clock from launch to the collective's
    completion callback), and ``comm_stats()`` reports the last backward's collective
    busy time, the part of it left exposed after backward's last kernel, and the overlap
    fraction -- the JSONL "comm ms / overlap %" of SURVEY.md section 5.5.
  * Direct gradients (``direct=True``, round 4): the native conv backward writes a conv
    weight's gradient straight into its bucket view with the wgrad kernel's own
    accumulate mode -- no AccumulateGrad add -- and may
    run it on the weight-gradient side stream (ops/hip.py ``wgrad_overlap``).  Readiness
    still comes from autograd: a leaf's post-accumulate hook fires once per backward after all
    of its producers ran, also when they all returned None because they wrote the bucket
    themselves; ``direct_done`` only records the side-stream event the bucket's all-reduce
    must wait on (it is issued from a comm stream that waits on both streams) and marks the
    param as written.  Nothing is pre-scaled (the collective averages), so a direct write and
    an autograd contribution to the same bucket mix freely.  Default on since round 5
    (``P2P_DIRECT_GRAD=0`` turns it off): step A/B with RCCL collectives at world 1 --
    direct 7849 / 7839, autograd 7838, no reducer 7870 img/s (profiles/force_comm_r5k.jsonl).
    The round-4 watchdog abort seen with it was a capture started while the c10d watchdog
    still tracked the warmup's eager all-reduces; since round 6 the captured collectives run on
    a fresh process group (engine/graph.py ``isolate_capture_collectives``).
  * Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per GPU); RCCL's ring /
    direct algorithms are per-link bound, so few large buckets (tens of MB) amortise the
    per-collective latency while still leaving >= 2-4 buckets per network to overlap.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time

import torch
import torch.distributed as dist


_DEBUG = os.environ.get("P2P_DDP_DEBUG", "0") == "1"


class _Bucket:
    __slots__ = ("params", "flat", "cbuf", "pending", "work", "index", "events", "side")

    def __init__(self, params, device, dtype, index, comm_dtype):
        self.params = params
        n = sum(p.numel() for p in params)
        self.flat = torch.zeros(n, device=device, dtype=dtype)
        self.cbuf = (torch.empty(n, device=device, dtype=comm_dtype)
                     if comm_dtype is not None and comm_dtype != dtype else None)
        self.pending = len(params)
        self.work = None
        self.index = index
        self.events = None
        self.side = []        # events of direct gradient writes enqueued on other streams


class _StreamJoin:
    """Work handle of a timed collective: waiting = ordering the current stream after the
    side stream that issued it."""
    __slots__ = ("stream",)

    def __init__(self, stream):
        self.stream = stream

    def wait(self):
        torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)


class _HostEvent:
    """Host-clock stand-in for a timing HIP event on CPU (gloo) process groups: ``record`` now,
    or ``record`` from a collective's completion callback; ``elapsed_time`` in ms."""
    __slots__ = ("t", "_done")

    def __init__(self):
        self.t = None
        self._done = threading.Event()

    def record(self, *_):
        self.t = time.perf_counter()
        self._done.set()
        return self

    def synchronize(self):
        if not self._done.wait(timeout=60.0):
            raise RuntimeError("GradReducer timing: a collective never completed")

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class GradReducer:
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 64.0, process_group=None,
                 comm_dtype: torch.dtype | None = None, tail_mb: float = 8.0, rebucket: bool = True,
                 force_comm: bool = False, direct: bool | None = None):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(process_group) if dist.is_initialized() else None
        self.comm = dist.is_initialized() and (self.world > 1 or force_comm)
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = params
        self.comm_dtype = comm_dtype if self.comm else None
        self.cap = int(bucket_mb * 1024 * 1024)
        self.tail_cap = min(self.cap, int(tail_mb * 1024 * 1024))
        self._build(list(reversed(params)))
        # the first backward records the order grads actually become ready; the next
        # zero_grad() re-buckets in that order (DDP's bucket rebuild), so every bucket fills
        # contiguously in time and the last-ready one -- the all-reduce nothing can hide --
        # is capped at tail_mb
        self._ready_order: list | None = [] if rebucket else None
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]
        self.active = True
        self._timing = False
        self._comm_stream = None
        # the stream the step's backward runs on, taken at zero_grad() on the step's thread:
        # autograd may run a leaf's post-accumulate hook on ANOTHER stream (a leaf whose
        # producers all returned None -- direct gradients -- gets no stream sync), so the
        # collectives are ordered and capture-checked against this one, not the hook's
        self._compute_stream = None
        self._last = None        # (bucket events, end-of-backward event) of the last finish()
        # gradients land unscaled (direct writes and autograd alike): RCCL averages inside the
        # collective (ReduceOp.AVG); other backends sum and scale each bucket once in finish()
        self.scale = 1.0
        # RCCL: ReduceOp.AVG at EVERY world size -- with force_comm at world 1 (the identity
        # average) the one-GPU tests and A/Bs run the exact op, dtype and capture path of a
        # world-8 job
        self._avg = self.comm and self.backend == "nccl"
        self._post_scale = (1.0 / self.world) if (self.comm and self.world > 1 and not self._avg) else None
        if direct is None:   # default on: bitwise equal to the autograd path (tools/ddp_rehearsal.py)
            direct = os.environ.get("P2P_DIRECT_GRAD", "1") == "1"
        self.direct = bool(direct)
        self._direct_seen: set = set()   # params written directly in the current backward
        self._names = {id(p): n for n, p in module.named_parameters()}
        if self.direct:
            for p in params:
                p._p2p_direct = self

    def _build(self, order):
        self.buckets: list[_Bucket] = []
        self._param_bucket = {}
        self._offset = {}
        groups, cur, cur_bytes = [], [], 0
        # pack from the END of the ready order so the last-ready bucket gets the small cap
        for p in reversed(order):
            nbytes = p.numel() * p.element_size()
            cap = self.tail_cap if not groups else self.cap
            if cur and (cur_bytes + nbytes > cap or p.dtype != cur[0].dtype):
                groups.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nbytes
        if cur:
            groups.append(cur)
        for g in reversed(groups):
            self._add_bucket(list(reversed(g)))

    def _agreed_order(self, order):
        """Rank 0's ready order, as parameter indices, on every rank."""
        if not self.comm:
            return order
        index = {id(p): i for i, p in enumerate(self.params)}
        dev = self.params[0].device
        if self.backend == "nccl" and dev.type != "cuda":
            dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([index[id(p)] for p in order], dtype=torch.int64, device=dev)
        src = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
        dist.broadcast(t, src, group=self.pg)
        return [self.params[i] for i in t.tolist()]

    def _rebucket(self):
        order = self._ready_order
        self._ready_order = None
        seen = set(id(p) for p in order)
        order = order + [p for p in reversed(self.params) if id(p) not in seen]
        order = self._agreed_order(order)
        old = {id(p): p.grad for p in self.params}
        self._build(order)
        for p in self.params:   # carry current grads over into the new flat buckets
            if old[id(p)] is not None:
                p.grad.copy_(old[id(p)])

    def _add_bucket(self, params):
        b = _Bucket(params, params[0].device, params[0].dtype, len(self.buckets), self.comm_dtype)
        off = 0
        for p in params:
            n = p.numel()
            p.grad = b.flat[off:off + n].view_as(p)
            self._param_bucket[p] = b
            self._offset[p] = off
            off += n
        self.buckets.append(b)

    # ------------------------------------------------------------------ hooks
    def _on_grad(self, p):
        if not self.active:
            return
        b = self._param_bucket[p]
        if b.work is not None:
            raise RuntimeError(
                "GradReducer: a gradient arrived for a bucket whose all-reduce was already "
                "launched (a second backward without zero_grad()/finish(); wrap backwards whose "
                f"gradients are discarded in reducer.paused()): parameter "
                f"{self._names.get(id(p), '?')} {tuple(p.shape)}, bucket {b.index} of "
                f"{len(self.buckets)} ({len(b.params)} params)")
        if self._ready_order is not None:
            self._ready_order.append(p)
        # autograd may have replaced the view (e.g. after set_to_none): copy back in.
        lo = b.flat.data_ptr()
        if not (lo <= p.grad.data_ptr() < lo + b.flat.numel() * b.flat.element_size()):
            self._rebind(p, b, copy=True)
        if id(p) not in self._direct_seen:
            if p.grad.is_cuda:
                hs = torch.cuda.current_stream(p.grad.device)
                if hs != self._stream(p.grad.device):
                    # accumulated on the leaf's own stream: the collective waits on it
                    ev = torch.cuda.Event()
                    ev.record(hs)
                    b.side.append(ev)
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    # ------------------------------------------------------------------ direct gradients
    def direct_ok(self, p) -> bool:
        """The backward may write ``p``'s gradient into its bucket view itself."""
        if not (self.direct and self.active) or p.grad is None:
            return False
        b = self._param_bucket.get(p)
        if b is None or b.work is not None:
            return False
        lo = b.flat.data_ptr()
        return lo <= p.grad.data_ptr() < lo + b.flat.numel() * b.flat.element_size()

    def direct_done(self, p, stream=None):
        """A direct contribution to ``p.grad`` has been enqueued (on ``stream``, default the
        current one).  Readiness still comes from autograd: its post-accumulate hook fires once
        per backward for every leaf the backward reached -- also when every contribution was
        None (written here) -- after all of that leaf's producers ran."""
        b = self._param_bucket[p]
        if _DEBUG:
            with torch.cuda.stream(stream or torch.cuda.current_stream()):
                cap = torch.cuda.is_current_stream_capturing()
            print(f"[reducer] direct {self._names.get(id(p), '?')} bucket {b.index}: stream "
                  f"{None if stream is None else stream.stream_id} capturing {cap}", flush=True)
        if stream is not None and stream != self._stream(stream.device):
            ev = torch.cuda.Event()
            ev.record(stream)
            b.side.append(ev)
        self._direct_seen.add(id(p))

    def _stream(self, device):
        """The step's compute stream (see ``_compute_stream``)."""
        if self._compute_stream is None or self._compute_stream.device != device:
            return torch.cuda.current_stream(device)
        return self._compute_stream

    def _rebind(self, p, b, copy):
        off = self._offset[p]
        dst = b.flat[off:off + p.numel()].view_as(p)
        if copy:
            dst.copy_(p.grad)
        p.grad = dst

    def set_group(self, pg):
        """Issue this reducer's collectives on ``pg`` from now on (same ranks and backend):
        ``CapturedStep`` moves the reducers onto a fresh capture group before recording
        (``parallel.dist.capture_group``)."""
        if self.comm:
            if dist.get_world_size(pg) != self.world or dist.get_backend(pg) != self.backend:
                raise ValueError("GradReducer.set_group: the group must span the same ranks and backend")
            self._join_inflight()
            self.pg = pg
        return self

    def _op(self):
        return dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM

    def _launch(self, b: _Bucket):
        if b.work is not None:
            return
        if not self.comm:
            b.work = True
            return
        if self._timing and not b.flat.is_cuda:
            # CPU process group: host clock from the launch to the collective's completion
            # callback (gloo completes it on its own thread while backward continues)
            buf = b.flat
            if b.cbuf is not None:
                b.cbuf.copy_(b.flat)
                buf = b.cbuf
            e0, e1 = _HostEvent().record(), _HostEvent()
            b.work = dist.all_reduce(buf, op=self._op(), group=self.pg, async_op=True)
            b.work.get_future().then(lambda _f, e=e1: e.record())
            b.events = (e0, e1)
            return
        cur = self._stream(b.flat.device) if b.flat.is_cuda else None
        capturing = False
        if cur is not None:
            with torch.cuda.stream(cur):
                capturing = torch.cuda.is_current_stream_capturing()
        timed = self._timing and not capturing and b.flat.is_cuda
        if _DEBUG and cur is not None:
            hs = torch.cuda.current_stream(b.flat.device)
            print(f"[reducer] bucket {b.index}: thread {threading.get_ident()} hook stream "
                  f"{hs.stream_id} compute stream {cur.stream_id} capturing {capturing} "
                  f"hook-stream capturing {torch.cuda.is_current_stream_capturing()} "
                  f"side events {len(b.side)}", flush=True)
        side = b.flat.is_cuda and bool(b.side) and not capturing
        if capturing and b.side:
            # under hipGraph capture the collective stays on the capturing stream (RCCL work
            # issued from a joined side stream trips the process-group watchdog's event
            # queries): that stream waits on the side-stream gradient writes instead
            for ev in b.side:
                cur.wait_event(ev)
        if timed or side:
            # a comm stream ordered after the compute stream AND the side-stream gradient
            # writes of this bucket (their events), so the compute stream itself never waits
            if self._comm_stream is None:
                self._comm_stream = torch.cuda.Stream(device=b.flat.device)
            cs = self._comm_stream
            cs.wait_stream(cur)
            for ev in b.side:
                cs.wait_event(ev)
            ctx = torch.cuda.stream(cs)
        else:
            ctx = torch.cuda.stream(cur) if cur is not None else contextlib.nullcontext()
        with ctx:
            buf = b.flat
            if b.cbuf is not None:
                b.cbuf.copy_(b.flat)            # the narrow comm buffer
                buf = b.cbuf
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(cs)
                work = dist.all_reduce(buf, op=self._op(), group=self.pg, async_op=True)
                work.wait()                     # cs waits for RCCL's stream (no host sync)
                e1.record(cs)
                b.flat.record_stream(cs)
                if b.cbuf is not None:
                    b.cbuf.record_stream(cs)
                b.events = (e0, e1)
                b.work = _StreamJoin(cs)
            elif side:
                work = dist.all_reduce(buf, op=self._op(), group=self.pg, async_op=True)
                work.wait()                     # cs waits for RCCL's stream (no host sync)
                b.work = _StreamJoin(cs)
            else:
                if _DEBUG:
                    print(f"[reducer] bucket {b.index}: all_reduce on stream "
                          f"{torch.cuda.current_stream().stream_id if buf.is_cuda else None} capturing "
                          f"{buf.is_cuda and torch.cuda.is_current_stream_capturing()}", flush=True)
                b.work = dist.all_reduce(buf, op=self._op(), group=self.pg, async_op=True)

    def _reset(self):
        for b in self.buckets:
            b.work = None
            b.events = None
            b.side = []
            b.pending = len(b.params)
        self._direct_seen = set()

    def _join_inflight(self):
        # collectives launched but never finished (e.g. a backward abandoned by an
        # exception): order the current stream after them before anything reuses the buckets
        for b in self.buckets:
            if b.work is not None and b.work is not True:
                b.work.wait()

    # ------------------------------------------------------------------ API
    @contextlib.contextmanager
    def paused(self):
        """Backwards run inside launch no collective and leave the bookkeeping alone (their
        gradients are discarded by the next ``zero_grad``)."""
        prev, self.active = self.active, False
        try:
            yield self
        finally:
            self.active = prev

    def finish(self):
        """Complete the reduction of this backward: launch stragglers, wait (stream-ordered),
        average, and reset bookkeeping for the next backward."""
        end_bwd = None
        if self._timing and self.comm and self.buckets:
            if not self.buckets[0].flat.is_cuda:
                end_bwd = _HostEvent().record()
            elif not torch.cuda.is_current_stream_capturing():
                end_bwd = torch.cuda.Event(enable_timing=True)
                end_bwd.record()
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        if end_bwd is not None:
            self._last = ([b.events for b in self.buckets if b.events is not None], end_bwd)
        for b in self.buckets:
            if b.work is not True and b.work is not None:
                b.work.wait()
            elif b.side:
                # no collective (world 1): order the compute stream after the side writes
                for ev in b.side:
                    self._stream(b.flat.device).wait_event(ev)
            if b.cbuf is not None:
                b.flat.copy_(b.cbuf)            # averaged by the collective
            if self._post_scale is not None and b.work is not None and b.work is not True:
                b.flat.mul_(self._post_scale)   # SUM backends: one scale per bucket
        self._reset()

    def enable_timing(self, on: bool = True):
        self._timing = bool(on)
        return self

    def comm_stats(self) -> dict:
        """Collective timing of the last timed backward (host-synchronises on its events):
        ``comm_ms`` = busy time of the bucket all-reduces (union of their intervals),
        ``exposed_ms`` = how long they ran past the end of backward's compute,
        ``overlap`` = 1 - exposed / comm."""
        if not self._last or not self._last[0]:
            return {}
        evs, end_bwd = self._last
        for _, e1 in evs:
            e1.synchronize()
        end_bwd.synchronize()
        ref = evs[0][0]
        spans = sorted((ref.elapsed_time(e0), ref.elapsed_time(e1)) for e0, e1 in evs)
        busy, cur_s, cur_e = 0.0, None, None
        for s0, s1 in spans:
            if cur_e is None or s0 > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s0, s1
            else:
                cur_e = max(cur_e, s1)
        busy += cur_e - cur_s
        t_end = ref.elapsed_time(end_bwd)
        exposed = max(0.0, max(s1 for _, s1 in spans) - t_end)
        return {"comm_ms": busy, "exposed_ms": exposed,
                "overlap": 1.0 - exposed / busy if busy > 0 else 1.0, "buckets": len(spans)}

    def all_reduce_max_(self, t: torch.Tensor):
        """In-place MAX over ranks of a small device tensor (e.g. the NaN-guard flag), so
        every rank takes the same skip decision."""
        if self.comm and self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.pg)
        return t

    def zero_grad(self):
        """Start a backward: join stale collectives, (re-bucket once), zero the buckets and
        reset the per-backward bookkeeping."""
        self._join_inflight()
        if self.buckets and self.buckets[0].flat.is_cuda:
            self._compute_stream = torch.cuda.current_stream(self.buckets[0].flat.device)
        if self._ready_order:
            self._rebucket()
        for b in self.buckets:
            b.flat.zero_()
            lo = b.flat.data_ptr()
            hi = lo + b.flat.numel() * b.flat.element_size()
            for p in b.params:  # keep grads as bucket views (set_to_none / foreign grads)
                if p.grad is None or not (lo <= p.grad.data_ptr() < hi):
                    self._rebind(p, b, copy=False)
        self._reset()

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for p in self.params:
            if getattr(p, "_p2p_direct", None) is self:
                del p._p2p_direct
