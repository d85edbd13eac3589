"""Bucketed gradient all-reduce overlapped with backward (RCCL over xGMI).

Why not ``DistributedDataParallel``: one pix2pix step runs D three times and G once,
with two optimizers and D frozen in the G phase.  DDP's
forward-coupled hooks mis-fire on that pattern; here every network has its own reducer
and the trainer says explicitly when a backward is complete (``finish``).

Mechanism
  * Parameters are packed into flat fp32 buckets of ``bucket_mb`` -- first in reverse
    registration order, then (after the first backward) in the order their grads actually
    became ready, with the last-ready bucket capped at ``tail_mb`` (its all-reduce is the
    one backward cannot hide).  Each ``p.grad`` is a *view*
    into its bucket, so autograd accumulates straight into communication memory --
    no gather/scatter copies.
  * ``register_post_accumulate_grad_hook`` counts ready params; the moment a bucket is
    complete its ``all_reduce`` is enqueued (async).  RCCL runs it on its own HIP stream,
    ordered after the producing kernels by an event, so it overlaps the rest of backward.
  * ``finish()`` enqueues any incomplete bucket (params that got no grad contribute
    zeros), makes the compute stream wait on every collective (no host sync) and scales
    by 1/world.
  * ``enable_timing()`` (logging only): collectives are issued from a side stream
    bracketed by HIP events, and ``comm_stats()`` reports the last backward's collective
    busy time, the part of it left exposed after backward's last kernel, and the overlap
    fraction -- the JSONL "comm ms / overlap %" of SURVEY.md section 5.5.
  * Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per GPU); RCCL's ring /
    direct algorithms are per-link bound, so few large buckets (tens of MB) amortise the
    per-collective latency while still leaving >= 2-4 buckets per network to overlap.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class _Bucket:
    __slots__ = ("params", "flat", "pending", "work", "index", "events")

    def __init__(self, params, device, dtype, index):
        self.params = params
        n = sum(p.numel() for p in params)
        self.flat = torch.zeros(n, device=device, dtype=dtype)
        self.pending = len(params)
        self.work = None
        self.index = index
        self.events = None


class _StreamJoin:
    """Work handle of a timed collective: waiting = ordering the current stream after the
    side stream that issued it."""
    __slots__ = ("stream",)

    def __init__(self, stream):
        self.stream = stream

    def wait(self):
        torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)


class GradReducer:
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 64.0, process_group=None,
                 comm_dtype: torch.dtype | None = None, tail_mb: float = 8.0, rebucket: bool = True):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(process_group) if dist.is_initialized() else None
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = params
        self.cap = int(bucket_mb * 1024 * 1024)
        self.tail_cap = min(self.cap, int(tail_mb * 1024 * 1024))
        self._build(list(reversed(params)))
        # the first backward records the order grads actually become ready; the next
        # zero_grad() re-buckets in that order (DDP's bucket rebuild), so every bucket fills
        # contiguously in time and the last-ready one -- the all-reduce nothing can hide --
        # is capped at tail_mb
        self._ready_order: list | None = [] if rebucket else None
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]
        self.comm_dtype = comm_dtype
        self.active = True
        self._timing = False
        self._comm_stream = None
        self._last = None        # (bucket events, end-of-backward event) of the last finish()

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

    def _rebucket(self):
        order = self._ready_order
        self._ready_order = None
        seen = set(id(p) for p in order)
        order = order + [p for p in reversed(self.params) if id(p) not in seen]
        old = {id(p): p.grad for p in self.params}
        self._build(order)
        for p in self.params:   # carry current grads over into the new flat buckets
            if old[id(p)] is not None:
                p.grad.copy_(old[id(p)])

    def _add_bucket(self, params):
        b = _Bucket(params, params[0].device, params[0].dtype, len(self.buckets))
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
        if self._ready_order is not None:
            self._ready_order.append(p)
        b = self._param_bucket[p]
        # autograd may have replaced the view (e.g. after set_to_none): copy back in.
        lo = b.flat.data_ptr()
        if not (lo <= p.grad.data_ptr() < lo + b.flat.numel() * b.flat.element_size()):
            self._rebind(p, b, copy=True)
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _rebind(self, p, b, copy):
        off = self._offset[p]
        dst = b.flat[off:off + p.numel()].view_as(p)
        if copy:
            dst.copy_(p.grad)
        p.grad = dst

    def _launch(self, b: _Bucket):
        if b.work is not None:
            return
        if self.world == 1:
            b.work = True
            return
        if not self._timing or torch.cuda.is_current_stream_capturing() or not b.flat.is_cuda:
            b.work = dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            return
        # timed: issue from a side stream so the events bracket the collective itself
        cur = torch.cuda.current_stream(b.flat.device)
        if self._comm_stream is None:
            self._comm_stream = torch.cuda.Stream(device=b.flat.device)
        cs = self._comm_stream
        cs.wait_stream(cur)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(cs):
            e0.record(cs)
            work = dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            work.wait()                     # cs waits for RCCL's stream (no host sync)
            e1.record(cs)
        b.flat.record_stream(cs)
        b.events = (e0, e1)
        b.work = _StreamJoin(cs)

    # ------------------------------------------------------------------ API
    def finish(self):
        """Complete the reduction of this backward: launch stragglers, wait (stream-ordered),
        average, and reset bookkeeping for the next backward."""
        end_bwd = None
        if self._timing and self.world > 1 and self.buckets and self.buckets[0].flat.is_cuda \
                and not torch.cuda.is_current_stream_capturing():
            end_bwd = torch.cuda.Event(enable_timing=True)
            end_bwd.record()
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        if end_bwd is not None:
            self._last = ([b.events for b in self.buckets if b.events is not None], end_bwd)
        inv = 1.0 / self.world
        for b in self.buckets:
            if b.work is not True and b.work is not None:
                b.work.wait()
            if self.world > 1:
                b.flat.mul_(inv)
            b.work = None
            b.events = None
            b.pending = len(b.params)

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
        evs[-1][1].synchronize()
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
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.pg)
        return t

    def zero_grad(self):
        if self._ready_order:
            self._rebucket()
        for b in self.buckets:
            b.flat.zero_()
            for p in b.params:  # keep grads as bucket views
                if p.grad is None:
                    self._rebind(p, b, copy=False)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
