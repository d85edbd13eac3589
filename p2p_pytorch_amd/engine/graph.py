"""Whole-training-step hipGraph capture.

A pix2pix step on the native backend is ~450 kernel launches (convs, norms, losses,
weight casts, Adam) driven from Python autograd.  Instead of a tracing compiler the step
is captured ONCE into a HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and
replayed: zero Python / launch overhead, identical kernels and numerics.

Requirements the native path already meets (see ops/hip.py, engine/optim.py):
  * no host synchronisation inside the step (losses stay on the device; the data-parallel
    reducer's collectives are stream-ordered, so RCCL all-reduces are captured too);
  * per-step state that must change between replays lives in device memory: the Adam
    step counter and learning rate (FusedAdam), the dropout seed (``hip.advance_rng``);
  * bf16 weight images are re-cast inside the captured region (``hip.begin_step``).

Warmup: capture needs a few real steps first (allocator pools, the reducer's ready-order
re-bucketing, fp8 scale bootstraps).  When the trainer exposes ``state_tensors()`` every
tensor a step mutates (parameters, buffers, optimizer moments and counters, RNG seeds,
guard counters) is snapshotted before the warmup and restored before the capture, so
replay k is exactly eager step k from the same initial state -- the warmup trains nothing
(tests/test_graph_gpu.py pins this bitwise in deterministic mode).
New input batches are copied into the static input buffers before each replay.
"""
from __future__ import annotations

import copy

import torch


# ProcessGroupNCCL's watchdog polls the end events of the eager collectives it tracks every
# ~100 ms (kWatchdogThreadSleepMillis) and only then retires them
_WATCHDOG_DRAIN_S = 0.35


def drain_collectives():
    """Let the c10d watchdog retire every eager collective before a capture begins.

    The capture's first collective makes the process group's RCCL stream join the capture.
    On HIP, ``hipEventQuery`` of an event recorded on a stream that is NOW capturing fails
    with ``hipErrorCapturedEvent`` -- and the watchdog still holds the end events of the
    warmup steps' all-reduces until its next poll, so a capture that starts within one poll
    interval of them aborts the process (tools/diag_capture_event.py
    reproduces it with one rank).  A device sync completes those Works; sleeping a few poll
    intervals lets the watchdog retire them."""
    import time

    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    if dist.get_backend() != "nccl":
        return
    torch.cuda.synchronize()
    time.sleep(_WATCHDOG_DRAIN_S)


class WarmupError(RuntimeError):
    """A warmup (eager) step raised before capture: not a capture failure -- the trainer
    itself is broken, and on a multi-rank job the other ranks are already blocked in that
    step's collectives, so the process must exit (the launcher restarts the job)."""


class CaptureError(RuntimeError):
    """``torch.cuda.graph`` raised while recording; the pre-warmup state (tensors, optimizer
    step counts, the dropout salt counter) has been restored, so eager can take over."""


def trainer_state_tensors(modules, optimizers, extra=()):
    """Every tensor a training step mutates in place: parameters and buffers of
    ``modules``, the optimizer state (moments, device step / lr counters) and ``extra``."""
    out, seen = [], set()

    def add(t):
        if isinstance(t, torch.Tensor) and id(t) not in seen:
            seen.add(id(t))
            out.append(t)

    for m in modules:
        if m is None:
            continue
        for t in m.parameters():
            add(t)          # the Parameter itself (``.data`` is a fresh object per access)
        for t in m.buffers():
            add(t)
    for opt in optimizers:
        if opt is None:
            continue
        for st in opt.state.values():
            for v in st.values():
                add(v)
        for t in getattr(opt, "_step_t", []):
            add(t)
    for t in extra:
        add(t)
    return out


class _Snapshot:
    def __init__(self, trainer):
        self.trainer = trainer
        self.tensors = list(trainer.state_tensors())
        self.saved = [t.detach().clone() for t in self.tensors]
        # python-side optimizer step counts (reported by state_dict only)
        self.py_steps = []
        for opt in getattr(trainer, "optimizers", lambda: [])():
            if opt is not None:
                self.py_steps.append((opt, {k: dict(st).get("step") for k, st in opt.state.items()}))

    def restore(self):
        now = list(self.trainer.state_tensors())
        if len(now) != len(self.tensors) or any(a is not b for a, b in zip(now, self.tensors)):
            raise RuntimeError("CapturedStep: the trainer's state tensors changed identity "
                               "during warmup; cannot restore the pre-warmup state")
        with torch.no_grad():
            for t, s in zip(self.tensors, self.saved):
                t.copy_(s)
        for opt, steps in self.py_steps:
            for k, v in steps.items():
                if v is not None and k in opt.state:
                    opt.state[k]["step"] = v


class CapturedStep:
    def __init__(self, step_fn, *example_inputs, warmup: int = 2, restore: bool = True):
        self.step_fn = step_fn
        self.static_inputs = [x.clone() for x in example_inputs]
        trainer = getattr(step_fn, "__self__", None)
        snap = None
        if restore and trainer is not None and hasattr(trainer, "state_tensors"):
            torch.cuda.synchronize()
            snap = _Snapshot(trainer)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        try:
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):
                    step_fn(*self.static_inputs)
        except Exception as e:  # noqa: BLE001
            raise WarmupError(f"warmup step failed: {type(e).__name__}: {e}") from e
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if snap is not None:
            snap.restore()
            torch.cuda.synchronize()
        drain_collectives()               # no eager RCCL Work left for the watchdog to poll
        # the capture allocates from a private pool that cannot reuse the caching allocator's
        # free blocks: hand the warmup's cached activations back first, so the captured step
        # needs about one step's memory, not two (HBM-sized batches: 3072 bf16 / 2048 fp8)
        from ..ops import hip as _hip
        _hip.release_handoffs()           # (their entries pin the warmup step's activations)
        torch.cuda.empty_cache()
        salt = copy.copy(_hip._salt)      # python-side state the capture advances
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph):
                self.static_out = step_fn(*self.static_inputs)
        except Exception as e:  # noqa: BLE001
            torch.cuda.synchronize()
            if snap is not None:
                snap.restore()
                torch.cuda.synchronize()
            _hip._salt = salt
            raise CaptureError(f"{type(e).__name__}: {e}") from e
        torch.cuda.synchronize()

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out


def capture_agreed(step_fn, *example_inputs, warmup: int = 2, log=None, info=None):
    """Capture ``step_fn`` as a :class:`CapturedStep` when it is safe on every rank, else run
    eager on every rank.  Returns ``(step, captured)``.

    * Only RCCL process groups are captured at world > 1: gloo (the CPU / one-GPU rehearsal
      backend) stages collectives through the host and cannot be captured, and a failed
      capture can leave the process in capture mode.
    * A failure DURING capture (``torch.cuda.graph`` raised, :class:`CaptureError`) on ANY
      rank makes every rank fall back to eager (``min_scalar`` consensus): collectives must
      match, so one rank replaying a graph while another runs eager would hang until the
      watchdog.  The failing capture restored the pre-warmup state first, so the fallback
      ranks and the ranks whose capture succeeded start eager from the same state.
    * Only capture failures are agreed: a WARMUP step that raises (:class:`WarmupError`) is
      re-raised -- the other ranks are blocked in that step's gradient all-reduces, a
      min_scalar would be matched against a bucket collective, so the process exits non-zero
      and the launcher (``torchrun --max-restarts``) / watchdog handles the restart.

    ``info`` (optional dict) receives ``capture_error``: this rank's capture exception as a
    string (None when it captured), so a caller's report can say WHY a run was eager.
    """
    from ..parallel import dist as pdist
    world = pdist.world_size()
    dev = example_inputs[0].device
    if dev.type != "cuda" or (world > 1 and pdist.backend() != "nccl"):
        return step_fn, False
    ok, step = 1.0, step_fn
    if info is not None:
        info["capture_error"] = None
    try:
        step = CapturedStep(step_fn, *example_inputs, warmup=warmup)
    except WarmupError:
        raise
    except Exception as e:  # noqa: BLE001 - a capture failure: eager on every rank
        if log is not None:
            log(f"graph capture failed ({type(e).__name__}: {e}); running eager")
        if info is not None:
            info["capture_error"] = f"{type(e).__name__}: {e}"[:400]
        ok = 0.0
    if world > 1:
        ok = pdist.min_scalar(ok, dev)
    if ok < 1.0:
        if info is not None and info["capture_error"] is None:
            info["capture_error"] = "another rank's capture failed"
        return step_fn, False
    return step, True
