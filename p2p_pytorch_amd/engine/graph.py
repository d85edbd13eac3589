"""Whole-training-step hipGraph capture.

A pix2pix step on the native backend is ~450 kernel launches (convs, norms, losses,
weight casts, Adam) driven from Python autograd.  Instead of a tracing compiler the step
is captured ONCE into a HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and
replayed: zero Python / launch overhead, identical kernels and numerics.

Requirements the native path already meets (see ops/hip.py, engine/optim.py):
  * no host synchronisation inside the step (losses stay on the device);
  * per-step state that must change between replays lives in device memory: the Adam
    step counter and learning rate (FusedAdam), the dropout seed (``hip.advance_rng``);
  * bf16 weight images are re-cast inside the captured region (``hip.begin_step``).
New input batches are copied into the static input buffers before each replay.
Multi-GPU runs use the eager path (RCCL collectives are launched from the reducer hooks).
"""
from __future__ import annotations

import torch


class CapturedStep:
    def __init__(self, step_fn, *example_inputs, warmup: int = 2):
        self.step_fn = step_fn
        self.static_inputs = [x.clone() for x in example_inputs]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                step_fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_out = step_fn(*self.static_inputs)
        torch.cuda.synchronize()

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out
