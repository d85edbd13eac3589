"""Minimal reproduction of the c10d watchdog abort ``hipErrorCapturedEvent``.

Hypothesis: the ProcessGroupNCCL watchdog polls the end events of EAGER collectives it
still tracks (every ~100 ms).  When a hipGraph capture starts before the watchdog has
retired the last eager collective, the capture's first collective makes the process
group's RCCL stream join the capture -- and HIP's ``hipEventQuery`` on an event whose
recording stream is NOW capturing fails with "operation not permitted on an event last
recorded in a capturing stream", which the watchdog turns into an abort.  (CUDA answers
such a query normally; the failure depends on how close the capture follows the last eager
collective, hence the intermittency of the direct-gradient bench runs.)

    python tools/diag_capture_event.py --mode isolated  # capture on a fresh group (the fix, round 6)
    python tools/diag_capture_event.py --mode race      # capture right behind a pending eager all-reduce

One rank, RCCL.  ``race``: a ~0.3 s GEMM chain keeps the eager all-reduce pending while the
capture (which holds another all-reduce) runs on the SAME group.  ``isolated``: the same
eager all-reduce, but the capture records its all-reduce on ``parallel.dist.capture_group()``
-- a group with no eager history, as ``CapturedStep`` does since round 6 -- with no drain, no
sync and no sleep between them (``tests/test_capture_group_gpu.py`` runs this mode).  Exit 0 = the watchdog never tripped; the
abort kills the process (SIGABRT) otherwise.
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["race", "isolated"], default="isolated")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--capture-mode", default="thread_local", choices=["global", "thread_local", "relaxed"],
                    help="torch.cuda.graph capture_error_mode: under 'global' HIP refuses the watchdog "
                         "thread's hipEventQuery of ANY eager Work while the capture runs")
    args = ap.parse_args()
    from p2p_pytorch_amd.parallel import dist as pdist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pdist.init_single(dev)
    x = torch.ones(1 << 16, device=dev)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    for rnd in range(args.rounds):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(200):                    # ~0.3 s of GEMMs ahead of the collective
                a = (a @ a).clamp_(-1, 1)
            dist.all_reduce(x)                      # eager: tracked by the watchdog
        torch.cuda.current_stream().wait_stream(s)
        pg = pdist.capture_group() if args.mode == "isolated" else None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=args.capture_mode):
            w = dist.all_reduce(x, op=dist.ReduceOp.AVG, group=pg, async_op=True)   # captured: its RCCL stream joins
            w.wait()
            time.sleep(0.5)                         # the watchdog polls while capturing
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(x, torch.ones_like(x)), "world-1 all-reduce changed the tensor"
        print(f"round {rnd}: ok ({args.mode})", flush=True)
    pdist.destroy()
    print("PASS", flush=True)


if __name__ == "__main__":
    main()
