"""Does a hipGraph replay run independent branches concurrently?

Two single-workgroup spin kernels (torch.cuda._sleep) on two streams, fork-joined, captured
into one graph: replay time ~1x one kernel = branches run concurrently, ~2x = serialised.
The same for eager launches.  Also two half-chip GEMMs (wide enough to be useful work,
small enough that one leaves CUs idle) on two streams vs one.
"""
import json
import time

import torch


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    cyc = 20_000_000
    out = {}

    def one():
        torch.cuda._sleep(cyc)

    def two_serial():
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)

    def two_fork():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
        torch.cuda.current_stream().wait_stream(side)

    out["eager_one_ms"] = timeit(one)
    out["eager_serial_ms"] = timeit(two_serial)
    out["eager_fork_ms"] = timeit(two_fork)
    for name, fn in (("one", one), ("serial", two_serial), ("fork", two_fork)):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(main_s)
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                fn()
        main_s.wait_stream(s)
        out[f"graph_{name}_ms"] = timeit(g.replay)

    # GEMMs: M=4096 rows x 1024 x 1024 bf16 each (few workgroups), two independent chains
    a = torch.randn(2, 8, 2048, 1024, device=dev, dtype=torch.bfloat16)
    w = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)

    def chain(x):
        for _ in range(8):
            x = x @ w
        return x

    def g_serial():
        chain(a[0])
        chain(a[1])

    def g_fork():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            chain(a[1])
        chain(a[0])
        torch.cuda.current_stream().wait_stream(side)

    for name, fn in (("gemm_serial", g_serial), ("gemm_fork", g_fork)):
        out[f"eager_{name}_ms"] = timeit(fn)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(main_s)
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                fn()
        main_s.wait_stream(s)
        out[f"graph_{name}_ms"] = timeit(g.replay)
    print(json.dumps({k: round(v, 3) for k, v in out.items()}))


if __name__ == "__main__":
    main()
