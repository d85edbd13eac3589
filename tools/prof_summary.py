#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace --output-format csv`` trace of ``bench.py``.

Only the steady-state timed steps are counted: the trace is cut at optimizer kernels
(eager: ``multi_tensor_apply``; native: ``adam_kernel``), two optimizer calls per pix2pix
step, and the last ``--steps`` steps are aggregated per kernel name.

    python tools/prof_summary.py TRACE.csv --steps 5 [--top 40] [--streams] > profiles/x.txt

``--streams``: per HIP stream (queue) busy time, the union of all kernels' intervals (GPU
active), the idle remainder of the wall and the overlapped time, plus the top kernels of
each stream -- which of the step's two streams (main / weight-gradient side) bounds the wall.
"""
from __future__ import annotations

import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--opt_per_step", type=int, default=2)
    ap.add_argument("--width", type=int, default=120)
    ap.add_argument("--streams", action="store_true")
    ap.add_argument("--calls", default=None,
                    help="substring: list every matching dispatch of the last step (offset, us, grid)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows)
           if "multi_tensor" in r["Kernel_Name"] or "adam" in r["Kernel_Name"].lower()]
    groups = []
    for i in idx:
        if groups and i - groups[-1][-1] <= 3:
            groups[-1].append(i)
        else:
            groups.append([i])
    need = a.steps * a.opt_per_step
    if len(groups) < need + 1:
        raise SystemExit(f"only {len(groups)} optimizer calls found, need {need + 1}")
    start = groups[-need - 1][-1] + 1
    end = groups[-1][-1] + 1
    sel = rows[start:end]
    t0 = int(sel[0]["Start_Timestamp"])
    t1 = int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"][: a.width]][0] += d
        agg[r["Kernel_Name"][: a.width]][1] += 1
    busy = sum(v[0] for v in agg.values())
    S = a.steps
    print(f"trace: {a.trace}")
    print(f"steady-state steps: {S}; wall (first->last kernel) {((t1 - t0) / 1e6 / S):.3f} ms/step; "
          f"kernel busy {busy / 1e6 / S:.3f} ms/step; dispatches/step {len(sel) / S:.0f}")
    print(f"{'ms/step':>8} {'%':>5} {'n/step':>7}  kernel")
    for k, v in sorted(agg.items(), key=lambda x: -x[1][0])[: a.top]:
        print(f"{v[0] / 1e6 / S:8.3f} {100 * v[0] / busy:5.1f} {v[1] / S:7.1f}  {k}")
    if a.streams:
        streams(sel, S, t0, t1, a.width)
    if a.calls is not None:
        last = rows[groups[-3][-1] + 1:end]
        s0 = int(last[0]["Start_Timestamp"])
        print(f"\ndispatches of the last step matching {a.calls!r}: start offset ms, us, blocks, workgroup")
        for r in last:
            if a.calls in r["Kernel_Name"]:
                b, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                g = [int(r.get(f"Grid_Size_{c}", 1) or 1) for c in "XYZ"]
                w = [int(r.get(f"Workgroup_Size_{c}", 1) or 1) for c in "XYZ"]
                blocks = (g[0] // w[0]) * (g[1] // w[1]) * (g[2] // w[2])
                print(f"  {(b - s0) / 1e6:9.3f} {(e - b) / 1e3:9.1f}  blocks {blocks:>7} "
                      f"({g[0] // w[0]}x{g[1] // w[1]}x{g[2] // w[2]}) wg {w[0]:>4}  {r['Kernel_Name'][:a.width]}")


def streams(sel, S, t0, t1, width):
    key = "Stream_Id" if "Stream_Id" in sel[0] else "Queue_Id"
    per = collections.defaultdict(list)
    for r in sel:
        per[r.get(key, "?")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ivs = sorted((b, e) for v in per.values() for b, e, _ in v)
    union, cb, ce = 0, None, None
    for b, e in ivs:
        if ce is None or b > ce:
            if ce is not None:
                union += ce - cb
            cb, ce = b, e
        else:
            ce = max(ce, e)
    if ce is not None:
        union += ce - cb
    tot = sum(e - b for b, e in ivs)
    wall = t1 - t0
    print(f"\nby {key}: wall {wall / 1e6 / S:.3f} ms/step, GPU active (union) {union / 1e6 / S:.3f}, "
          f"idle {(wall - union) / 1e6 / S:.3f}, overlapped {(tot - union) / 1e6 / S:.3f} ms/step")
    for sid, v in sorted(per.items(), key=lambda x: -sum(e - b for b, e, _ in x[1])):
        busy = sum(e - b for b, e, _ in v)
        print(f"  {key} {sid}: {busy / 1e6 / S:8.3f} ms/step busy, {len(v) / S:.0f} kernels/step")
        agg = collections.defaultdict(int)
        for b, e, n in v:
            agg[n[:width]] += e - b
        for n, d in sorted(agg.items(), key=lambda x: -x[1])[:8]:
            print(f"      {d / 1e6 / S:8.3f}  {n}")


if __name__ == "__main__":
    main()
