#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace --output-format csv`` trace of ``bench.py``.

Only the steady-state timed steps are counted: the trace is cut at optimizer kernels
(eager: ``multi_tensor_apply``; native: ``adam_kernel``), two optimizer calls per pix2pix
step, and the last ``--steps`` steps are aggregated per kernel name.

    python tools/prof_summary.py TRACE.csv --steps 5 [--top 40] > profiles/x.txt
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


if __name__ == "__main__":
    main()
