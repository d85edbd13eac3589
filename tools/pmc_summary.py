#!/usr/bin/env python
"""Aggregate rocprofv3 --pmc CSVs (one row per dispatch x counter) into per-kernel means.

    python tools/pmc_summary.py gpurun_out/pmc [--table]

--table: one line per kernel -- dispatches, instruction mix per MFMA (VALU / SALU / LDS) and the
issue-active fraction of wave cycles, sorted by total wave cycles.
"""
import collections
import csv
import glob
import os
import sys


def table(vals):
    rows = []
    for k, cs in vals.items():
        if "p2p::" not in k:
            continue
        tot = {c: sum(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        rows.append((tot.get("SQ_WAVE_CYCLES", 0.0), k, n, tot))
    rows.sort(reverse=True)
    print(f"{'wave_cyc%':>9s} {'calls':>6s} {'MFMA':>10s} {'VALU/M':>7s} {'SALU/M':>7s} {'LDS/M':>6s} "
          f"{'active':>6s}  kernel")
    allw = sum(r[0] for r in rows) or 1.0
    for wc, k, n, t in rows:
        mf = t.get("SQ_INSTS_MFMA", 0.0)
        per = (lambda c: f"{t.get(c, 0.0) / mf:7.2f}") if mf else (lambda c: "      -")
        act = t.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else 0.0
        name = k.replace("void p2p::", "").split("(")[0][:70]
        print(f"{100 * wc / allw:9.1f} {n:6d} {mf:10.0f} {per('SQ_INSTS_VALU')} {per('SQ_INSTS_SALU')} "
              f"{per('SQ_INSTS_LDS')[1:]} {act:6.3f}  {name}")


def main(d, as_table=False):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if as_table:
        table(vals)
        return
    for k, cs in sorted(vals.items()):
        if "p2p::" not in k:
            continue
        print(k[:150])
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.0f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':40s} {m[c] / wc:6.3f}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0] if args else "gpurun_out/pmc", "--table" in sys.argv)
