#!/usr/bin/env python
"""Aggregate rocprofv3 --pmc CSVs (one row per dispatch x counter) into per-kernel means.

    python tools/pmc_summary.py gpurun_out/pmc
"""
import collections
import csv
import glob
import os
import sys


def main(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
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
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
