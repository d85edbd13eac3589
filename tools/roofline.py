#!/usr/bin/env python
"""Per-kernel roofline table from tools/gpu_roofline.sh's counter passes.

    python tools/roofline.py gpurun_out/roof --steps 3

Per kernel name (sorted by total time per step): calls / step, mean us, achieved MFMA
TFLOP/s (SQ_INSTS_MFMA x 16384 FLOP -- every conv MFMA is v_mfma_f32_16x16x32_bf16),
MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES, as reported), LDS bank-
conflict cycles per LDS instruction, HBM bytes (2 x FETCH_SIZE: gfx950 tallies 128-B reads
at 64 B -- MI355X_MICROARCH.md; + WRITE_SIZE), achieved GB/s and arithmetic intensity.
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def load(d):
    """{kernel: {counter: [per-dispatch values]}} and {kernel: [durations ns]}."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[key[0]] = r.get("Kernel_Name", "?")
        for (disp, c), v in per.items():
            vals[names[disp]][c].append(v)
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, dur


def short(k):
    return k.replace("void p2p::", "").replace("p2p::", "").split("(")[0][:64]


def main(root, steps):
    sq, dur = load(os.path.join(root, "sq"))
    fe, _ = load(os.path.join(root, "fetch"))
    wr, _ = load(os.path.join(root, "write"))
    rows = []
    for k, ds in dur.items():
        if not k.startswith(("void p2p::", "p2p::", "_ZN3p2p")):
            continue
        n = len(ds)
        mean_ns = sum(ds) / n
        c = sq.get(k, {})

        def m(cs, name):
            v = cs.get(name)
            return sum(v) / len(v) if v else None

        mf = m(c, "SQ_INSTS_MFMA")
        busy, mbusy = m(c, "SQ_BUSY_CYCLES"), m(c, "SQ_VALU_MFMA_BUSY_CYCLES")
        lds, conf = m(c, "SQ_INSTS_LDS"), m(c, "SQ_LDS_BANK_CONFLICT")
        fetch = m(fe.get(k, {}), "FETCH_SIZE")
        write = m(wr.get(k, {}), "WRITE_SIZE")
        flop = mf * 16384 if mf else 0.0
        byts = ((2 * fetch if fetch else 0.0) + (write or 0.0)) * 1024
        rows.append((sum(ds) / steps, k, n / steps, mean_ns, flop, mbusy / busy if busy and mbusy else None,
                     conf / lds if lds and conf is not None else None, byts))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows) or 1.0
    print("| kernel | %step | calls/step | us/call | MFMA TF/s | MFMA busy | LDS confl/instr | HBM MB/call | GB/s | FLOP/B |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for t, k, calls, mean_ns, flop, mb, cf, byts in rows[:40]:
        tf = flop / mean_ns / 1e3 if mean_ns else 0.0
        gbs = byts / mean_ns if mean_ns else 0.0
        ai = flop / byts if byts else 0.0
        print(f"| {short(k)} | {100 * t / tot:.1f} | {calls:.1f} | {mean_ns / 1e3:.1f} | {tf:.0f} | "
              f"{'-' if mb is None else f'{mb:.2f}'} | {'-' if cf is None else f'{cf:.2f}'} | "
              f"{byts / 1e6:.1f} | {gbs:.0f} | {ai:.1f} |")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = 3
    if "--steps" in sys.argv:
        steps = float(sys.argv[sys.argv.index("--steps") + 1])
    main(args[0] if args else "gpurun_out/roof", steps)
