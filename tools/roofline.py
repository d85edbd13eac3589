#!/usr/bin/env python
"""Per-kernel roofline table from tools/gpu_roofline.sh's counter passes, with the MFMA
counters CALIBRATED on a kernel of known MFMA count (tools/probes/mfma_count_probe.hip).

    python tools/roofline.py gpurun_out/roof --steps 3 --probe gpurun_out/r3a/probe_pmc

Columns per kernel name (sorted by time per step): calls / step, mean us, achieved MFMA
TFLOP/s, MFMA busy as a true % of the chip's SIMD-cycles, LDS bank-conflict cycles per LDS
instruction, HBM bytes per call (2 x FETCH_SIZE: gfx950 tallies 128-B reads at 64 B --
MI355X_MICROARCH.md -- + WRITE_SIZE), achieved GB/s and arithmetic intensity.

Calibration (from the probe's own counter pass; its kernels issue exactly
2048 blocks x 4 waves x 4096 x 4 MFMAs, bf16 16x16x32 in k_bf16, e4m3 16x16x128 in k_fp8):
  * inst_scale  = SQ_INSTS_MFMA / expected wave-MFMAs          (how the counter tallies)
  * busy_per_mfma (bf16 / fp8) = SQ_VALU_MFMA_BUSY_CYCLES / expected wave-MFMAs
  * clock = GRBM_GUI_ACTIVE / 8 / duration  (GRBM sums the 8 XCDs; MI355X_MICROARCH.md)
  * MFMA busy % = 100 x (busy cycles / busy_per_mfma_bf16 x 16) / (1024 SIMDs x kernel cycles)
    -- i.e. MFMA-pipe cycles (16 per bf16 16x16x32, 32 per fp8 16x16x128) over the SIMD-cycles
    the kernel had; the probe's own row must read its FLOP-derived utilisation.
FLOPs per MFMA instruction: 16384 (bf16 16x16x32), 32768 (bf16 32x32x16: the *_m32_kernel
tiles, instruction counts calibrated on the probe's k_bf16_32), 65536 (fp8 16x16x128, the conv
kernels' F8 template argument != 0).  MFMA busy % converts the busy counter to pipe-cycles
with the 16x16x32 calibration; the probe's k_bf16_32 row checks that the same conversion
holds for the 32-cycle 32x32x16 instruction (its util_true must read ~1).
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import re
import sys

SIMDS = 1024           # 256 CUs x 4
XCDS = 8
PROBE_WAVE_MFMAS = 2048 * 4 * 4096 * 4


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


def mean(v):
    return sum(v) / len(v) if v else None


def calibrate(probe_dir):
    """Calibration constants from the probe's counter pass (see module docstring)."""
    vals, dur = load(probe_dir)
    cal = {}
    for k, c in vals.items():
        tag = ("bf16_32" if "k_bf16_32" in k else "bf16" if "k_bf16" in k else
               ("fp8" if "k_fp8" in k else None))
        if tag is None:
            continue
        ns = mean(dur.get(k, []))
        inst, busy, grbm = mean(c.get("SQ_INSTS_MFMA")), mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES")), \
            mean(c.get("GRBM_GUI_ACTIVE"))
        flop = PROBE_WAVE_MFMAS * {"bf16": 16384, "bf16_32": 32768, "fp8": 65536}[tag]
        clock = grbm / XCDS / ns if grbm and ns else None              # GHz
        pipe = PROBE_WAVE_MFMAS * (16 if tag == "bf16" else 32)       # MFMA-pipe SIMD-cycles
        cal[tag] = {
            "ns": ns, "tflops": flop / ns / 1e3 if ns else None, "clock_ghz": clock,
            "inst_scale": inst / PROBE_WAVE_MFMAS if inst else None,
            "busy_per_mfma": busy / PROBE_WAVE_MFMAS if busy else None,
            "util_true": pipe / (SIMDS * grbm / XCDS) if grbm else None,
        }
    return cal


def _targs(kernel, name):
    m = re.search(name + r"<([^>]*)>", kernel)
    return [x.strip() for x in m.group(1).split(",")] if m else None


def is_fp8(kernel):
    """fp8 (f8f6f4) MFMA kernels: the glds conv tile's FP8 argument, the fp8 weight-gradient
    and s2t instances, and the round-6 32x32x64 m32 instances (5th template argument F8)."""
    g = _targs(kernel, "conv_fwd_glds_kernel")
    if g:
        return len(g) > 8 and g[8] not in ("0",)
    if "conv_wgrad_f8_kernel" in kernel:
        return True
    for name, pos in (("conv_fwd_m32_kernel", 4), ("conv_s2t_kernel", 3)):
        g = _targs(kernel, name)
        if g:
            return len(g) > pos and g[pos] not in ("0",)
    return False


def is_m32(kernel):
    """The 32x32 MFMA kernels: conv_fwd_m32 (32x32x16 bf16 / 32x32x64 f8f6f4), conv_wgrad_m32."""
    return "_m32_kernel" in kernel


def flop_per_mfma(kernel):
    """FLOP of one MFMA instruction of the kernel: 16x16x32 bf16 16384, 32x32x16 bf16 32768,
    16x16x128 f8f6f4 65536, 32x32x64 f8f6f4 131072."""
    return (131072 if is_m32(kernel) else 65536) if is_fp8(kernel) else \
        (32768 if is_m32(kernel) else 16384)


def short(k):
    return k.replace("void p2p::", "").replace("p2p::", "").split("(")[0][:72]


def main(root, steps, probe):
    cal = calibrate(probe) if probe else {}
    if cal:
        print("calibration (tools/probes/mfma_count_probe.hip, known MFMA counts):")
        print("```")
        print(json.dumps(cal, indent=1))
        print("```")
    inst_scale = cal.get("bf16", {}).get("inst_scale") or 1.0
    busy_bf16 = cal.get("bf16", {}).get("busy_per_mfma") or 16.0
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
        mf = mean(c.get("SQ_INSTS_MFMA", []))
        busy = mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        grbm = mean(c.get("GRBM_GUI_ACTIVE", []))
        lds, conf = mean(c.get("SQ_INSTS_LDS", [])), mean(c.get("SQ_LDS_BANK_CONFLICT", []))
        fetch = mean(fe.get(k, {}).get("FETCH_SIZE", []))
        write = mean(wr.get(k, {}).get("WRITE_SIZE", []))
        fpi = flop_per_mfma(k)
        scale_i = (cal.get("bf16_32", {}).get("inst_scale") or inst_scale) if is_m32(k) else inst_scale
        flop = (mf / scale_i) * fpi if mf else 0.0
        # MFMA-pipe SIMD-cycles: the busy counter in units of one bf16 16x16x32 (16 cycles)
        pipe = busy / busy_bf16 * 16 if busy else None
        util = 100.0 * pipe / (SIMDS * grbm / XCDS) if pipe and grbm else None
        clock = grbm / XCDS / mean_ns if grbm else None
        byts = ((2 * fetch if fetch else 0.0) + (write or 0.0)) * 1024
        rows.append((sum(ds) / steps, k, n / steps, mean_ns, flop, util,
                     conf / lds if lds and conf is not None else None, byts, clock))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows) or 1.0
    print()
    print("| kernel | %step | calls/step | us/call | MFMA TF/s | MFMA busy % | LDS confl/instr | "
          "HBM MB/call | GB/s | FLOP/B | clock GHz |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for t, k, calls, mean_ns, flop, util, cf, byts, clock in rows[:45]:
        tf = flop / mean_ns / 1e3 if mean_ns else 0.0
        gbs = byts / mean_ns if mean_ns else 0.0
        ai = flop / byts if byts else 0.0
        print(f"| {short(k)} | {100 * t / tot:.1f} | {calls:.1f} | {mean_ns / 1e3:.1f} | {tf:.0f} | "
              f"{'-' if util is None else f'{util:.1f}'} | {'-' if cf is None else f'{cf:.2f}'} | "
              f"{byts / 1e6:.1f} | {gbs:.0f} | {ai:.1f} | {'-' if clock is None else f'{clock:.2f}'} |")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = 3
    probe = None
    if "--steps" in sys.argv:
        steps = float(sys.argv[sys.argv.index("--steps") + 1])
        args = [a for a in args if a != sys.argv[sys.argv.index("--steps") + 1]]
    if "--probe" in sys.argv:
        probe = sys.argv[sys.argv.index("--probe") + 1]
        args = [a for a in args if a != probe]
    main(args[0] if args else "gpurun_out/roof", steps, probe)
