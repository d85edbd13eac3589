"""The measurement tools the profiles/ tables come from, on synthetic rocprofv3 CSVs (CPU).

``tools/roofline.py`` turns per-dispatch PMC counters into TF/s and MFMA-busy columns: the
FLOP each MFMA instruction stands for depends on the kernel's instruction shape (16x16x32 /
32x32x16 bf16, 16x16x128 / 32x32x64 f8f6f4), read off the template arguments of the demangled
kernel name -- a wrong attribution silently mis-states a kernel's TF/s by 2-8x.
``tools/prof_summary.py`` cuts a kernel trace into steady-state steps at the optimizer kernels.
"""
import csv
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import roofline  # noqa: E402

M32_BF16 = "void p2p::conv_fwd_m32_kernel<256, 0, false, false, 0, 256>(p2p::ConvFwdArgs)"
M32_512 = "void p2p::conv_fwd_m32_kernel<128, 1, false, true, 0, 512>(p2p::ConvFwdArgs)"
M32_F8 = "void p2p::conv_fwd_m32_kernel<128, 1, false, true, 2, 256>(p2p::ConvFwdArgs)"
GLDS_BF16 = "void p2p::conv_fwd_glds_kernel<128, 128, 2, 2, 1, 2, false, false, 0, false, false>(p2p::ConvFwdArgs)"
GLDS_F8 = "void p2p::conv_fwd_glds_kernel<256, 256, 2, 4, 0, 2, true, false, 1, false, false>(p2p::ConvFwdArgs)"
WGRAD_M32 = "void p2p::conv_wgrad_m32_kernel<0, 128>(p2p::ConvWgradArgs, int)"
WGRAD_F8 = "void p2p::conv_wgrad_f8_kernel<256, 128, 4, 2, 3, 0, 1, 0>(p2p::ConvWgradArgs, int)"
S2T_BF16 = "void p2p::conv_s2t_kernel<64, false, true, 0>(p2p::ConvFwdArgs, int, int)"
S2T_F8 = "void p2p::conv_s2t_kernel<64, true, false, 1>(p2p::ConvFwdArgs, int, int)"
HALO = "void p2p::halo_pk8_kernel<4, 2, false, false>(p2p::HaloPk8Args)"


@pytest.mark.parametrize("name,flop", [
    (M32_BF16, 32768), (M32_512, 32768), (WGRAD_M32, 32768),   # v_mfma_f32_32x32x16_bf16
    (M32_F8, 131072),                                            # v_mfma_scale_f32_32x32x64_f8f6f4
    (GLDS_F8, 65536), (WGRAD_F8, 65536), (S2T_F8, 65536),        # v_mfma_scale_f32_16x16x128_f8f6f4
    (GLDS_BF16, 16384), (S2T_BF16, 16384), (HALO, 16384),        # v_mfma_f32_16x16x32_bf16
])
def test_flop_per_mfma_from_kernel_name(name, flop):
    assert roofline.flop_per_mfma(name) == flop


def _write_csv(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_roofline_table_from_counters(tmp_path, capsys):
    """One 32x32x64 fp8 kernel: 1000 MFMA instructions over 1 us -> 131 TF/s; MFMA busy from
    the busy counter against GRBM cycles; HBM bytes = 2 x FETCH_SIZE (KB) + WRITE_SIZE (KB)."""
    k = M32_F8
    counters = [("SQ_INSTS_MFMA", 1000.0), ("SQ_VALU_MFMA_BUSY_CYCLES", 16000.0), ("GRBM_GUI_ACTIVE", 8000.0),
                ("SQ_INSTS_LDS", 100.0), ("SQ_LDS_BANK_CONFLICT", 25.0)]
    for sub, rows in (("sq", counters), ("fetch", [("FETCH_SIZE", 10.0)]), ("write", [("WRITE_SIZE", 5.0)])):
        _write_csv(str(tmp_path / sub / "run_counter_collection.csv"),
                   ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"],
                   [(1, k, c, v) for c, v in rows])
        _write_csv(str(tmp_path / sub / "run_kernel_trace.csv"),
                   ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], [(k, 0, 1000)])
    roofline.main(str(tmp_path), 1, None)
    out = capsys.readouterr().out
    row = next(line for line in out.splitlines() if "conv_fwd_m32_kernel<128, 1, false, true, 2, 256>" in line)
    cells = [c.strip() for c in row.strip("|").split("|")]
    # kernel | %step | calls/step | us/call | TF/s | busy % | confl | MB/call | GB/s | FLOP/B | GHz
    assert cells[3] == "1.0"                       # us per call (3 trace files x 1 dispatch / 3 dirs)
    assert cells[4] == "131"                       # 1000 x 131072 FLOP / 1000 ns
    assert cells[6] == "0.25"                      # LDS conflicts per LDS instruction
    assert cells[7] == "0.0"                       # (2 x 10 + 5) KB = 0.0256 MB


def _trace(path, names_durations):
    rows, t = [], 0
    for n, d in names_durations:
        rows.append((n, t, t + d, 0))
        t += d + 10
    _write_csv(path, ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id"], rows)


def test_prof_summary_cuts_steady_steps(tmp_path):
    """Warm-up dispatches before the first counted optimizer pair are excluded; each step is
    [conv x2, norm x2, adam (D), norm x4, adam (G)] (optimizer dispatches closer than 4 apart count as
    one call: multi-tensor bursts); 3 steps counted -> 2 conv calls per step at 1 us each."""
    step = [(M32_BF16, 1000), (M32_BF16, 1000)] + [("norm_apply", 500)] * 2 + [("p2p::adam_kernel(...)", 100)] + \
        [("norm_apply", 500)] * 4 + [("p2p::adam_kernel(...)", 100)]
    trace = str(tmp_path / "t.csv")
    _trace(trace, [("warmup_only_kernel", 5000)] + step * 4)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_summary.py"), trace, "--steps", "3",
                          "--width", "200"], capture_output=True, text=True, check=True).stdout
    assert "steady-state steps: 3" in out
    line = next(ln for ln in out.splitlines() if "conv_fwd_m32_kernel" in ln)
    ms, pct, n = line.split()[:3]
    assert float(ms) == pytest.approx(0.002) and float(n) == pytest.approx(2.0)
    assert "warmup_only_kernel" not in out
