"""Runtime utilities on CPU: NaN guard skips poisoned updates, watchdog aborts a hung
process, JSONL metrics, roctx ranges / phase timer are safe without a GPU."""
import json
import subprocess
import sys

import torch

from p2p_pytorch_amd.engine.pix2pix import Pix2PixStep
from p2p_pytorch_amd.models import define_D, define_G
from p2p_pytorch_amd.utils import JsonlLogger, PhaseTimer, nonfinite, trace_range


def test_nonfinite_flag():
    assert float(nonfinite(torch.tensor(1.0), torch.tensor(2.0))) == 0.0
    assert float(nonfinite(torch.tensor(1.0), torch.tensor(float("inf")))) == 1.0
    assert float(nonfinite(torch.tensor(float("nan")))) == 1.0


def test_nan_guard_skips_update():
    torch.manual_seed(0)
    G = define_G(netG="unet_64", gpu_id="cpu", verbose=False)
    D = define_D(6, 64, norm="instance", netD="basic", gpu_id="cpu", verbose=False)
    st = Pix2PixStep(G, D)
    a = torch.rand(2, 3, 64, 64) * 2 - 1
    b = torch.rand(2, 3, 64, 64) * 2 - 1
    st.step(a, b)
    assert float(st.skipped) == 0.0
    g0 = [p.detach().clone() for p in G.parameters()]
    d0 = [p.detach().clone() for p in D.parameters()]
    b[0, 0, 0, 0] = float("nan")   # poisons loss_D (real branch) and loss_G (L1)
    st.step(a, b)
    assert float(st.skipped) == 2.0
    assert all(torch.equal(x, y) for x, y in zip(g0, G.parameters()))
    assert all(torch.equal(x, y) for x, y in zip(d0, D.parameters()))


def test_watchdog_aborts_hung_process():
    code = ("import time; from p2p_pytorch_amd.utils import StepWatchdog; "
            "StepWatchdog(timeout_s=1.0).start(); time.sleep(30)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=60)
    assert r.returncode == 124
    assert b"watchdog" in r.stderr


def test_jsonl_logger(tmp_path):
    p = tmp_path / "m.jsonl"
    lg = JsonlLogger(str(p), rank=0)
    lg.log(step=1, img_s=10.0, loss=torch.tensor(0.5).item())
    lg.close()
    rec = json.loads(p.read_text().strip())
    assert rec["step"] == 1 and rec["img_s"] == 10.0
    JsonlLogger(str(tmp_path / "x.jsonl"), rank=1).log(a=1)   # non-zero ranks write nothing
    assert not (tmp_path / "x.jsonl").exists()


def test_trace_range_and_timer_cpu():
    t = PhaseTimer()
    with trace_range("x"), t.phase("y"):
        pass
    assert isinstance(t.report(), dict)
