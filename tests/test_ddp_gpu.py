"""Data-parallel path on the GPU kernels: 2 ranks sharing the box's one GPU through the gloo
rehearsal backend (tools/ddp_rehearsal.py).  The RCCL production path differs only in the
process-group backend; its 8-GPU run is the driver's scaling bench."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_rehearsal_on_one_gpu():
    env = dict(os.environ, P2P_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tools", "ddp_rehearsal.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(lines[-1])
    assert res["ok"], res
