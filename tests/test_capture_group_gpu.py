"""A hipGraph capture right behind a pending eager RCCL collective.

``tools/diag_capture_event.py --mode race --capture-mode global`` is the one-rank
reproduction of the c10d watchdog abort: the watchdog queries an eager all-reduce's end event
while a capture runs.  HIP refuses that query (a) from any thread under the default "global"
capture mode (``hipErrorStreamCaptureUnsupported`` -- measured in round 6 even with the
captured collective on another group) and (b) for an event last recorded on a stream that
joined the capture.  Since round 6 ``CapturedStep`` captures in "thread_local" mode and
records its collectives on ``parallel.dist.capture_group()`` -- a fresh group with no eager
history -- instead of sleeping a few watchdog polls.  Here the eager all-reduce is still pending (a GEMM
chain ahead of it) when the capture starts, with no sync and no sleep in between, and the
capture holds a ``ReduceOp.AVG`` all-reduce for 0.5 s while the watchdog polls: the process
must survive three rounds.  Run in a child process, so an abort fails this test instead of
killing the runner.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_capture_behind_pending_eager_collective_isolated():
    env = dict(os.environ)
    env.pop("MASTER_PORT", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diag_capture_event.py"),
                        "--mode", "isolated", "--capture-mode", "thread_local", "--rounds", "3"],
                       capture_output=True, text=True, timeout=110, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "PASS" in r.stdout and r.stdout.count("ok (isolated)") == 3, out[-3000:]
