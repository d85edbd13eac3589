"""Step watchdog: a daemon thread that aborts the job when no step completes in time.

A collective that never returns (a dead peer, a hung link) otherwise blocks every rank
forever; RCCL's own timeout (``init_process_group(timeout=...)`` plus async error
handling) covers the collectives, this covers everything else.  On expiry it dumps every
thread's stack (``faulthandler``), tries to abort the process group, and exits with
status 124 so a launcher restarts from the latest checkpoint.

The abort never blocks the exit: with a collective hung, ``destroy_process_group`` itself can
wait on that collective forever, so the abort (``_abort_process_group`` -- ncclCommAbort on
RCCL -- where torch has it) runs on a helper thread that gets ``abort_grace_s`` seconds, and
``os._exit(124)`` follows regardless.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time


class StepWatchdog:
    def __init__(self, timeout_s: float = 1800.0, on_expire=None, abort_grace_s: float = 5.0):
        self.timeout_s = float(timeout_s)
        self.abort_grace_s = float(abort_grace_s)
        self.on_expire = on_expire
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._t = None

    def start(self):
        if self.timeout_s <= 0 or self._t is not None:
            return self
        self._t = threading.Thread(target=self._run, name="p2p-watchdog", daemon=True)
        self._t.start()
        return self

    def beat(self):
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(min(10.0, self.timeout_s / 4)):
            if time.monotonic() - self._last > self.timeout_s:
                sys.stderr.write(f"[watchdog] no step finished in {self.timeout_s:.0f}s; aborting\n")
                faulthandler.dump_traceback(all_threads=True)
                if self.on_expire is not None:
                    try:
                        self.on_expire()
                    except Exception:  # noqa: BLE001 - best effort before exiting
                        pass
                t = threading.Thread(target=_abort_group, name="p2p-watchdog-abort", daemon=True)
                t.start()
                t.join(self.abort_grace_s)
                sys.stderr.flush()
                os._exit(124)


def _abort_group():
    try:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return
        abort = getattr(dist.distributed_c10d, "_abort_process_group", None)
        if abort is not None:
            abort()
        else:
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - best effort; the exit follows regardless
        pass
