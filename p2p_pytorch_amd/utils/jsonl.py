"""JSONL metrics stream (rank 0 only): one JSON object per line, flushed per record."""
from __future__ import annotations

import json
import os
import time


class JsonlLogger:
    def __init__(self, path, rank: int = 0):
        self.path = path if (path and rank == 0) else None
        self._f = None
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            self._f = open(self.path, "a")

    def log(self, **rec):
        if self._f is None:
            return
        rec.setdefault("time", time.time())
        self._f.write(json.dumps(rec, default=float) + "\n")
        self._f.flush()

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None
