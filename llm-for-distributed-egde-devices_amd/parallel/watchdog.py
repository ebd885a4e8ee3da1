"""Failure detection for the pipeline (the reference has none).

``Watchdog`` is a heartbeat monitor: the stage loop calls ``beat()`` every tick; if no beat
arrives within ``timeout_s`` the watchdog logs which tick the rank was stuck after and aborts
the WHOLE process (a stuck peer or a hung collective would otherwise block every rank forever —
RCCL P2P has no per-op timeout).  torchrun then tears down the job; with
``TORCH_NCCL_ASYNC_ERROR_HANDLING=1`` the other ranks' pending RCCL ops error out too.
``init_pg_timeout`` sets the process-group timeout used by collectives.
"""
from __future__ import annotations

import os
import threading
import time
from datetime import timedelta
from typing import Callable, Optional

from ..utils.log import get_logger

log = get_logger("watchdog")


class Watchdog:
    def __init__(self, timeout_s: float = 300.0, on_timeout: Optional[Callable[[str], None]] = None,
                 poll_s: float = 0.5, name: str = "pipeline"):
        self.timeout_s, self.poll_s, self.name = timeout_s, poll_s, name
        self.on_timeout = on_timeout or self._abort
        self._last = time.monotonic()
        self._what = "start"
        self._stop = threading.Event()
        self.fired = False
        self._t = threading.Thread(target=self._run, daemon=True)

    def start(self) -> "Watchdog":
        self._last = time.monotonic()
        self._t.start()
        return self

    def beat(self, what: str = ""):
        self._last = time.monotonic()
        self._what = what

    def stop(self):
        self._stop.set()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def _run(self):
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self.fired = True
                msg = f"{self.name}: no progress for {idle:.1f}s (last: {self._what})"
                log.error(msg)
                self.on_timeout(msg)
                return

    @staticmethod
    def _abort(msg: str):  # pragma: no cover - kills the process
        os._exit(124)


def init_pg_timeout(seconds: float = 600.0) -> timedelta:
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    return timedelta(seconds=seconds)
