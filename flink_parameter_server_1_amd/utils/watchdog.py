"""Fail-fast heartbeat watchdog.

The reference has no failure detection beyond Flink job failure and ends by an
idle timeout (``M/FlinkParameterServer.scala:49-52``; ``README.md:62-69``).  A
tensor-engine rank blocked in a collective whose peer died or hung would only
fail at the process group's timeout (minutes).  ``Watchdog`` is a daemon thread
fed by ``beat()`` once per step: when no beat arrives for ``timeout_s`` it
writes a diagnostic line and ends THIS process with ``exit_code`` (``os._exit``:
no re-exec, no unwinding into a blocked collective).  The peers then fail their
next collective (gloo: connection closed; RCCL: their own watchdog), so a hung
or dead rank stops the whole job within about one watchdog budget instead of
the process-group timeout.  Restart from the last ``utils.io.Checkpointer``
snapshot.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, Optional

#: exit status of a process ended by the watchdog
WATCHDOG_EXIT = 17


class Watchdog:
    def __init__(self, timeout_s: float, name: str = "fps", exit_code: int = WATCHDOG_EXIT,
                 on_timeout: Optional[Callable[[str], None]] = None, poll_s: Optional[float] = None):
        if timeout_s <= 0:
            raise ValueError("timeout_s must be > 0")
        self.timeout_s = float(timeout_s)
        self.name, self.exit_code = name, exit_code
        self.on_timeout = on_timeout
        self.poll_s = poll_s if poll_s is not None else min(1.0, self.timeout_s / 4)
        self._last = time.monotonic()
        self._step = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.fired = False

    def beat(self, step=None) -> None:
        self._last = time.monotonic()
        self._step = step

    def start(self) -> "Watchdog":
        self._last = time.monotonic()
        self._thread = threading.Thread(target=self._run, name=f"{self.name}-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2 * self.poll_s + 1)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def _run(self):
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self.fired = True
                msg = (f"[{self.name}] watchdog: no progress for {idle:.1f} s (budget {self.timeout_s:.1f} s, "
                       f"last step {self._step}, pid {os.getpid()}, rank {os.environ.get('RANK', '0')}); aborting")
                try:
                    print(msg, file=sys.stderr, flush=True)
                    if self.on_timeout is not None:
                        self.on_timeout(msg)
                        return
                finally:
                    if self.on_timeout is None:
                        os._exit(self.exit_code)
