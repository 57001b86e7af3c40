"""Stall watchdog (SURVEY.md §5 'failure detection').

The reference gets Horovod's stall inspector for free behind ``hvd.init()`` (``/root/reference/scripts/train.py:24``):
a rank that stops reaching the collectives is reported instead of hanging the job silently. Here a monitor thread
watches the training steps themselves:

* the host marks a step's start and end (``step_begin`` / ``step_end``);
* at ``step_end`` a device event is recorded on the compute stream, so a step only counts as complete once the GPU
  has finished it (a hung kernel or RCCL collective never completes, even though the host launched everything);
* if no step completes for ``timeout_s`` while a step is in flight (on the host or on the device), the thread logs
  rank, step, phase and the last launched gradient bucket, flushes every log handler and ends the process with
  ``os._exit(exit_code)`` — no re-exec, no cleanup that could block on the hung device. The launcher
  (``launcher/spawn.py``) then sees a non-zero exit code and tears the whole group down.

Time spent between steps (data loading, callbacks, evaluation) is not counted.
"""
from __future__ import annotations

import logging
import os
import sys
import threading
import time
from collections import deque
from typing import Callable, Optional

import torch

logger = logging.getLogger(__name__)

EXIT_CODE = 124  # timeout(1)'s code: "the job was stopped because it stopped making progress"


class StepWatchdog:
    def __init__(self, timeout_s: float, rank: int = 0, describe: Optional[Callable[[], str]] = None,
                 exit_code: int = EXIT_CODE, poll_s: Optional[float] = None, on_stall: Optional[Callable] = None):
        """``describe``: returns a one-line context for the report (phase, last bucket, ...).
        ``on_stall``: replaces the ``os._exit`` (tests of the detection logic itself)."""
        if timeout_s <= 0:
            raise ValueError("timeout_s must be > 0")
        self.timeout_s = float(timeout_s)
        self.rank = int(rank)
        self.describe = describe
        self.exit_code = int(exit_code)
        self.poll_s = float(poll_s) if poll_s else min(1.0, self.timeout_s / 4.0)
        self.on_stall = on_stall
        self._lock = threading.Lock()
        self._pending = deque()  # (step, event or None, t_end_host)
        self._in_step: Optional[int] = None
        self._last_progress = time.monotonic()
        self._last_done = -1
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.fired = False

    # ---------------------------------------------------------------- host-side marks
    def start(self) -> "StepWatchdog":
        if self._thread is None:
            self._last_progress = time.monotonic()
            self._thread = threading.Thread(target=self._run, name=f"hsd-watchdog-r{self.rank}", daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5 * self.poll_s)
            self._thread = None

    def step_begin(self, step: int) -> None:
        with self._lock:
            if self._in_step is None and not self._pending:
                self._last_progress = time.monotonic()  # idle -> busy: the clock starts now
            self._in_step = int(step)

    def step_end(self, step: int, device: Optional[torch.device] = None) -> None:
        ev = None
        if device is not None and device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(device))
        with self._lock:
            self._in_step = None
            self._pending.append((int(step), ev, time.monotonic()))

    # ---------------------------------------------------------------- monitor
    def _poll(self) -> Optional[str]:
        """Retire completed steps; return a stall report if the job made no progress for timeout_s."""
        now = time.monotonic()
        with self._lock:
            while self._pending:
                step, ev, _ = self._pending[0]
                if ev is not None and not ev.query():
                    break
                self._pending.popleft()
                self._last_done = step
                self._last_progress = now
            busy = self._in_step is not None or bool(self._pending)
            if not busy:
                self._last_progress = now
                return None
            idle = now - self._last_progress
            if idle <= self.timeout_s:
                return None
            where = (f"host in step {self._in_step}" if self._in_step is not None
                     else f"device still running step {self._pending[0][0]}")
            ctx = ""
            if self.describe is not None:
                try:
                    ctx = self.describe()
                except Exception as e:  # the report must not die on a broken context
                    ctx = f"(context unavailable: {e})"
            return (f"step watchdog: rank {self.rank} made no progress for {idle:.1f}s (> {self.timeout_s:g}s); "
                    f"{where}; last completed step {self._last_done}; {ctx}")

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            report = self._poll()
            if report is None:
                continue
            self.fired = True
            logger.error(report)
            print(report, file=sys.stderr, flush=True)
            for h in logging.getLogger().handlers:
                try:
                    h.flush()
                except Exception:
                    pass
            if self.on_stall is not None:
                self.on_stall(report)
                return
            os._exit(self.exit_code)
