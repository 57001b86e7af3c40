"""roctx ranges and a torch.profiler window.

On ROCm builds ``torch.cuda.nvtx`` emits roctx markers, which rocprofv3 (``--marker-trace``) and the
torch profiler both pick up; ranges are off unless enabled (``--profile`` or ``HSD_RANGES=1``) so the hot
loop pays nothing by default.
"""
from __future__ import annotations

import contextlib
import logging
import os
from typing import Optional

import torch

logger = logging.getLogger(__name__)

_RANGES = os.environ.get("HSD_RANGES", "0") == "1"


def set_ranges(on: bool) -> None:
    global _RANGES
    _RANGES = bool(on)


def ranges_enabled() -> bool:
    return _RANGES


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    if not _RANGES or not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class ProfilerCallback:
    """Profile steps ``[start, start + steps)`` of the first epoch with torch.profiler (CPU + HIP activity)
    and write ``trace_rank{r}.json`` (Chrome trace) plus a kernel summary table to ``out_dir``."""

    def __init__(self, out_dir: str, start: int = 3, steps: int = 3, rank: int = 0):
        self.out_dir = out_dir
        self.start, self.steps, self.rank = int(start), int(steps), int(rank)
        self._prof: Optional[torch.profiler.profile] = None
        self._done = False

    def on_train_begin(self, trainer):
        set_ranges(True)

    def on_batch_end(self, trainer, step):
        if self._done:
            return
        if step + 1 == self.start and self._prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()
        elif self._prof is not None and step + 1 == self.start + self.steps:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._prof.__exit__(None, None, None)
            os.makedirs(self.out_dir, exist_ok=True)
            path = os.path.join(self.out_dir, f"trace_rank{self.rank}.json")
            self._prof.export_chrome_trace(path)
            sort = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
            with open(os.path.join(self.out_dir, f"kernels_rank{self.rank}.txt"), "w") as f:
                f.write(self._prof.key_averages().table(sort_by=sort, row_limit=60))
            logger.info("profiler trace written to %s", path)
            self._prof, self._done = None, True

    def on_epoch_end(self, trainer, epoch, logs):
        pass

    def on_train_end(self, trainer):
        if self._prof is not None:
            self._prof.__exit__(None, None, None)
            self._prof = None
        set_ranges(False)
