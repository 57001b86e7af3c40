"""Throughput meter: whole-node sequences/sec measured with device events.

Step time comes from events recorded on the compute stream at every step end (so it measures the
device, not host enqueue), warmup steps are excluded, and the per-rank times are max-reduced so the
reported number is the slowest rank's (what a synchronous DP job achieves). Writes ``metrics.jsonl``
(one line per log interval) and ``benchmark.json`` at the end of training on rank 0.
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Dict, List, Optional

import torch

from ..parallel import backend

logger = logging.getLogger(__name__)


class ThroughputMeter:
    def __init__(self, out_dir: str, per_rank_batch: int, seq_len: int, warmup: int = 3, log_every: int = 50,
                 info: Optional[Dict] = None):
        self.out_dir = out_dir
        self.per_rank_batch = int(per_rank_batch)
        self.seq_len = int(seq_len)
        self.warmup = max(0, int(warmup))
        self.log_every = int(log_every)
        self.info = dict(info or {})
        self.cuda = torch.cuda.is_available()
        self._events: List = []
        self._t_host: List[float] = []
        self.result: Optional[Dict] = None

    def _stamp(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    @staticmethod
    def _elapsed_ms(a, b) -> float:
        if isinstance(a, float):
            return (b - a) * 1e3
        return a.elapsed_time(b)

    def on_train_begin(self, trainer):
        self._events = []
        # per-bucket comm timeline (native RCCL engine only; other bucketers report False)
        buck = getattr(trainer, "bucketer", None)
        set_timing = getattr(buck, "set_timing", None)
        self._timing = bool(set_timing(True)) if set_timing is not None else False

    def on_batch_end(self, trainer, step):
        self._events.append(self._stamp())
        n = len(self._events)
        if self.log_every and backend.rank() == 0 and n > self.warmup + 1 and n % self.log_every == 0:
            if self.cuda:
                self._events[-1].synchronize()
            ms = self._elapsed_ms(self._events[self.warmup], self._events[-1]) / (n - 1 - self.warmup)
            self._append({"step": trainer.global_step, "ms_per_step": ms,
                          "seq_per_s_rank": self.per_rank_batch * 1e3 / ms, "time": time.time()})

    def on_epoch_end(self, trainer, epoch, logs):
        pass

    def _append(self, rec: Dict) -> None:
        os.makedirs(self.out_dir, exist_ok=True)
        with open(os.path.join(self.out_dir, "metrics.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")

    def on_train_end(self, trainer):
        n = len(self._events)
        timed = n - 1 - self.warmup
        if timed < 1:
            return
        if self.cuda:
            torch.cuda.synchronize()
        ms = self._elapsed_ms(self._events[self.warmup], self._events[-1]) / timed
        t = torch.tensor([ms], dtype=torch.float64, device=trainer.device)
        if backend.is_distributed():
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        ms = float(t.item())
        world = backend.size()
        comm = None
        if getattr(self, "_timing", False):
            comm = trainer.bucketer.overlap_report()  # last step's bucket timeline (this rank)
            trainer.bucketer.set_timing(False)
        seqs = self.per_rank_batch * world * 1e3 / ms
        self.result = {
            "metric": "sequences/sec (whole node)", "value": seqs, "seq_per_s_per_gpu": seqs / world,
            "tokens_per_s": seqs * self.seq_len, "ms_per_step": ms, "n_gpus": world, "timed_steps": timed,
            "warmup_steps": self.warmup, "per_gpu_batch": self.per_rank_batch, "global_batch": self.per_rank_batch * world,
            "seq_len": self.seq_len, **self.info,
        }
        if comm is not None:
            self.result["comm_overlap"] = comm
        if backend.rank() == 0:
            os.makedirs(self.out_dir, exist_ok=True)
            with open(os.path.join(self.out_dir, "benchmark.json"), "w") as f:
                json.dump(self.result, f, indent=1)
            logger.info("throughput: %.1f seq/s whole node (%.1f per GPU), %.2f ms/step over %d steps", seqs,
                        seqs / world, ms, timed)
