"""Host -> device batch pipeline.

Replaces ``tf.data.Dataset.from_tensor_slices(...).batch(B)`` (``scripts/train.py:84-86``). Batches
are gathered from the in-memory arrays into pinned host buffers by a background thread and copied
to the GPU with non-blocking H2D on a dedicated copy stream, so the input pipeline never sits on
the compute stream's critical path.
"""
from __future__ import annotations

import queue
import threading
from typing import Dict, Iterator, Optional

import numpy as np
import torch

from ..parallel.sampler import ShardSampler
from .datasets import ArrayDataset


class _Failure:
    __slots__ = ("exc",)

    def __init__(self, exc: BaseException):
        self.exc = exc


class BatchLoader:
    def __init__(self, ds: ArrayDataset, sampler: ShardSampler, device: torch.device, prefetch: int = 3):
        self.ds = ds
        self.sampler = sampler
        self.device = torch.device(device)
        self.prefetch = prefetch
        self._cuda = self.device.type == "cuda"
        self._stream = torch.cuda.Stream(device=self.device) if self._cuda else None

    def __len__(self) -> int:
        return self.sampler.num_batches()

    def _host_batch(self, idx) -> Dict[str, torch.Tensor]:
        ix = np.asarray(idx, dtype=np.int64)
        pad = ix < 0  # ShardSampler(mark_padding=True): repeats that only even out the ranks
        if pad.any():
            ix = np.where(pad, -ix - 1, ix)
        labels = self.ds.labels[ix].astype(np.int64)
        if pad.any():
            labels[pad] = -100  # ignored by the loss and by the metric meter
        b = {
            "input_ids": torch.from_numpy(self.ds.input_ids[ix].astype(np.int64)),
            "attention_mask": torch.from_numpy(self.ds.attention_mask[ix].astype(np.int64)),
            "labels": torch.from_numpy(labels),
        }
        if self._cuda:
            b = {k: v.pin_memory() for k, v in b.items()}
        if pad.any():
            b["num_valid"] = int((~pad).sum())  # host int: lets evaluate skip an all-padding batch without a sync
        return b

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        stop = object()

        def work():
            try:
                for idx in self.sampler.batches():
                    q.put(self._host_batch(idx))
            except BaseException as e:  # surfaces in the consumer instead of silently ending the epoch
                q.put(_Failure(e))
            finally:
                q.put(stop)

        t = threading.Thread(target=work, daemon=True)
        t.start()
        while True:
            hb = q.get()
            if hb is stop:
                break
            if isinstance(hb, _Failure):
                t.join()
                raise RuntimeError("batch prefetch thread failed") from hb.exc
            if self._cuda:
                with torch.cuda.stream(self._stream):
                    db = {k: (v.to(self.device, non_blocking=True) if torch.is_tensor(v) else v)
                          for k, v in hb.items()}
                ev = self._stream.record_event()
                torch.cuda.current_stream(self.device).wait_event(ev)
                for v in db.values():
                    if torch.is_tensor(v):
                        v.record_stream(torch.cuda.current_stream(self.device))
                yield db
            else:
                yield hb
        t.join()
