"""Python side of the native RCCL communication engine (``csrc/comm/comm_engine.cpp``).

The reference's data-parallel runtime is Horovod's C++ core over NCCL (``hvd.init()``,
``hvd.DistributedOptimizer``, ``BroadcastGlobalVariablesCallback`` — ``scripts/train.py:24,114,133``;
SURVEY.md §2.5 C.1). Here one :class:`CommEngine` per process owns an RCCL communicator (xGMI between
the GPUs of a node), a high-priority HIP stream for collectives and the static gradient buckets; the
``ncclUniqueId`` travels through torch's TCPStore (the rendezvous ``torch.distributed`` already made),
so no MPI is involved.

``get_engine()`` returns ``None`` when the native path does not apply (CPU / gloo worlds, a world of
one, or ``HSD_COMM=torch``), and callers fall back to ``torch.distributed`` collectives — the same
RCCL library underneath on GPUs, but without the engine's bucket bookkeeping in C++.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from . import backend

logger = logging.getLogger(__name__)

_ENGINE = None
_ENGINE_KEY = None
_SERIAL = [0]
_DISABLED = [False]


def native_requested() -> bool:
    return os.environ.get("HSD_COMM", "native").lower() != "torch"


def _all_ranks_ok(ok: bool, device) -> bool:
    """Agreement over the torch process group (its own RCCL communicator): True iff every rank passes ``ok``."""
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def get_engine():
    """The process's :class:`CommEngine` (created on first use), or ``None`` if not applicable.

    Creation is agreed collectively: if any rank fails to load the extension, to build the communicator or to
    pass the all-reduce self-test, EVERY rank falls back to ``torch.distributed`` (logged), so a native-engine
    problem costs the overlap bookkeeping, never a hang or a crashed job."""
    global _ENGINE, _ENGINE_KEY
    st = backend.state()
    if st.world_size <= 1 or st.device.type != "cuda" or st.backend != "nccl" or not native_requested():
        return None
    if not dist.is_initialized() or _DISABLED[0]:
        return None
    key = (st.rank, st.world_size, st.device.index)
    if _ENGINE is not None and _ENGINE_KEY == key:
        return _ENGINE
    C, err = None, None
    try:
        from ..ops._ext import load

        C = load()
    except Exception as e:  # noqa: BLE001 - any failure -> agreed fallback below
        err = e
    if not _all_ranks_ok(C is not None, st.device):
        return _disable(f"extension unavailable on some rank ({err!r})")
    store = dist.distributed_c10d._get_default_store()
    _SERIAL[0] += 1
    skey = f"hsd/comm_uid/{_SERIAL[0]}"
    if st.rank == 0:
        uid = C.CommEngine.unique_id()
        store.set(skey, uid)
    else:
        store.wait([skey])
        uid = store.get(skey)
    eng, ok = None, False
    try:
        eng = C.CommEngine(st.rank, st.world_size, bytes(uid), st.device.index, True)
        # one-time self-test: an all-reduce of ones must give the world size everywhere
        t = torch.ones(256, dtype=torch.float32, device=st.device)
        eng.allreduce(t, True)
        ok = bool(torch.all(t == float(st.world_size)).item())
        if not ok:
            err = RuntimeError("CommEngine self-test failed (all-reduce of ones != world size)")
    except Exception as e:  # noqa: BLE001
        err = e
    if not _all_ranks_ok(ok, st.device):
        return _disable(f"native engine failed on some rank ({err!r})")
    logger.info("native RCCL CommEngine up: rank %d/%d device %d", st.rank, st.world_size, st.device.index)
    _ENGINE, _ENGINE_KEY = eng, key
    return eng


def _disable(why: str):
    _DISABLED[0] = True
    logger.warning("native RCCL CommEngine disabled, using torch.distributed collectives: %s", why)
    return None


def native_active() -> bool:
    """True once the native engine is up (False after an agreed fallback)."""
    return _ENGINE is not None and not _DISABLED[0]


def reset() -> None:
    global _ENGINE, _ENGINE_KEY
    _ENGINE, _ENGINE_KEY = None, None
    _DISABLED[0] = False


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    eng = get_engine()
    if eng is not None and t.is_cuda and t.is_contiguous():
        eng.broadcast(t, src)
    elif backend.is_distributed():
        dist.broadcast(t, src=src)
    return t


def allreduce_(t: torch.Tensor) -> torch.Tensor:
    eng = get_engine()
    if eng is not None and t.is_cuda and t.is_contiguous():
        eng.allreduce(t, True)
    elif backend.is_distributed():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t
