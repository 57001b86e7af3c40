"""Process-group lifecycle: the ``hvd.init()`` / device-pinning equivalent.

Reference behaviour: ``hvd.init()`` at import time (``scripts/train.py:24``) then one GPU per
process (``scripts/train.py:27-31``). Here: one process per GPU, ``torch.distributed`` with backend
``nccl`` (= RCCL on ROCm, over xGMI) on GPUs, ``gloo`` on CPU. A world of one is a valid world with
no-op collectives.
"""
from __future__ import annotations

import datetime
import logging
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.env import dist_env

logger = logging.getLogger(__name__)


@dataclass
class DistState:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    initialized_here: bool = False


_STATE = DistState()


def _want_cuda(device: Optional[str]) -> bool:
    if device is not None:
        return device.startswith("cuda")
    return torch.cuda.is_available()


def init(device: Optional[str] = None, timeout_s: float = 1800.0, backend: Optional[str] = None) -> DistState:
    """Initialise (idempotent). Reads RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* (or MPI/Horovod vars)."""
    global _STATE
    env = dist_env()
    use_cuda = _want_cuda(device)
    if use_cuda:
        from . import rccl_env

        rccl_env.apply(env["world_size"])  # before any communicator exists
    if use_cuda:
        torch.cuda.set_device(env["local_rank"] % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    # HSD_DIST_BACKEND=gloo: force the CPU-transport backend (e.g. several ranks sharing one GPU in a test)
    be = backend or os.environ.get("HSD_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    here = False
    if env["world_size"] > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = dict(backend=be, rank=env["rank"], world_size=env["world_size"],
                  timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
        here = True
        logger.info("process group up: backend=%s rank=%d/%d local_rank=%d", be, env["rank"], env["world_size"],
                    env["local_rank"])
    _STATE = DistState(rank=env["rank"], world_size=env["world_size"], local_rank=env["local_rank"],
                       local_world_size=env["local_world_size"],
                       backend=be if env["world_size"] > 1 else "none", device=dev, initialized_here=here)
    return _STATE


def state() -> DistState:
    return _STATE


def rank() -> int:
    return _STATE.rank


def size() -> int:
    return _STATE.world_size


def local_rank() -> int:
    return _STATE.local_rank


def local_size() -> int:
    return _STATE.local_world_size


def is_distributed() -> bool:
    return _STATE.world_size > 1 and dist.is_initialized()


def barrier() -> None:
    if is_distributed():
        if _STATE.backend == "nccl":
            dist.barrier(device_ids=[_STATE.device.index])
        else:
            dist.barrier()


def shutdown() -> None:
    global _STATE
    if dist.is_initialized() and _STATE.initialized_here:
        dist.destroy_process_group()
    _STATE = DistState()
