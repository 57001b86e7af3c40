"""SageMaker-style environment contract (SURVEY.md §2.7 'Environment contract').

The reference reads ``SM_OUTPUT_DATA_DIR``, ``SM_MODEL_DIR``, ``SM_NUM_GPUS``
(``scripts/train.py:48-50``) and probes ``SM_FRAMEWORK_PARAMS`` through
``transformers.file_utils.is_sagemaker_dp_enabled`` (``scripts/train.py:16``).
Our launcher (``launcher/smenv.py``) writes all of them; outside a launcher we fall back to a
local ``./output`` tree instead of raising ``KeyError``.
"""
from __future__ import annotations

import json
import os

_LOCAL_DEFAULTS = {
    "SM_OUTPUT_DATA_DIR": os.path.join("output", "data"),
    "SM_MODEL_DIR": os.path.join("output", "model"),
    "SM_NUM_GPUS": None,  # resolved lazily
}


def _local_gpu_count() -> int:
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover - torch always importable here
        return 0


def sm_default(name: str) -> str:
    v = os.environ.get(name)
    if v is not None:
        return v
    if name == "SM_NUM_GPUS":
        return str(_local_gpu_count())
    return _LOCAL_DEFAULTS[name]


def framework_params() -> dict:
    raw = os.environ.get("SM_FRAMEWORK_PARAMS", "{}")
    try:
        v = json.loads(raw)
        return v if isinstance(v, dict) else {}
    except json.JSONDecodeError:
        return {}


def is_sagemaker_dp_enabled() -> bool:
    """Same probe semantics as transformers' helper: the JSON key must be true.

    (The reference additionally requires the ``smdistributed`` package; our RCCL engine serves
    the SMDDP request, so only the flag matters here.)
    """
    return bool(framework_params().get("sagemaker_distributed_dataparallel_enabled", False))


def is_sagemaker_mpi_enabled() -> bool:
    p = framework_params()
    return bool(p.get("sagemaker_mpi_enabled", False))


def dist_env() -> dict:
    """Rank/world information from torchrun-style variables, falling back to MPI/Horovod ones."""

    def first(*names, default=None):
        for n in names:
            if n in os.environ:
                return os.environ[n]
        return default

    rank = int(first("RANK", "OMPI_COMM_WORLD_RANK", "HOROVOD_RANK", "PMI_RANK", default=0))
    world = int(first("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "HOROVOD_SIZE", "PMI_SIZE", default=1))
    local_rank = int(first("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "HOROVOD_LOCAL_RANK", default=rank))
    local_world = int(first("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "HOROVOD_LOCAL_SIZE", default=world))
    return {"rank": rank, "world_size": world, "local_rank": local_rank, "local_world_size": local_world}
