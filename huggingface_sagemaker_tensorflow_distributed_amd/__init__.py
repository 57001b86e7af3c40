"""MI355X-native data-parallel transformer fine-tuning framework.

Capabilities of ``philschmid/huggingface_sagemaker_tensorflow_distributed`` (a SageMaker/TF2/Horovod
BERT fine-tuning job), re-designed for AMD Instinct MI355X (gfx950): PyTorch-ROCm framework layer,
hand-written HIP/CDNA4 kernels for the BERT hot path, RCCL-over-xGMI bucketed all-reduce.

The top level doubles as the ``hvd``-style facade the reference script programs against
(``scripts/train.py:16-31,112-133``)::

    import huggingface_sagemaker_tensorflow_distributed_amd as hvd
    hvd.init(); hvd.rank(); hvd.size(); hvd.local_rank()
    hvd.allreduce(t) / hvd.allgather(t) / hvd.broadcast(t, 0) / hvd.broadcast_object(obj, 0)
"""
from __future__ import annotations

__version__ = "0.1.0"

from .parallel.backend import barrier, init, is_distributed, local_rank, local_size, rank, shutdown, size


class Compression:  # noqa: N801 - Horovod's ``hvd.Compression`` namespace
    """Wire dtype of the gradient all-reduce: ``none`` (fp32), ``fp16`` (Horovod's), ``bf16`` (MI355X-native)."""

    none = "none"
    fp16 = "fp16"
    bf16 = "bf16"


def DistributedOptimizer(optimizer, store=None, bucket_mb=None, compression=Compression.none,
                         backward_passes_per_step: int = 1):
    """``hvd.DistributedOptimizer(opt, compression=..., backward_passes_per_step=...)``: a wrapped optimizer whose
    ``step()`` applies the rank-averaged gradient (``parallel/dist_optim.py``). ``.bucketer`` is the underlying
    RCCL bucket engine (None in a single process); the wrapped optimizer's attributes (``lr``, state) pass through."""
    from .parallel.dist_optim import DistributedOptimizer as _DO

    return _DO(optimizer, store=store, bucket_mb=bucket_mb, compression=compression,
               backward_passes_per_step=backward_passes_per_step)


class callbacks:  # noqa: N801 - the ``hvd.callbacks`` namespace
    """``hvd.callbacks.BroadcastGlobalVariablesCallback`` / ``MetricAverageCallback`` equivalents (train/callbacks.py)."""

    from .train.callbacks import BroadcastGlobalVariablesCallback, MetricAverageCallback  # noqa: F401


from .parallel.collectives import Average, Max, Min, Sum  # noqa: E402
from .parallel.collectives import hvd_allgather as allgather  # noqa: E402
from .parallel.collectives import hvd_allgather_object as allgather_object  # noqa: E402
from .parallel.collectives import hvd_allreduce as allreduce  # noqa: E402
from .parallel.collectives import hvd_broadcast as broadcast  # noqa: E402


def broadcast_object(obj, root_rank: int = 0):
    """``hvd.broadcast_object``: ``root_rank``'s picklable object on every rank."""
    from .parallel.collectives import broadcast_object as _bo

    return _bo(obj, src=root_rank)


def broadcast_parameters(store, optimizer=None, root_rank: int = 0):
    from .parallel.collectives import broadcast_parameters as _b

    _b(store, optimizer, src=root_rank)


__all__ = ["init", "rank", "size", "local_rank", "local_size", "barrier", "is_distributed", "shutdown",
           "DistributedOptimizer", "Compression", "broadcast_parameters", "callbacks", "allreduce", "allgather", "broadcast",
           "broadcast_object", "allgather_object", "Average", "Sum", "Min", "Max", "__version__"]
