from . import backend
from .backend import barrier, init, is_distributed, local_rank, local_size, rank, shutdown, size, state
from .collectives import allreduce_sums, broadcast_object, broadcast_parameters, params_in_sync
from .ddp import GradBucketer
from .flat_params import FlatParamStore
from .sampler import ShardSampler

__all__ = [
    "backend", "init", "rank", "size", "local_rank", "local_size", "barrier", "is_distributed", "shutdown",
    "state", "allreduce_sums", "broadcast_object", "broadcast_parameters", "params_in_sync", "GradBucketer",
    "FlatParamStore", "ShardSampler",
]
