from .estimator import HuggingFace, LocalEstimator
from .spawn import launch, maybe_self_spawn, visible_gpu_count

__all__ = ["LocalEstimator", "HuggingFace", "launch", "maybe_self_spawn", "visible_gpu_count"]
