from .adam import FusedAdam

__all__ = ["FusedAdam"]
