from .callbacks import Callback, ModelCheckpoint, load_checkpoint, save_checkpoint
from .trainer import History, Trainer

__all__ = ["Trainer", "History", "Callback", "ModelCheckpoint", "save_checkpoint", "load_checkpoint"]
