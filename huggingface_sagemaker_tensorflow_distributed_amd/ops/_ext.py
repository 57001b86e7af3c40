"""Loader for the compiled gfx950 extension (``_C.so``, built in-tree by ``_build.py``).

On a GPU machine the HIP path is mandatory: if the shared object is missing we try to build it
(hipcc is part of the image) and otherwise raise — ops never fall back silently to eager PyTorch.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = importlib.import_module("huggingface_sagemaker_tensorflow_distributed_amd._C")
        except ImportError as e:
            if os.environ.get("HSD_NO_AUTOBUILD"):
                raise RuntimeError("native extension _C.so is missing; run "
                                   "`python -m huggingface_sagemaker_tensorflow_distributed_amd._build`") from e
            from .. import _build

            _build.build()
            _mod = importlib.import_module("huggingface_sagemaker_tensorflow_distributed_amd._C")
    return _mod
