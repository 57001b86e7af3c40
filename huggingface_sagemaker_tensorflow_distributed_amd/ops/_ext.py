"""Loader for the compiled gfx950 extension (``_C.so``, built in-tree by ``_build.py``).

On a GPU machine the HIP path is mandatory: if the shared object is missing we try to build it
(hipcc is part of the image) and otherwise raise — ops never fall back silently to eager PyTorch.
``HSD_DEBUG=1`` loads the debug build ``_C_debug.so`` instead (synchronising launch checks, device
asserts, host-side index range checks; ``python -m ..._build --debug``).
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
        debug = os.environ.get("HSD_DEBUG", "0") not in ("", "0")
        name = "huggingface_sagemaker_tensorflow_distributed_amd." + ("_C_debug" if debug else "_C")
        try:
            _mod = importlib.import_module(name)
        except ImportError as e:
            if os.environ.get("HSD_NO_AUTOBUILD"):
                raise RuntimeError(f"native extension {name} is missing; run `python -m "
                                   "huggingface_sagemaker_tensorflow_distributed_amd._build"
                                   f"{' --debug' if debug else ''}`") from e
            from .. import _build

            _build.build(debug=debug)
            _mod = importlib.import_module(name)
    return _mod
