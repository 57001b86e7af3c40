"""HIP (gfx950) implementations of the fused ops, as autograd Functions over ``_C`` kernels.

Weight gradients are written straight into the flat ``main_grad`` buffer
(:class:`parallel.FlatParamStore`) by the backward kernels, which then signal bucket readiness
(``p._hsd_ready``) so the RCCL all-reduce of a completed bucket overlaps the rest of backward.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import load

_C = load()


def adam_step(p, m, v, g, out, decay, step, eps, b1, b2, gscale, lr_wd):
    _C.adam_step(p, m, v, g, out, decay, step, eps, b1, b2, gscale, lr_wd)
