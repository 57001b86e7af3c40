"""Fused Adam / AdamW over the flat parameter store — one kernel launch per step.

Reference optimizer: ``tf.keras.optimizers.Adam(learning_rate)`` (``scripts/train.py:113``,
``scripts/singe_node_train.py:78``) — TF 2.4 Keras defaults β1=0.9, β2=0.999, ε=1e-7, no weight decay,
and the ε-hat update::

    lr_t = lr·√(1-β2ᵗ)/(1-β1ᵗ);  m = β1 m + (1-β1) g;  v = β2 v + (1-β2) g²;  θ -= lr_t·m/(√v + ε)

PyTorch's form divides √v by √(1-β2ᵗ) before adding ε; both are ``θ -= step·m/(√v + ε_eff)`` with
``ε_eff = ε`` (keras) or ``ε·√(1-β2ᵗ)`` (torch), so one kernel serves both (``eps_mode``).
The DP ``1/N`` gradient average (``hvd.DistributedOptimizer`` semantics) and the optional
gradient-accumulation ``1/k`` are folded into ``grad_scale``; with bf16 compute the kernel also
writes the bf16 weight copy the next forward reads (no separate cast pass).
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional

import torch

from ..parallel.flat_params import ALIGN, FlatParamStore


class FusedAdam:
    def __init__(self, store: FlatParamStore, lr: float = 1e-3, betas=(0.9, 0.999), eps: Optional[float] = None,
                 weight_decay: float = 0.0, eps_mode: str = "keras", decoupled: bool = True):
        if eps_mode not in ("keras", "torch"):
            raise ValueError(eps_mode)
        self.store = store
        self.lr = float(lr)
        self.beta1, self.beta2 = map(float, betas)
        self.eps = float(eps if eps is not None else (1e-7 if eps_mode == "keras" else 1e-8))
        self.eps_mode = eps_mode
        self.weight_decay = float(weight_decay)
        self.decoupled = decoupled
        self.step_count = 0
        self.exp_avg = torch.zeros_like(store.master)
        self.exp_avg_sq = torch.zeros_like(store.master)
        self._decay_mask = store.decay_block_mask(ALIGN) if weight_decay else None

    # --------------------------------------------------------------------------
    def state_tensors(self) -> List[torch.Tensor]:
        return [self.exp_avg, self.exp_avg_sq]

    def state_dict(self) -> dict:
        return {"step": self.step_count, "exp_avg": self.exp_avg.cpu(), "exp_avg_sq": self.exp_avg_sq.cpu(),
                "lr": self.lr, "betas": (self.beta1, self.beta2), "eps": self.eps, "eps_mode": self.eps_mode,
                "weight_decay": self.weight_decay}

    def load_state_dict(self, sd: dict) -> None:
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"].to(self.exp_avg.device))
        self.exp_avg_sq.copy_(sd["exp_avg_sq"].to(self.exp_avg_sq.device))

    def _coeffs(self):
        t = self.step_count
        bc1 = 1.0 - self.beta1 ** t
        bc2 = 1.0 - self.beta2 ** t
        step = self.lr * math.sqrt(bc2) / bc1
        eps_eff = self.eps if self.eps_mode == "keras" else self.eps * math.sqrt(bc2)
        return step, eps_eff

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0) -> None:
        self.step_count += 1
        step, eps_eff = self._coeffs()
        s = self.store
        write_compute = s.compute is not s.master
        if s.master.is_cuda:
            from ..ops import hip

            hip.join_side_streams()  # weight gradients may still be in flight on the wgrad stream
            hip.adam_step(s.master, self.exp_avg, self.exp_avg_sq, s.grad, s.compute if write_compute else None,
                          self._decay_mask, step, eps_eff, self.beta1, self.beta2, float(grad_scale),
                          self.lr * self.weight_decay)
            s.refresh_transposed()
            return
        # reference path (CPU): identical math on flat buffers
        g = s.grad.to(torch.float32) * grad_scale
        if self.weight_decay:
            wd = self._decay_mask.repeat_interleave(ALIGN)[: s.numel].to(torch.float32)
            s.master.mul_(1.0 - self.lr * self.weight_decay * wd)
        self.exp_avg.mul_(self.beta1).add_(g, alpha=1.0 - self.beta1)
        self.exp_avg_sq.mul_(self.beta2).addcmul_(g, g, value=1.0 - self.beta2)
        s.master.addcdiv_(self.exp_avg, self.exp_avg_sq.sqrt().add_(eps_eff), value=-step)
        if write_compute:
            s.compute.copy_(s.master)
