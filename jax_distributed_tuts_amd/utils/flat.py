"""Flat parameter storage: one fp32 master buffer, its bf16 compute shadow and
one fp32 gradient buffer, with named views.

The reference keeps params as a flax pytree and lets XLA fuse the per-leaf
AdamW, casts and grad accumulation (util.py:74-77, data_paral.py:214-217).
On MI355X the whole state is three contiguous buffers instead, so that

* the optimizer is ONE fused kernel over all 407,050 elements (K14),
* the DP gradient sync is ONE all-reduce of one buffer (X03) -- the 4 metric
  scalars ride along in a trailing slot (X04),
* every GEMM reads the bf16 shadow the optimizer wrote (K02), never casting.

Each view starts on a 64-element (256 B) boundary so vector loads stay aligned.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

ALIGN = 64
N_METRIC_SLOTS = 4  # [loss_sum, loss_count, correct_sum, acc_count]


@dataclass
class ParamSpec:
    name: str                 # flax-style path, e.g. "input_dense/kernel"
    shape: Tuple[int, ...]
    init: str = "lecun_normal"  # | "zeros" | "ones" | "normal:<std>"


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def init_tensor(spec: ParamSpec, gen: torch.Generator) -> torch.Tensor:
    """flax defaults: kernels lecun_normal (truncated normal, var 1/fan_in), biases zeros."""
    shape = spec.shape
    if spec.init == "zeros":
        return torch.zeros(shape)
    if spec.init == "ones":
        return torch.ones(shape)
    if spec.init.startswith("normal:"):
        std = float(spec.init.split(":", 1)[1])
        return torch.randn(shape, generator=gen) * std
    if spec.init == "lecun_normal":
        fan_in = int(math.prod(shape[:-1])) if len(shape) > 1 else shape[0]
        # truncated at +-2 sigma; 0.87962566 rescales to unit variance (jax.nn.initializers)
        std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
        t = torch.empty(shape)
        torch.nn.init.trunc_normal_(t, mean=0.0, std=1.0, a=-2.0, b=2.0, generator=gen)
        return t * std
    raise ValueError(f"unknown init {spec.init}")


class FlatParams:
    """Named views into flat fp32 master / bf16 shadow / fp32 grad buffers."""

    def __init__(self, specs: Sequence[ParamSpec], device="cpu", *, with_grad: bool = True,
                 with_shadow: bool = True, metric_slots: int = N_METRIC_SLOTS):
        self.specs: List[ParamSpec] = list(specs)
        self.device = torch.device(device)
        self.offsets: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
        off = 0
        for s in self.specs:
            self.offsets[s.name] = (off, tuple(s.shape))
            off += _align(int(math.prod(s.shape)))
        self.numel = off                     # optimizer range (padded, pads stay 0)
        self.metric_off = off
        total = off + (_align(metric_slots) if metric_slots else 0)
        self.master = torch.zeros(total, dtype=torch.float32, device=self.device)
        self.shadow = torch.zeros(total, dtype=torch.bfloat16, device=self.device) if with_shadow else None
        self.grad = torch.zeros(total, dtype=torch.float32, device=self.device) if with_grad else None
        self.metric_slots = metric_slots

    # -- views ---------------------------------------------------------------
    def _view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        off, shape = self.offsets[name]
        return buf[off: off + int(math.prod(shape))].view(shape)

    def p(self, name: str) -> torch.Tensor:
        return self._view(self.master, name)

    def s(self, name: str) -> torch.Tensor:
        return self._view(self.shadow, name)

    def g(self, name: str) -> torch.Tensor:
        return self._view(self.grad, name)

    @property
    def metrics_slot(self) -> torch.Tensor:
        """The 4 metric scalars that share the gradient all-reduce bucket."""
        return self.grad[self.metric_off: self.metric_off + N_METRIC_SLOTS]

    @property
    def grad_params(self) -> torch.Tensor:
        return self.grad[: self.numel]

    def names(self) -> List[str]:
        return [s.name for s in self.specs]

    # -- init / sync ---------------------------------------------------------
    def init_(self, seed: int, only: Optional[Callable[[str], bool]] = None) -> "FlatParams":
        gen = torch.Generator().manual_seed(int(seed))
        for s in self.specs:
            t = init_tensor(s, gen)  # always drawn, so the stream does not depend on `only`
            if only is None or only(s.name):
                self.p(s.name).copy_(t.to(self.device))
        self.sync_shadow()
        return self

    def sync_shadow(self):
        if self.shadow is not None:
            from ..ops.kernels import cast_bf16_

            cast_bf16_(self.master[: self.numel], self.shadow[: self.numel])

    def zero_grad(self):
        if self.grad is not None:
            self.grad.zero_()

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {n: self.p(n).detach().clone() for n in self.names()}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        for n in self.names():
            self.p(n).copy_(sd[n].to(self.device))
        self.sync_shadow()

    def num_params(self) -> int:
        return sum(int(math.prod(s.shape)) for s in self.specs)
