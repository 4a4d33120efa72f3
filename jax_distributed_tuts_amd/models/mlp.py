"""MLP classifiers with an explicit (hand-scheduled) backward pass.

Reference model (data_paral.py:75-102, param_sharding.py:194-224)::

    Dense(512, dtype=bf16, name="input_dense") -> silu -> Dropout(0.1)
    -> Dense(10, dtype=bf16, name="output_dense") -> float32

``MLP(dims=[784, 512, 10])`` is exactly that model (param names, [in,out]
kernel layout, lecun_normal/zeros init, bf16 compute, fp32 params).
``dims=[784, 512, 512, 512, 10]`` is the 4-layer MLP of BASELINE config #2 and
``MLPStage`` slices any MLP into pipeline stages (config #4).

Why an explicit backward instead of autograd: every hidden layer's backward is
exactly two GEMM launches on MI355X --
    dW_i += h_{i-1}^T . dz_i                          (fp32, accumulated in place)
    dz_{i-1} = (dz_i . W_i^T) * mask/keep * act'(z_{i-1}), db_{i-1} += colsum
the second folding the lower layer's activation-grad, dropout mask and bias
grad into its epilogue.  The softmax-CE kernel produces dz of the top layer and
its bias grad.  So one minibatch fwd+bwd of the reference classifier is 5
kernels (2 fwd GEMMs, CE, 2 bwd GEMMs + 1 dW GEMM) with no elementwise passes,
no grad-accumulation adds (K12) and no mask tensors (K04).

``backward(..., on_ready=cb)`` reports each layer's params as soon as their
grads are final, which the DP trainer uses to launch bucketed all-reduces that
overlap the rest of the backward pass.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from ..ops import kernels as K
from ..utils import rng as R
from ..utils.flat import FlatParams, ParamSpec


@dataclass
class LayerCache:
    x: torch.Tensor                       # input of the stack (fp32 data or bf16 activations)
    z: List[Optional[torch.Tensor]] = field(default_factory=list)  # pre-activations (bf16) of hidden layers
    h: List[torch.Tensor] = field(default_factory=list)            # layer outputs (bf16)
    offsets: List[int] = field(default_factory=list)
    seed: int = 0
    keep: float = 1.0
    step: Optional[torch.Tensor] = None


class MLP:
    """Dense stack.  Layer i maps dims[i] -> dims[i+1]; every layer except the
    last applies act + dropout (the last too if ``final_act``)."""

    def __init__(self, dims: Sequence[int], act: str = "silu", dropout_rate: float = 0.1,
                 names: Optional[Sequence[str]] = None, final_act: bool = False, layer_id_base: int = 0):
        self.dims = list(dims)
        self.L = len(dims) - 1
        self.act = act
        self.dropout_rate = float(dropout_rate)
        self.final_act = final_act
        if names is None:
            if self.L == 2:
                names = ["input_dense", "output_dense"]
            else:
                names = ["input_dense"] + [f"hidden_dense_{i}" for i in range(1, self.L - 1)] + ["output_dense"]
        self.names = list(names)
        self.layer_id_base = layer_id_base  # folds into the dropout stream so stages differ

    # ------------------------------------------------------------------ flax-style apply
    def __call__(self, variables, x: torch.Tensor, train: bool = False, rngs: Optional[dict] = None) -> torch.Tensor:
        """``model.apply({"params": params}, x, train=..., rngs={"dropout": key})`` of
        the reference (data_paral.py:180, 86-100) as a DIFFERENTIABLE forward: nested
        ``params[layer]["kernel" | "bias"]`` tensors, one ``ops.autograd.dense``
        (GEMM + bias + act + dropout epilogue on the HIP kernels) per layer, fp32
        logits.  Used by reference-style ``loss_fn``s through ``util.accum_grads``."""
        from ..ops.autograd import dense

        params = variables["params"] if "params" in variables else variables
        keep = 1.0 - self.dropout_rate if train else 1.0
        key = (rngs or {}).get("dropout", 0)
        seed = int(key) & 0xFFFFFFFF
        # a graph-replayed scan minibatch (utils.rng.ScanKey): its key is selected on the device
        seed_dev = key.device_seed() if (isinstance(key, R.ScanKey) and keep < 1.0) else None
        h = x
        for i, n in enumerate(self.names):
            hid = self._hidden(i)
            h = dense(h, params[n]["kernel"], params[n]["bias"], act=self.act if hid else "none",
                      keep=keep if hid else 1.0, seed=seed, offset=(self.layer_id_base + i) << 1,
                      seed_dev=seed_dev if hid else None)
        return h.float()

    apply = __call__

    # ------------------------------------------------------------------ params
    def param_specs(self) -> List[ParamSpec]:
        out = []
        for i, n in enumerate(self.names):
            out.append(ParamSpec(f"{n}/kernel", (self.dims[i], self.dims[i + 1]), "lecun_normal"))
            out.append(ParamSpec(f"{n}/bias", (self.dims[i + 1],), "zeros"))
        return out

    # stage / loss-head metadata shared with TransformerLM (pipeline + loss code is model-agnostic)
    @property
    def head_bias_name(self) -> Optional[str]:
        return None if self.final_act else f"{self.names[-1]}/bias"

    def input_shape(self, rows: int):
        return (rows, self.dims[0])

    def input_dtype(self):
        return torch.bfloat16

    def output_shape(self, rows: int):
        return (rows, self.dims[-1])

    @staticmethod
    def flatten_labels(y: torch.Tensor) -> torch.Tensor:
        return y

    def _hidden(self, i: int) -> bool:
        return i < self.L - 1 or self.final_act

    # ------------------------------------------------------------------ forward
    def forward(self, P: FlatParams, x: torch.Tensor, *, train: bool = False, seed: int = 0, offset: int = 0,
                step: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, LayerCache]:
        keep = 1.0 - self.dropout_rate if train else 1.0
        cache = LayerCache(x=x, seed=seed, keep=keep, step=step)
        h = x
        M = x.shape[0]
        for i, n in enumerate(self.names):
            hid = self._hidden(i)
            out = torch.empty(M, self.dims[i + 1], dtype=torch.bfloat16, device=x.device)
            z = torch.empty_like(out) if hid else None
            off = int(offset) + ((self.layer_id_base + i) << 1)
            K.gemm(h, P.s(f"{n}/kernel"), a_layout="mk", b_layout="kn", out=out, bias=P.s(f"{n}/bias"),
                   act=self.act if hid else "none", z_out=z, keep_prob=keep if hid else 1.0, seed=seed,
                   offset=off, step=step)
            cache.z.append(z)
            cache.h.append(out)
            cache.offsets.append(off)
            h = out
        return h, cache

    # ------------------------------------------------------------------ backward
    def backward(self, P: FlatParams, cache: LayerCache, dout: torch.Tensor, *, dout_is_dz: bool = True,
                 need_dx: bool = False, on_ready=None, wgrad=None, opt=None) -> Optional[torch.Tensor]:
        """Accumulate param grads into ``P.grad``; return dx if ``need_dx``.
        ``opt`` (the in-epilogue AdamW of the transformer stages) is not supported here
        and must be None (the stage trainer only builds it for models that list
        ``gemm_weight_names``).

        ``dout`` is the gradient w.r.t. the stack output.  With ``dout_is_dz``
        (the CE kernel already wrote dz and the top bias grad) it is used as the
        top layer's dz directly; otherwise the top layer's act/dropout backward
        and bias grad are applied first (pipeline stage boundary)."""
        assert opt is None, "MLP.backward has no in-epilogue optimizer"
        L = self.L
        top = self.names[L - 1]
        if dout_is_dz:
            dz = dout
        else:
            dz = K.act_bwd(dout, cache.z[L - 1], self.act, keep_prob=cache.keep if self._hidden(L - 1) else 1.0,
                           seed=cache.seed, offset=cache.offsets[L - 1], step=cache.step,
                           dbias=P.g(f"{top}/bias"))
        dx = None
        for i in range(L - 1, -1, -1):
            n = self.names[i]
            h_prev = cache.x if i == 0 else cache.h[i - 1]
            # dW_i += h_prev^T . dz ([in, out], fp32 accumulate) and the input gradient
            # only need dz: one grouped launch on GPU (ops.kernels.gemm_group)
            with K.gemm_group():
                K.dw_gemm(wgrad if on_ready is None else None, h_prev, dz, P.g(f"{n}/kernel"))
                if i > 0:
                    pn = self.names[i - 1]
                    dz_prev = torch.empty(dz.shape[0], self.dims[i], dtype=torch.bfloat16, device=dz.device)
                    K.gemm(dz, P.s(f"{n}/kernel"), a_layout="mk", b_layout="nk", out=dz_prev,
                           z_in=cache.z[i - 1], act_bwd=self.act, keep_prob=cache.keep, seed=cache.seed,
                           offset=cache.offsets[i - 1], step=cache.step, dbias=P.g(f"{pn}/bias"))
                elif need_dx:
                    dx = torch.empty(dz.shape[0], self.dims[0], dtype=torch.bfloat16, device=dz.device)
                    K.gemm(dz, P.s(f"{n}/kernel"), a_layout="mk", b_layout="nk", out=dx)
            if on_ready is not None:  # layer i's kernel and bias grads are final (its bias came with dz)
                on_ready([f"{n}/kernel", f"{n}/bias"])
            if i > 0:
                dz = dz_prev
        return dx


class Classifier(MLP):
    """The reference ``Classifier`` (data_paral.py:75-102): 784 -> hidden -> classes.

    ``num_layers`` counts Dense layers: 2 is the reference model, 4 is BASELINE
    config #2's 4-layer MLP."""

    def __init__(self, input_size: int = 784, hidden_size: int = 512, num_classes: int = 10,
                 dropout_rate: float = 0.1, num_layers: int = 2, act: str = "silu"):
        dims = [input_size] + [hidden_size] * (num_layers - 1) + [num_classes]
        super().__init__(dims, act=act, dropout_rate=dropout_rate)

    @classmethod
    def from_config(cls, cfg) -> "Classifier":
        return cls(input_size=cfg.get("input_size", 784), hidden_size=cfg.hidden_size,
                   num_classes=cfg.num_classes, dropout_rate=cfg.dropout_rate,
                   num_layers=cfg.get("num_layers", 2), act=cfg.get("act", "silu"))


def loss_and_grad(model, P: FlatParams, x: torch.Tensor, labels: torch.Tensor, *, train: bool, seed: int,
                  offset: int, step: Optional[torch.Tensor], grad_scale: Optional[float] = None,
                  metrics: Optional[torch.Tensor] = None, on_ready=None):
    """One minibatch: forward, fused CE(+metrics, +head bias grad), explicit backward
    into P.grad (beta=1).  ``grad_scale`` defaults to 1/#labels (mean loss).
    Works for any model exposing forward/backward/flatten_labels/head_bias_name."""
    logits, cache = model.forward(P, x, train=train, seed=seed, offset=offset, step=step)
    y = model.flatten_labels(labels)
    if grad_scale is None:
        grad_scale = 1.0 / y.numel()
    dlogits = torch.empty_like(logits)
    hb = model.head_bias_name
    K.softmax_xent(logits, y, grad_scale=grad_scale, dlogits=dlogits, dbias=P.g(hb) if hb else None,
                   metrics=metrics)
    if on_ready is not None:
        model.backward(P, cache, dlogits, on_ready=on_ready)
    else:
        model.backward(P, cache, dlogits)
    return logits
