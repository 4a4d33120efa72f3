"""Training core: TrainState, Batch, optimizers, gradient accumulation
(reference util.py:21-167).

* ``TrainState`` (util.py:21-22): step, apply_fn, params, tx, opt_state, rng.
  Params are a :class:`FlatParams`; ``apply_gradients`` is ONE fused optimizer
  kernel over the flat buffer that also writes the bf16 compute shadow and
  zeroes the grad buffer.  Updates are in place (the analogue of
  ``donate_argnames=("state",)``), and the device-side step counter makes the
  update replayable from a hipGraph.
* ``accum_grads_loop`` / ``accum_grads_scan`` (util.py:41-137): minibatch
  gradient accumulation.  Gradients accumulate IN PLACE into the fp32 grad
  buffer through beta=1 GEMM epilogues, so "sum the grads" costs nothing; the
  final ``/ n_minbatch`` (util.py:77) is folded into the optimizer's grad scale
  (returned as ``GradBuffer.scale``).  The "scan" variant replays one captured
  minibatch step (a hipGraph on GPU) with a device-resident minibatch index.
"""
from __future__ import annotations

import inspect
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Optional, Tuple, Union

import torch

from ..ops import kernels as K
from .flat import FlatParams
from .metrics import Metrics
from . import rng as R

Pytree = Any
# pipeline_parallel.py:24-26 of the reference: a parameter leaf is a plain array or
# an axis-annotated shard (flax ``nn.Partitioned`` -> parallel.fsdp.Partitioned)
Parameter = Union[torch.Tensor, "Partitioned"]  # noqa: F821 (forward ref, parallel/fsdp.py)


# ---------------------------------------------------------------------------- batch
@dataclass
class Batch:
    """util.py:25-28.  ``inputs`` [B, ...], ``labels`` [B] int32."""

    inputs: torch.Tensor
    labels: torch.Tensor

    def slice(self, start: int, size: int) -> "Batch":
        return Batch(self.inputs[start: start + size], self.labels[start: start + size])

    def map(self, fn: Callable[[torch.Tensor], torch.Tensor]) -> "Batch":
        return Batch(fn(self.inputs), fn(self.labels))

    @property
    def size(self) -> int:
        return int(self.inputs.shape[0])

    def same_storage(self, other: "Batch") -> bool:
        return (self.inputs.data_ptr() == other.inputs.data_ptr() and self.labels.data_ptr() == other.labels.data_ptr()
                and self.inputs.shape == other.inputs.shape and self.labels.shape == other.labels.shape)


def check_static_batch(static: Optional[Batch], batch: Batch) -> None:
    """A captured hipGraph reads the batch tensors it was captured with: a step on
    other tensors would silently train on the captured data.  New data goes into the
    captured tensors through the trainer's ``set_batch`` (which also drops a run-ahead
    forward computed from the old contents)."""
    if static is not None and batch is not static and not batch.same_storage(static):
        raise ValueError("this trainer replays hipGraphs captured on another batch: copy the new data in with "
                         "trainer.set_batch(batch) (or call trainer.invalidate() and capture again)")


def load_static_batch(static: Batch, batch: Batch, engines=()) -> None:
    """Copy ``batch`` into the captured batch tensors; engines whose run-ahead launch
    already computed the next forward from the old contents restart cold."""
    if batch is static or batch.same_storage(static):
        pass
    else:
        if batch.inputs.shape != static.inputs.shape or batch.labels.shape != static.labels.shape:
            raise ValueError(f"set_batch: shapes {tuple(batch.inputs.shape)} / {tuple(batch.labels.shape)} differ "
                             f"from the captured {tuple(static.inputs.shape)} / {tuple(static.labels.shape)}")
        static.inputs.copy_(batch.inputs)
        static.labels.copy_(batch.labels)
    for e in engines:
        if e is not None and hasattr(e, "ahead_primed"):
            e.ahead_primed = False


# ---------------------------------------------------------------------------- optimizers
@dataclass
class AdamW:
    """optax.adamw defaults (b1 .9, b2 .999, eps 1e-8, weight_decay 1e-4, no mask)."""

    learning_rate: float = 1e-3
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    weight_decay: float = 1e-4

    def init(self, params: FlatParams) -> Dict[str, torch.Tensor]:
        dev = params.master.device
        return {"m": torch.zeros(params.numel, device=dev), "v": torch.zeros(params.numel, device=dev),
                "count": torch.zeros(1, dtype=torch.int32, device=dev),
                "ticket": torch.zeros(1, dtype=torch.int32, device=dev)}

    def update(self, params: FlatParams, opt_state, grad_scale: float, zero_grad: bool = True):
        K.adamw_step(params.master[: params.numel], params.grad[: params.numel], opt_state["m"], opt_state["v"],
                     params.shadow[: params.numel] if params.shadow is not None else None, lr=self.learning_rate,
                     b1=self.b1, b2=self.b2, eps=self.eps, wd=self.weight_decay, grad_scale=grad_scale,
                     step=opt_state["count"], ticket=opt_state["ticket"], zero_grad=zero_grad)


@dataclass
class SGD:
    learning_rate: float = 1e-2
    momentum: float = 0.0
    weight_decay: float = 0.0

    def init(self, params: FlatParams) -> Dict[str, torch.Tensor]:
        dev = params.master.device
        st = {"count": torch.zeros(1, dtype=torch.int32, device=dev),
              "ticket": torch.zeros(1, dtype=torch.int32, device=dev)}
        if self.momentum:
            st["buf"] = torch.zeros(params.numel, device=dev)
        return st

    def update(self, params: FlatParams, opt_state, grad_scale: float, zero_grad: bool = True):
        K.sgd_step(params.master[: params.numel], params.grad[: params.numel], opt_state.get("buf"),
                   params.shadow[: params.numel] if params.shadow is not None else None, lr=self.learning_rate,
                   momentum=self.momentum, wd=self.weight_decay, grad_scale=grad_scale, step=opt_state["count"],
                   ticket=opt_state["ticket"], zero_grad=zero_grad)


def adamw(learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
          weight_decay: float = 1e-4) -> AdamW:
    return AdamW(learning_rate, b1, b2, eps, weight_decay)


def sgd(learning_rate: float, momentum: float = 0.0, weight_decay: float = 0.0) -> SGD:
    return SGD(learning_rate, momentum, weight_decay)


# ---------------------------------------------------------------------------- grads handle
@dataclass
class GradBuffer:
    """Accumulated gradients living in ``params.grad``; the true gradient is
    ``flat * scale`` (the mean over minibatches/devices is applied lazily, fused
    into the optimizer kernel)."""

    params: FlatParams
    scale: float = 1.0

    @property
    def flat(self) -> torch.Tensor:
        return self.params.grad_params

    def materialize(self) -> Dict[str, torch.Tensor]:
        return {n: self.params.g(n) * self.scale for n in self.params.names()}


# ---------------------------------------------------------------------------- train state
@dataclass
class TrainState:
    step: int
    apply_fn: Any
    params: FlatParams
    tx: Any
    opt_state: Dict[str, torch.Tensor]
    rng: int = 0
    extra: Dict[str, Any] = field(default_factory=dict)

    @classmethod
    def create(cls, *, apply_fn, params: FlatParams, tx, rng: int = 0) -> "TrainState":
        return cls(step=0, apply_fn=apply_fn, params=params, tx=tx, opt_state=tx.init(params), rng=rng)

    @property
    def step_tensor(self) -> torch.Tensor:
        """Device step counter (advanced inside the optimizer kernel)."""
        return self.opt_state["count"]

    def apply_gradients(self, *, grads: Optional[GradBuffer] = None, rng: Optional[int] = None,
                        grad_scale: Optional[float] = None) -> "TrainState":
        scale = grad_scale if grad_scale is not None else (grads.scale if grads is not None else 1.0)
        self.tx.update(self.params, self.opt_state, scale)
        self.step += 1
        if rng is not None:
            self.rng = rng
        return self


def get_num_params(state) -> int:
    """util.py:184-185 -- global (unsharded) parameter count."""
    if isinstance(state, TrainState):
        p = state.params
    else:
        p = state
    if hasattr(p, "global_num_params"):
        return p.global_num_params()
    return p.num_params()


# ---------------------------------------------------------------------------- accumulation
LossFn = Callable[..., Tuple[torch.Tensor, Metrics]]


def _metrics_add(a, b):
    if a is None:
        return {k: tuple(x for x in v) for k, v in b.items()}
    return {k: tuple(x + y for x, y in zip(a[k], b[k])) for k in a}


def _detach_metrics(m):
    return {k: tuple(x.detach() if torch.is_tensor(x) else x for x in v) for k, v in m.items()}


def is_reference_loss_fn(loss_fn: Callable) -> bool:
    """True for a reference-contract ``loss_fn(params, apply_fn, batch, rng) ->
    (mean_loss, metrics)`` whose gradient must come from autograd (data_paral.py:
    171-189); False for the engine contract, which also accepts
    ``minibatch_index=`` / ``state=`` keywords and writes its own gradient into
    ``params.grad`` (beta = 1 GEMM epilogues)."""
    try:
        sig = inspect.signature(loss_fn)
    except (TypeError, ValueError):
        return True
    ps = sig.parameters
    return not ("minibatch_index" in ps or "state" in ps
                or any(p.kind == inspect.Parameter.VAR_KEYWORD for p in ps.values()))


def param_tree(params: FlatParams, requires_grad: bool = True) -> Tuple[Dict[str, Any], Dict[str, torch.Tensor]]:
    """The flax-style nested pytree ``{layer: {"kernel": W, "bias": b}}`` over the
    fp32 master views (leaves share storage with ``params.master``), and the flat
    ``{path: leaf}`` map autograd differentiates."""
    leaves = {n: params.p(n).detach().requires_grad_(requires_grad) for n in params.names()}
    tree: Dict[str, Any] = {}
    for path, t in leaves.items():
        node = tree
        parts = path.split("/")
        for part in parts[:-1]:
            node = node.setdefault(part, {})
        node[parts[-1]] = t
    return tree, leaves


def value_and_grad_into(loss_fn: LossFn, state: "TrainState", batch: Batch, rng: int):
    """``jax.value_and_grad(loss_fn, has_aux=True)`` (util.py:53,65) for a
    reference-contract loss: differentiate w.r.t. the parameter pytree with torch
    autograd and ACCUMULATE the gradient into ``params.grad`` (the grads "+" of
    util.py:74).  Returns (mean loss, metrics), detached."""
    P = state.params
    tree, leaves = param_tree(P)
    loss, metrics = loss_fn(tree, state.apply_fn, batch, rng)
    names = [n for n, t in leaves.items()]
    grads = torch.autograd.grad(loss, [leaves[n] for n in names], allow_unused=True)
    for n, g in zip(names, grads):
        if g is not None:
            P.g(n).add_(g.to(P.grad.dtype))
    return loss.detach(), _detach_metrics(metrics)


def accum_grads_loop(batch: Batch, state: TrainState, key: int, n_minbatch: int,
                     loss_fn: LossFn) -> Tuple[GradBuffer, Metrics]:
    """util.py:41-78.  Two ``loss_fn`` contracts (:func:`is_reference_loss_fn`):

    * reference: ``loss_fn(params_pytree, apply_fn, minibatch, rng) -> (mean_loss,
      metrics)`` built from differentiable torch ops / ``state.apply_fn`` -- its
      gradient is taken with autograd and accumulated into ``params.grad``;
    * engine (fast path): ``loss_fn(params, apply_fn, minibatch, rng,
      minibatch_index=i, state=state)`` accumulates its own gradient into
      ``params.grad`` (beta = 1 kernels).
    Either way the returned :class:`GradBuffer` is the SUM with ``scale`` =
    1/n_minbatch (the mean of util.py:77, applied lazily by the optimizer)."""
    bs = batch.size
    mb = bs // n_minbatch
    keys = R.split(key, n_minbatch)
    metrics = None
    ref = is_reference_loss_fn(loss_fn)
    for i in range(n_minbatch):
        minibatch = batch.slice(i * mb, mb)
        if ref:
            _, m = value_and_grad_into(loss_fn, state, minibatch, keys[i])
        else:
            _, m = loss_fn(state.params, state.apply_fn, minibatch, keys[i], minibatch_index=i, state=state)
        metrics = _metrics_add(metrics, m)
    return GradBuffer(state.params, 1.0 / n_minbatch), metrics


def accum_grads_scan(batch: Batch, state: TrainState, key: int, n_minbatch: int,
                     loss_fn: LossFn) -> Tuple[GradBuffer, Metrics]:
    """util.py:81-137.  Rolled loop: ONE minibatch step, captured once as a hipGraph
    that reads its minibatch from device-resident input slots, replayed
    ``n_minbatch`` times on GPU (eagerly, one minibatch at a time, on CPU).

    * engine contract: the captured call gets ``rng = key`` and ``minibatch_index`` =
      a device int32 tensor holding ``i`` during replay ``i`` (a captured Python int
      could not change between replays), so the loss draws per-minibatch randomness
      by folding that device index in -- as the DP trainer's ``accum="scan"`` mode
      does (parallel/dp.py), where scan == loop bit for bit;
    * reference contract (autograd ``loss_fn(params, apply_fn, batch, rng)``): the
      forward AND its autograd backward are captured; ``rng`` is a
      :class:`~jax_distributed_tuts_amd.utils.rng.ScanKey` holding every minibatch's
      split key with the device index selecting one -- the reference's
      ``keys[batch_idx]`` (util.py:107-108) -- so models' dropout draws the loop's
      masks exactly (tests/test_reference_loss_fn.py).  A loss whose ops cannot be
      captured runs the same body eagerly, with a warning.

    The captured minibatch program is cached (like ``jax.jit``'s trace cache) under
    (loss_fn, parameter / gradient buffers, minibatch shape and dtypes, n_minbatch):
    the next call only loads its minibatches into the slots and replays.  A
    reference-contract call refreshes the device copy of its split keys in place, so
    a training loop whose rng changes every step captures once; an engine-contract
    loss receives ``key`` as a host int, which a graph bakes in, so the key is part
    of its cache entry."""
    bs = batch.size
    mb = bs // n_minbatch
    dev = batch.inputs.device
    ref = is_reference_loss_fn(loss_fn)
    if ref:
        return _accum_scan_reference(batch, state, key, n_minbatch, loss_fn)
    if dev.type != "cuda":
        return accum_grads_loop(batch, state, key, n_minbatch, loss_fn)
    ck = _scan_key("engine", batch, state, n_minbatch, loss_fn) + (int(key),)
    ent = _SCAN_CACHE.get(ck)
    metrics = None
    if ent is None:
        # device-resident slot the captured step reads its minibatch from
        xin = torch.empty((mb,) + tuple(batch.inputs.shape[1:]), dtype=batch.inputs.dtype, device=dev)
        yin = torch.empty((mb,), dtype=batch.labels.dtype, device=dev)
        mslot = {}
        idx = torch.zeros(1, dtype=torch.int32, device=dev)

        def _body():
            _, m = loss_fn(state.params, state.apply_fn, Batch(xin, yin), key, minibatch_index=idx, state=state)
            mslot["m"] = m

        # warm up on minibatch 0 eagerly (allocations, library load), then capture the body once
        _scan_load(batch, xin, yin, idx, 0, mb)
        _body()
        metrics = _metrics_add(metrics, _clone_metrics(mslot["m"]))
        g = None
        if n_minbatch > 1:
            _scan_load(batch, xin, yin, idx, 1, mb)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                _body()
            SCAN_STATS["captures"] += 1
        ent = _SCAN_CACHE.put(ck, {"graph": g, "xin": xin, "yin": yin, "idx": idx, "out": mslot, "body": _body})
        first = 1
    else:
        first = 0
    for i in range(first, n_minbatch):
        _scan_load(batch, ent["xin"], ent["yin"], ent["idx"], i, mb)
        if ent["graph"] is None:
            ent["body"]()   # one minibatch: nothing was captured, the body runs eagerly
        else:
            ent["graph"].replay()
        metrics = _metrics_add(metrics, _clone_metrics(ent["out"]["m"]))
    return GradBuffer(state.params, 1.0 / n_minbatch), metrics


def _clone_metrics(m: Metrics) -> Metrics:
    return {k: tuple(x.clone() if torch.is_tensor(x) else x for x in v) for k, v in m.items()}


class _LRU:
    """A small least-recently-used map (captured scan programs hold graph memory)."""

    def __init__(self, cap: int = 8):
        from collections import OrderedDict

        self.cap, self.d = cap, OrderedDict()

    def get(self, k):
        v = self.d.get(k)
        if v is not None:
            self.d.move_to_end(k)
        return v

    def put(self, k, v):
        self.d[k] = v
        self.d.move_to_end(k)
        while len(self.d) > self.cap:
            self.d.popitem(last=False)
        return v

    def clear(self):
        self.d.clear()


_SCAN_CACHE = _LRU()
# captures of a rolled minibatch program since import (tests assert a training loop captures once)
SCAN_STATS = {"captures": 0}


def _scan_key(kind: str, batch: Batch, state: "TrainState", n_minbatch: int, loss_fn) -> tuple:
    P = state.params
    return (kind, loss_fn, id(P), P.master.data_ptr(), P.grad.data_ptr(), id(state.apply_fn), n_minbatch,
            batch.size // n_minbatch, tuple(batch.inputs.shape[1:]), batch.inputs.dtype, batch.labels.dtype,
            str(batch.inputs.device))


def _scan_load(batch: Batch, xin, yin, idx, i: int, mb: int):
    xin.copy_(batch.inputs[i * mb:(i + 1) * mb])
    yin.copy_(batch.labels[i * mb:(i + 1) * mb])
    idx.fill_(i)


# (grads buffer, capture outcome) of the most recent reference-contract scan, for tests / logs
LAST_SCAN_MODE = {"mode": None}


def _accum_scan_reference(batch: Batch, state: TrainState, key: int, n_minbatch: int,
                          loss_fn: LossFn) -> Tuple[GradBuffer, Metrics]:
    """The reference-contract scan (see :func:`accum_grads_scan`)."""
    bs = batch.size
    mb = bs // n_minbatch
    dev = batch.inputs.device
    keys = R.split(key, n_minbatch)
    ck = _scan_key("reference", batch, state, n_minbatch, loss_fn)
    ent = _SCAN_CACHE.get(ck) if (dev.type == "cuda" and n_minbatch > 1) else None
    metrics = None
    if ent is not None:
        # cached program: this call's split keys into the device key table it reads
        ent["skey"].dev.copy_(torch.tensor([R._s64(k) for k in keys], dtype=torch.int64))
        LAST_SCAN_MODE["mode"] = "graph"
        for i in range(n_minbatch):
            _scan_load(batch, ent["xin"], ent["yin"], ent["idx"], i, mb)
            ent["graph"].replay()
            metrics = _metrics_add(metrics, _clone_metrics(ent["out"]["m"]))
        return GradBuffer(state.params, 1.0 / n_minbatch), metrics
    xin = torch.empty((mb,) + tuple(batch.inputs.shape[1:]), dtype=batch.inputs.dtype, device=dev)
    yin = torch.empty((mb,), dtype=batch.labels.dtype, device=dev)
    idx = torch.zeros(1, dtype=torch.int32, device=dev)
    skey = R.ScanKey.from_keys(keys, idx)
    out = {}

    def _body():
        out["m"] = value_and_grad_into(loss_fn, state, Batch(xin, yin), skey)[1]

    _scan_load(batch, xin, yin, idx, 0, mb)
    _body()   # minibatch 0 eagerly: warm-up (allocations, autograd graph, kernel library)
    metrics = _metrics_add(metrics, _clone_metrics(out["m"]))
    if n_minbatch == 1:
        LAST_SCAN_MODE["mode"] = "eager"
        return GradBuffer(state.params, 1.0), metrics
    graph = None
    if dev.type == "cuda":
        _scan_load(batch, xin, yin, idx, 1, mb)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                _body()
            graph = g
            SCAN_STATS["captures"] += 1
            _SCAN_CACHE.put(ck, {"graph": g, "xin": xin, "yin": yin, "idx": idx, "skey": skey, "out": out})
        except Exception as e:   # an op of the user's loss that cannot be captured
            import logging

            logging.getLogger("jdt.util").warning("accum_grads_scan: loss_fn not capturable (%s); "
                                                  "running the rolled step eagerly", e)
            torch.cuda.synchronize()
    LAST_SCAN_MODE["mode"] = "graph" if graph is not None else "eager"
    for i in range(1, n_minbatch):
        _scan_load(batch, xin, yin, idx, i, mb)
        if graph is not None:
            graph.replay()
        else:
            _body()
        metrics = _metrics_add(metrics, _clone_metrics(out["m"]))
    return GradBuffer(state.params, 1.0 / n_minbatch), metrics


def accum_grads(state: TrainState, batch: Batch, key: int, num_minibatches: int, loss_fn: LossFn,
                use_scan: bool = False) -> Tuple[GradBuffer, Metrics]:
    """util.py:140-167 (same signature and argument order)."""
    if use_scan:
        return accum_grads_scan(batch=batch, state=state, key=key, n_minbatch=num_minibatches, loss_fn=loss_fn)
    return accum_grads_loop(batch=batch, state=state, key=key, n_minbatch=num_minibatches, loss_fn=loss_fn)
