"""GPipe pipeline parallelism and hybrid DP x PP.

The reference's pipeline_parallel.py:1-39 is an imports-only stub; its imports
(``fold_rng_over_axis`` from the DP tutorial, the multi-axis ``sync_gradients``
from the FSDP tutorial, ``Parameter = Array | nn.Partitioned``) and BASELINE
configs #4/#5 define the intended behaviour (SURVEY §3.5 [inferred]):

  mesh (data=N_dp, pipe=S); batch split over 'data', then into n_mb microbatches
  GPipe fill/drain: at tick t stage s runs microbatch t-s; activations move
  s -> s+1 (ppermute), activation grads s+1 -> s in the reverse schedule
  loss + metrics on the last stage only
  sync_gradients(grads, ('data','pipe')): stage params are sharded on 'pipe'
  -> mean over 'data' only
  AdamW on the local stage params

MI355X mapping: one process per GPU, stage s = pipe coordinate; activation
hand-off is RCCL send/recv on the 'pipe' sub-group (every pair of GPUs on an
MI355X node is one xGMI hop, so stage adjacency needs no placement care).
Each stage runs the explicit-backward MLP/transformer kernels; grads of all
microbatches accumulate in place (beta = 1); the 'data' all-reduce is ONE
bucket (grads + metric slots) per stage; the optimizer is the same fused AdamW.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from ..comm import collectives as C
from ..models.mlp import MLP
from ..ops import kernels as K
from ..runtime.dist import Mesh, is_initialized
from ..utils import rng as R
from ..utils.flat import FlatParams, N_METRIC_SLOTS
from ..utils.profiling import named_scope
from ..utils.train_state import Batch, TrainState


def split_layers(n_layers: int, n_stages: int) -> List[range]:
    """Contiguous, as-even-as-possible assignment of layers to stages."""
    if n_stages > n_layers:
        raise ValueError(f"{n_stages} stages for {n_layers} layers")
    return [range(s * n_layers // n_stages, (s + 1) * n_layers // n_stages) for s in range(n_stages)]


def mlp_stage(dims: Sequence[int], n_stages: int, stage: int, act: str = "silu", dropout_rate: float = 0.1,
              names: Optional[Sequence[str]] = None) -> MLP:
    """Stage ``stage`` of MLP(dims): its Dense layers keep their global names and
    dropout-stream ids, so any split trains the same model."""
    L = len(dims) - 1
    full = MLP(dims, act=act, dropout_rate=dropout_rate, names=names)
    r = split_layers(L, n_stages)[stage]
    last = stage == n_stages - 1
    m = MLP(list(dims[r.start: r.stop + 1]), act=act, dropout_rate=dropout_rate,
            names=full.names[r.start: r.stop], final_act=not last, layer_id_base=r.start)
    return m


def init_stage_params(stage_model, full_specs, seed: int, device) -> FlatParams:
    """Initialise exactly the values the un-split model would get (the init stream
    runs over every global param in order; a stage keeps its own)."""
    P = FlatParams(stage_model.param_specs(), device=device)
    full = FlatParams(full_specs, device="cpu", with_grad=False, with_shadow=False, metric_slots=0).init_(seed)
    for n in P.names():
        P.p(n).copy_(full.p(n))
    P.sync_shadow()
    return P


@dataclass
class PipeConfig:
    num_microbatches: int = 4
    data_axis: str = "data"
    pipe_axis: str = "pipe"


class GPipeTrainer:
    """Runs one stage of a GPipe schedule (``stage.forward/backward`` explicit API)."""

    def __init__(self, state: TrainState, mesh: Optional[Mesh], cfg: PipeConfig, act_dtype=torch.bfloat16):
        self.state, self.mesh, self.cfg = state, mesh, cfg
        self.model = state.apply_fn
        self.S = C.axis_size(mesh, cfg.pipe_axis)
        self.s = C.axis_index(mesh, cfg.pipe_axis)
        self.n_dp = C.axis_size(mesh, cfg.data_axis)
        self.first, self.last = self.s == 0, self.s == self.S - 1
        self.act_dtype = act_dtype
        dev = state.params.master.device
        self.metrics = torch.zeros(N_METRIC_SLOTS, dtype=torch.float32, device=dev)

    # ------------------------------------------------------------------ p2p
    def _send(self, x: torch.Tensor, to: int):
        with named_scope("pipe_send"):
            C.send(x, self.mesh, self.cfg.pipe_axis, to)

    def _recv(self, shape, to_dtype, frm: int) -> torch.Tensor:
        with named_scope("pipe_recv"):
            buf = torch.empty(shape, dtype=to_dtype, device=self.state.params.master.device)
            return C.recv(buf, self.mesh, self.cfg.pipe_axis, frm)

    # ------------------------------------------------------------------ step
    def step(self, batch: Batch):
        st, P, cfg = self.state, self.state.params, self.cfg
        n_mb = cfg.num_microbatches
        mb = batch.size // n_mb
        rng = R.fold_rng_over_axis(st.rng, self.mesh, cfg.data_axis)
        seed = rng & 0xFFFFFFFF
        caches, dlogits = [None] * n_mb, [None] * n_mb
        # ---- forward fill/drain: tick t, stage s handles microbatch t - s
        for t in range(n_mb + self.S - 1):
            i = t - self.s
            if not (0 <= i < n_mb):
                continue
            if self.first:
                x = batch.inputs[i * mb:(i + 1) * mb]
            else:
                x = self._recv(self.model.input_shape(mb), self.act_dtype, self.s - 1)
            out, cache = self.model.forward(P, x, train=True, seed=seed, offset=i << 16, step=st.step_tensor)
            caches[i] = cache
            if self.last:
                d = torch.empty_like(out)
                self.loss_head(out, batch.labels[i * mb:(i + 1) * mb], d)
                dlogits[i] = d
            else:
                self._send(out, self.s + 1)
        # ---- backward, reverse microbatch order
        for i in reversed(range(n_mb)):
            if self.last:
                dx = self.model.backward(P, caches[i], dlogits[i], dout_is_dz=True, need_dx=not self.first)
            else:
                dh = self._recv(self.model.output_shape(mb), self.act_dtype, self.s + 1)
                dx = self.model.backward(P, caches[i], dh, dout_is_dz=False, need_dx=not self.first)
            if not self.first:
                self._send(dx, self.s - 1)
            caches[i] = None
        # ---- sync_gradients(('data','pipe')): stage params are pipe-sharded -> data only
        with named_scope("sync_grads"):
            C.psum_(P.grad, self.mesh, cfg.data_axis)
        st.apply_gradients(grad_scale=1.0 / (n_mb * self.n_dp))
        with named_scope("sync_metrics"):
            K.metrics_fold_(self.metrics, P.metrics_slot)

    def loss_head(self, logits, labels, dlogits):
        y = self.model.flatten_labels(labels)
        hb = self.model.head_bias_name
        K.softmax_xent(logits, y, grad_scale=1.0 / y.numel(), dlogits=dlogits,
                       dbias=self.state.params.g(hb) if hb else None, metrics=self.state.params.metrics_slot)

    def gather_metrics(self) -> torch.Tensor:
        """Metrics live on the last stage; bring them to every pipe member."""
        m = self.metrics.clone()
        if self.mesh is not None and self.S > 1 and is_initialized():
            if not self.last:
                m.zero_()
            C.psum_(m, self.mesh, self.cfg.pipe_axis)
        return m
