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

import math
import contextlib
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from ..comm import collectives as C
from ..models.mlp import MLP
from ..ops import kernels as K
from ..runtime.dist import Mesh, is_initialized
from ..utils import rng as R
from ..utils.flat import FlatParams, N_METRIC_SLOTS
from ..utils.profiling import named_scope, replay_scope
from ..utils.train_state import AdamW, Batch, TrainState, check_static_batch, load_static_batch


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


def default_microbatches(n_stages: int) -> int:
    """GPipe microbatch count when the caller does not pick one.

    Measured, not the textbook 2S-or-more (profiles/r3_pp_schedule.json,
    tools/pp_schedule.py: per-stage fwd / bwd tick cost on one MI355X at n = 1..16
    microbatches): the stage kernels are latency-bound, so a tick costs nearly the
    same at 8 rows as at 64 (8-stage MLP backward tick 12.9 us at 64 rows, 12.5 at 16,
    15.3 at 8) and every extra microbatch adds a whole tick.  Modeled step time
    (n + S - 1) * (t_f + t_b), hand-off hops excluded: 8-stage MLP 204 / 183 / 203 /
    268 / 468 us at n = 1 / 2 / 4 / 8 / 16; 4-stage LM (8 sequences per pipe) 1023 /
    1055 / 1196 / 1616 us at n = 1 / 2 / 4 / 8.  n = 2 is the MLP's best and within 3 %
    of the LM's (n = 1 is no pipelining at all); per-tick xGMI hops only widen the gap
    to larger n.  A single stage keeps the tutorial's 4 minibatches (its merged /
    layer-major pass makes the count a loss-weighting detail)."""
    return 4 if n_stages <= 1 else 2


@dataclass
class PipeConfig:
    num_microbatches: int = 4
    data_axis: str = "data"
    pipe_axis: str = "pipe"
    comm: str = "auto"   # "auto" | "xgmi" | "rccl": stage hand-off + data-axis all-reduce
    # weight-gradient GEMMs on a side stream (GPU), joined before the sync.  Off by
    # default: measured slower in the captured step (transformer 3.07 -> 3.78 ms,
    # 8-layer MLP 0.79 -> 1.05 ms on one MI355X -- the fork/join graph edges cost
    # more than the overlap gains at these kernel sizes)
    overlap_wgrad: bool = field(default_factory=lambda: os.environ.get("JDT_OVERLAP_WGRAD") == "1")
    # single stage (pipe axis of size 1): GPipe has no neighbour to feed, so the
    # microbatches may run as ONE pass over all local rows (each row keeps its
    # microbatch's 1/mb loss weight: the same gradient as the microbatch loop, the
    # dropout masks drawn over the merged rows).  Ignored when the pipe axis > 1.
    merge_single_stage: bool = False
    # GPU, MLP stages of the tutorial shapes: one fused md_fwd / md_bwd launch per
    # layer and microbatch (parallel/fused_stage.py) instead of the generic chain
    fused_stage: bool = True
    # pipe axis of size 1: run the microbatches layer-major, one pass per layer over all
    # local rows, whenever that draws exactly the microbatch loop's dropout masks --
    # the fused MLP kernels keep per-microbatch streams (_single_stage_engine); a model
    # without dropout (the transformer LM) has no masks to keep, so its merged pass IS
    # the loop's gradient (each row keeps its microbatch's 1/mb loss weight).  False:
    # per-microbatch passes, as on a real multi-stage pipeline.  A model whose
    # per-microbatch passes run on concurrent streams (mb_streams > 1, below) takes
    # those instead: the LM step measured 1.07 vs 1.17 ms layer-major on one MI355X
    # (profiles/r3_lm_mb_streams_ab.txt).
    layer_major_single_stage: bool = True
    # one GPU, one stage, AdamW: apply the optimizer layer by layer on a side stream
    # as the backward finishes each layer's gradients (ops.kernels.OverlappedAdamW).
    # Opt-in (env JDT_OVERLAP_OPT=1): measured SLOWER on the transformer step (1.39 vs
    # 1.18 ms, profiles/r2_overlapped_adamw_ab.txt) -- the forked AdamW grids contend
    # with the backward GEMMs for CUs instead of filling idle ones
    overlap_optimizer: bool = True
    # per-microbatch passes of a model with deferrable weight gradients (the transformer
    # LM): each microbatch's backward runs only the input-gradient chain and the
    # weight-gradient GEMMs run ONCE per step over all microbatches' rows (the "W pass"
    # of zero-bubble schedules, Qi et al. 2023) -- 4x the K per GEMM, 1/n_mb the
    # launches, and the gradient an upstream stage waits for is sent sooner.
    # JDT_DEFER_WGRAD=0 turns it off (A/B).
    defer_wgrad: bool = field(default_factory=lambda: os.environ.get("JDT_DEFER_WGRAD", "1") != "0")
    # one stage, per-microbatch passes with deferred weight gradients (GPU): microbatch i
    # runs its forward and input-gradient chain on stream i % mb_streams.  With the
    # weight gradients deferred the chains share no buffer (every cross-microbatch
    # accumulation -- bias / LayerNorm / embedding grads, metrics -- is an fp32 atomic,
    # split-K slabs are per stream), and a 512-row microbatch GEMM fills half the CUs.
    # 0 (default) = auto: 4, except a one-stage model whose layer-major pass takes the
    # one-launch W pass (below) -- the LM step measured 0.91 ms that way against 1.01 on
    # 4 microbatch streams (profiles/r6_s5_lm.txt)
    mb_streams: int = field(default_factory=lambda: int(os.environ.get("JDT_MB_STREAMS", "0")))
    # one stage, layer-major (one pass over all rows), GPU: weight gradients deferred and
    # issued per part on this many streams, overlapping the input-gradient chain
    # (GPipeTrainer._layer_major_wpass); 1 = the weight GEMMs inline in the backward.
    # Opt-in: measured SLOWER (1.21-1.28 vs 1.17 ms: the side-stream GEMMs take CUs from
    # the chain they were meant to hide behind)
    wpass_streams: int = field(default_factory=lambda: int(os.environ.get("JDT_LM_WSTREAMS", "1")))
    # concurrent microbatch passes: > 0 runs the W pass on this many dedicated streams,
    # each part's GEMMs as soon as every chain has passed it (0: after the join)
    wpass_early: int = field(default_factory=lambda: int(os.environ.get("JDT_WPASS_EARLY", "0")))
    # ... the W pass after the join round-robin over the first wpass_rr microbatch streams
    # (0: all of them; measured 1 stream 1.27 ms, 2: 1.12, 3-4: 1.07-1.09)
    wpass_rr: int = field(default_factory=lambda: int(os.environ.get("JDT_WPASS_STREAMS", "0")))
    # GPU: the deferred W pass (every weight-gradient GEMM of the step, AdamW in the
    # epilogues) as ONE launch (ops.kernels.gemm_wpass, csrc/gemm.hip gemm_wpass_kernel)
    # instead of one GEMM per weight round-robin over streams
    wpass_one_launch: bool = field(default_factory=lambda: os.environ.get("JDT_WPASS_ONE", "1") == "1")
    # S > 1 (xGMI inbox hand-offs): microbatch chains of a stage on concurrent streams
    # (mb_streams of them) -- opt-in, see GPipeTrainer._streams_ok
    multi_stage_streams: bool = field(default_factory=lambda: os.environ.get("JDT_PP_STREAMS", "0") == "1")
    # S > 1 with a data axis on the xGMI all-reduce + AdamW kernel: the data-axis sync is
    # issued per group (the embedding, then each weight-gradient GEMM's weight with the
    # bias / LayerNorm parameters beside it) on a comm stream as soon as the W pass has
    # produced that group's gradients, instead of one call after the whole W pass
    # (GPipeTrainer._overlapped_sync).  "auto": when every rank has a GPU of its own --
    # with ranks sharing one GPU it measured 4.4x SLOWER (profiles/r4_overlap_sync_ab.txt:
    # the comm streams' spinning collectives time-share the card's queues, as the
    # multi-stage streams above); "1" / "0" force it (JDT_PP_OVERLAP_SYNC)
    overlap_data_sync: str = field(default_factory=lambda: os.environ.get("JDT_PP_OVERLAP_SYNC", "auto"))


def _no_dropout(model) -> bool:
    """The stage model draws no dropout masks (merging microbatches changes nothing)."""
    rate = getattr(model, "dropout_rate", None)
    if rate is None:
        rate = getattr(getattr(model, "cfg", None), "dropout_rate", 1.0)
    return float(rate) == 0.0


def hw_queues() -> int:
    """HIP hardware queues per process (GPU_MAX_HW_QUEUES; HIP's default is 4), the cap
    on concurrent-stream schedules.  ``JDT_HWQ_CAP=0`` lifts the cap (diagnosis of the
    more-streams-than-queues case, tools/sessions/gpu_r4_hwq.sh)."""
    if os.environ.get("JDT_HWQ_CAP", "1") == "0":
        return 1 << 10
    try:
        return max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
    except ValueError:
        return 4


class _MbStreams:
    """``with on(i)``: run work item i on stream i % k (item 0, k, 2k, ... on the main
    stream); ``fork``: the side streams wait for the main stream's work so far;
    ``join``: the main stream waits for the side streams.  ``main=None``: one stream."""

    def __init__(self, main, side):
        self.main, self.side = main, side or []

    def fork(self):
        for s in self.side:
            s.wait_stream(self.main)

    def join(self):
        for s in self.side:
            self.main.wait_stream(s)

    def __call__(self, i: int):
        k = len(self.side) + 1
        return torch.cuda.stream(self.side[i % k - 1]) if (self.side and i % k) else contextlib.nullcontext()


class GPipeTrainer:
    """Runs one stage of a GPipe schedule (``stage.forward/backward`` explicit API).

    On GPUs of one node the stage hand-off is the xGMI inbox kernels
    (comm/p2p.py) and the data-axis gradient sync is the xGMI all-reduce with
    AdamW fused in (comm/xgmi.py), so the whole step -- every tick's compute,
    send and receive, the sync and the optimizer -- is kernels on this rank's
    stream and ``capture`` records it as one hipGraph (several steps per graph
    with ``steps_per_graph``).  Otherwise (gloo CPU simulation, ``comm="rccl"``,
    or if the xGMI mapping fails) the hand-off is RCCL/gloo send/recv, eager."""

    def __init__(self, state: TrainState, mesh: Optional[Mesh], cfg: PipeConfig, act_dtype=torch.bfloat16):
        self.state, self.mesh, self.cfg = state, mesh, cfg
        self.model = state.apply_fn
        self.S = C.axis_size(mesh, cfg.pipe_axis)
        self.s = C.axis_index(mesh, cfg.pipe_axis)
        self.n_dp = C.axis_size(mesh, cfg.data_axis)
        self.first, self.last = self.s == 0, self.s == self.S - 1
        self.act_dtype = act_dtype
        P = state.params
        self.dev = P.master.device
        self.metrics = torch.zeros(N_METRIC_SLOTS, dtype=torch.float32, device=self.dev)
        # the CE's per-workgroup metric rows (ops.kernels.softmax_xent mslab), folded at the
        # step's end -- only where that fold is local (no data axis: with one, the metric
        # slots ride the gradient all-reduce); JDT_XENT_SLAB=0 restores the slot atomics
        self._mslab = (torch.zeros(1024, 4, dtype=torch.float32, device=self.dev)
                       if (self.dev.type == "cuda" and self.n_dp == 1
                           and os.environ.get("JDT_XENT_SLAB", "1") != "0") else None)
        self.graph = None
        self._ahead = None
        self.multi = None
        self.p2p = None
        self._p2p_tried = False
        self.xg = None
        self._xg_fused_opt = False
        self.wgrad = K.WGradStream(self.dev) if (self.dev.type == "cuda" and cfg.overlap_wgrad) else None
        self._mb_streams = None
        self._w_streams = None
        self.stage_engine = None
        self._engine_tried = False
        self.deep_engine = None
        self._deep_tried = False
        self.pp_kernel = None          # the in-kernel GPipe step (parallel/pp_kernel.py)
        self._pp_kernel_tried = False
        self._handoffs_stale = False   # a checkpoint restore moved the step counter: rebuild them
        from ..utils.checkpoint import bind_trainer

        bind_trainer(state, self)
        if self.dev.type == "cuda" and self.n_dp > 1:
            from ..comm.xgmi import create_for

            self.xg = create_for(mesh, cfg.data_axis, P.grad.numel(), self.dev, cfg.comm)
            self._xg_fused_opt = self.xg is not None and isinstance(state.tx, AdamW)
        # ranks time-sharing one GPU (rehearsals): schedules with concurrent spinning
        # streams stay off in "auto" mode (collective: every rank builds its trainer)
        from ..runtime.dist import ranks_share_gpu

        self._gpu_shared = ranks_share_gpu() if self.dev.type == "cuda" else False

    # ------------------------------------------------------------------ p2p
    def _setup_p2p(self, mb: int):
        if self._p2p_tried or self.S == 1 or self.dev.type != "cuda":
            return
        self._p2p_tried = True
        from ..comm.p2p import create_for

        es = torch.tensor([], dtype=self.act_dtype).element_size()
        nbytes = max(math.prod(self.model.input_shape(mb)), math.prod(self.model.output_shape(mb))) * es
        # slot i: forward activation of microbatch i; slot n_mb + i: its gradient
        self.p2p = create_for(self.mesh, self.cfg.pipe_axis, nbytes, 2 * self.cfg.num_microbatches, self.dev,
                              self.cfg.comm)

    def _send(self, x: torch.Tensor, to: int, slot: int):
        with named_scope("pipe_send"):
            if self.p2p is not None:
                self.p2p.send(x, to, slot, self.state.step_tensor)
            else:
                C.send(x, self.mesh, self.cfg.pipe_axis, to)

    def _recv(self, shape, to_dtype, frm: int, slot: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        with named_scope("pipe_recv"):
            buf = torch.empty(shape, dtype=to_dtype, device=self.dev) if out is None else out
            if self.p2p is not None:
                return self.p2p.recv(buf, slot, self.state.step_tensor)
            return C.recv(buf, self.mesh, self.cfg.pipe_axis, frm)

    @property
    def capturable(self) -> bool:
        """Whether the step can be recorded as a hipGraph: every hand-off and collective
        is an xGMI kernel or an RCCL call (RCCL send / recv / all-reduce enqueue on the
        capturing stream); a gloo group's host-side ops keep it eager."""
        from ..runtime.dist import collectives_capturable

        rccl = collectives_capturable()
        return (self.dev.type == "cuda" and (self.S == 1 or self.p2p is not None or self.pp_kernel is not None or rccl)
                and (self.n_dp == 1 or self.xg is not None or rccl))

    @property
    def comm_backend(self) -> str:
        if self.S * self.n_dp == 1:
            return "none"
        if (self.S == 1 or self.p2p is not None or self.pp_kernel is not None) and (self.n_dp == 1 or self.xg is not None):
            return "xgmi"
        from ..runtime.dist import backend

        b = backend()
        return "rccl" if b == "nccl" else (b or "none")

    @property
    def xgmi_status(self) -> str:
        from ..comm.xgmi import status

        dp = status(self.xg, self.n_dp, self.dev, self.cfg.comm)
        if self.S == 1:
            return dp
        pipe = "passed" if (self.p2p is not None or self.pp_kernel is not None) else (
            "failed->rccl" if self._p2p_tried and self.dev.type == "cuda"
                                                      and self.cfg.comm != "rccl" else "off")
        return f"data:{dp},pipe:{pipe}"

    # ------------------------------------------------------------------ step
    def _drop_stale_handoffs(self):
        """After a restore (``invalidate``): the stage hand-offs wait until a flag is >= the
        step epoch -- the in-kernel GPipe engine's inbox / weight-box / counter words and the
        per-tick xGMI inbox (comm/p2p.py, epoch = the device step) -- and their flags still
        hold the epochs of steps the restore rolled back, so every wait would pass at once
        on stale data.  Drop both so the next step rebuilds them from zeroed buffers.
        Collective (every rank restores, then steps or captures); quiesce first so no peer
        still writes into the old inboxes.  Never called inside a stream capture."""
        if not self._handoffs_stale:
            return
        from ..runtime.dist import quiesce

        self._handoffs_stale = False
        quiesce(self.dev)
        for r in (self.pp_kernel, self.p2p):
            if r is not None:
                r.close()
        self.pp_kernel = self.p2p = None
        self._pp_kernel_tried = self._p2p_tried = False

    def _pp_kernel_engine(self, mb: int, seed: int):
        """The whole stage step as one persistent launch (parallel/pp_kernel.py), when
        every stage of the pipe axis can run it (collective on first use); with a pipe
        axis of size 1, the one-GPU chain: every layer of the MLP a stage of one launch."""
        self._drop_stale_handoffs()
        if not self._pp_kernel_tried:
            self._pp_kernel_tried = True
            if self.S == 1 and self.dev.type == "cuda":
                from . import pp_kernel as PK

                if PK.chain_ok(self, mb):
                    self.pp_kernel = PK.PPChainKernel(self, mb, seed)
            elif self.S > 1 and self.dev.type == "cuda":
                from ..comm.tile_exchange import agree
                from . import pp_kernel as PK

                ok = agree(self.mesh.group(self.cfg.pipe_axis), PK.local_ok(self, mb), self.dev)
                if ok:
                    eng = PK.PPStageKernel(self, mb, seed)
                    self.pp_kernel = eng if eng.ok else None
        return self.pp_kernel

    def _compute(self, batch: Batch):
        st, P, cfg = self.state, self.state.params, self.cfg
        n_mb = cfg.num_microbatches
        mb = batch.size // n_mb
        rng = R.fold_rng_over_axis(st.rng, self.mesh, cfg.data_axis)
        seed = rng & 0xFFFFFFFF
        if self._pp_kernel_engine(mb, seed) is not None:
            # every tick and hand-off in ONE launch, then the AdamW launch (csrc/pp_stage.hip)
            self.pp_kernel.step(batch, seed)
            return
        self._setup_p2p(mb)
        if self.S == 1:
            deep = self._single_stage_engine(batch.size, mb)
            if deep is not None:
                deep.forward_backward(batch)
                return
        eo = self._epilogue_opt()
        if self.S == 1 and (cfg.merge_single_stage or (cfg.layer_major_single_stage and _no_dropout(self.model)
                                                       and self._mb_streams_k() <= 1)):
            if self._layer_major_wpass(batch, P, st, seed, eo, n_mb):
                return
            out, cache = self.model.forward(P, batch.inputs, train=True, seed=seed, offset=0, step=st.step_tensor)
            d = torch.empty_like(out)
            self.loss_head(out, batch.labels, d, n_parts=n_mb)
            ov = self._overlapped_opt() if eo is None else None
            if eo is not None:
                eo.only_contribution = True   # one pass: each weight's only gradient contribution
            self.model.backward(P, cache, d, dout_is_dz=True, need_dx=False, wgrad=self.wgrad,
                                on_ready=ov.ready if ov is not None else None, opt=eo)
            return
        eng = self._fused_stage(mb, seed)
        if eng is not None:
            self._compute_fused(batch, eng, n_mb, mb)
            return
        caches, dlogits = [None] * n_mb, [None] * n_mb
        arena = self._wgrad_arena(batch.size)
        akw = {"arena": arena, "n_mb": n_mb} if arena is not None else {}
        on = self._mb_stream_ctx(arena, n_mb)
        on.fork()   # after the previous step's optimizer / this step's inputs
        # ---- forward fill/drain: tick t, stage s handles microbatch t - s
        for t in range(n_mb + self.S - 1):
            i = t - self.s
            if not (0 <= i < n_mb):
                continue
            with on(i):
                self._forward_mb(batch, P, st, seed, caches, dlogits, arena, akw, i, mb)
        # ---- backward, reverse microbatch order (the last one, i = 0, carries the
        # weights' final gradients: the in-epilogue optimizer when enabled)
        if eo is not None:
            eo.only_contribution = n_mb == 1
        top = list(getattr(self.model, "layers", []))[-1:] if arena is not None else []
        # early W pass (on dedicated streams): each part's weight-gradient GEMMs start once
        # every microbatch chain has passed that part (per-chain events), not after the join
        nw = int(self.cfg.wpass_early) if (on.side and hasattr(self.model, "weight_grads_of")) else 0
        evs: dict = {}

        def mark(part):
            ev = torch.cuda.Event()
            ev.record()
            evs.setdefault(part, []).append(ev)

        bkw = {"after": mark} if nw else {}
        for i in reversed(range(n_mb)):
            oi = eo if (i == 0 and arena is None) else None
            with on(i):
                if self.last:
                    dx = self.model.backward(P, caches[i], dlogits[i], dout_is_dz=True, need_dx=not self.first,
                                             wgrad=self.wgrad, opt=oi, **bkw)
                else:
                    into = arena.rows(arena.blocks[top[0]]["dx3"], i, n_mb) if top else None
                    dh = self._recv(self.model.output_shape(mb), self.act_dtype, self.s + 1, n_mb + i, out=into)
                    dx = self.model.backward(P, caches[i], dh, dout_is_dz=False, need_dx=not self.first,
                                             wgrad=self.wgrad, opt=oi, **bkw)
                if not self.first:
                    self._send(dx, self.s - 1, n_mb + i)
                caches[i] = None
        if nw:
            if self._w_streams is None or len(self._w_streams) != nw:
                self._w_streams = [torch.cuda.Stream(self.dev) for _ in range(nw)]
            ws, j = self._w_streams, 0
            for part in (["head"] if self.model.has_head else []) + list(reversed(list(self.model.layers))):
                for w in ws:
                    for ev in evs[part]:
                        w.wait_event(ev)
                j = self.model.weight_grads_of(P, arena, part, opt=eo, on=lambda g: torch.cuda.stream(ws[g % nw]),
                                               j0=j)
            for w in ws:
                on.main.wait_stream(w)
            on.join()
            return
        if arena is not None and not on.side and self._overlap_sync_ok():
            self._overlapped_sync(P, arena)
            return
        if arena is not None:
            # the W pass: every weight gradient of the step, one GEMM per weight over all
            # rows (the GEMMs round-robin over the streams once every chain has finished)
            on.join()
            on.fork()
            if self._wpass_one_ok():
                with K.gemm_wpass():   # one launch on the main stream
                    self.model.weight_grads(P, arena, opt=eo)
            else:
                nw = max(1, int(self.cfg.wpass_rr) or len(on.side) + 1)
                self.model.weight_grads(P, arena, wgrad=self.wgrad, opt=eo, on=lambda j: on(j % nw))
        on.join()

    def _wpass_one_ok(self) -> bool:
        return (self.cfg.wpass_one_launch and self.dev.type == "cuda" and self.wgrad is None
                and hasattr(self.model, "weight_grads"))

    def _overlap_sync_ok(self) -> bool:
        mode = str(self.cfg.overlap_data_sync)
        on = mode == "1" or (mode == "auto" and not self._gpu_shared)
        return (on and self.S > 1 and self._xg_fused_opt and self.wgrad is None and self.dev.type == "cuda"
                and hasattr(self.model, "sync_groups") and hw_queues() >= 2)

    @property
    def data_sync_mode(self) -> str:
        """How the data-axis sync runs (bench JSON): "none" (no data axis), "one call",
        or "overlapped (k buckets)" -- per W-pass group on a comm stream."""
        if self.n_dp == 1:
            return "none"
        if self._overlap_sync_ok():
            return f"overlapped ({len(self._sync_buckets())} buckets)"
        return "one call"

    def _sync_buckets(self):
        """The overlapped data-axis sync's buckets, in issue order: (key, lo, hi, metrics,
        advance).  One bucket per group of ``model.sync_groups`` (the embedding, then one
        per weight-gradient GEMM in W-pass order), each the flat range from the group's
        first parameter to the next group's (FlatParams offsets are 4-aligned, so every
        range is a valid kernel bucket); the range that ends the flat buffer also carries
        the metric slots, and the last bucket issued advances the optimizer step."""
        if getattr(self, "_buckets", None) is None:
            P = self.state.params
            groups = self.model.sync_groups()
            starts = sorted((P.offsets[first][0], key) for key, first in groups)
            rng = {}
            for k, (lo, key) in enumerate(starts):
                hi = starts[k + 1][0] if k + 1 < len(starts) else P.numel
                rng[key] = (lo, hi, k + 1 == len(starts))
            self._buckets = [(key, *rng[key], i + 1 == len(groups)) for i, (key, _) in enumerate(groups)]
        return self._buckets

    def _overlapped_sync(self, P, arena):
        """The W pass with the data-axis sync overlapped: each weight-gradient GEMM on the
        main stream, then its group's xGMI all-reduce + AdamW on a comm stream (the kernel
        only reads the group's final gradients and writes its parameters / moments /
        shadow, which nothing on the main stream touches until the join).  Same
        per-element reduction order and AdamW as the single call."""
        st, cfg = self.state, self.cfg
        tx, o = st.tx, st.opt_state
        scale = 1.0 / (cfg.num_microbatches * self.n_dp)
        main = torch.cuda.current_stream(self.dev)
        cs = getattr(self, "_comm_stream", None)
        if cs is None:
            cs = self._comm_stream = torch.cuda.Stream(self.dev)
        G = P.grad
        gemms = {}
        for part in (["head"] if self.model.has_head else []) + list(self.model.layers):
            for name, h, dz in self.model.weight_grad_items(arena, part):
                gemms[name] = (h, dz)
        for key, lo, hi, metrics, advance in self._sync_buckets():
            if key != "embed":
                h, dz = gemms[key]
                K.dw_gemm(None, h, dz, P.g(key), name=key)
            cs.wait_stream(main)
            with torch.cuda.stream(cs), named_scope("sync_grads_part"):
                end = G.numel() if metrics else hi
                self.xg.all_reduce_adamw_(
                    G[lo:end], p=P.master[lo:end], m=o["m"][lo:end], v=o["v"][lo:end], shadow=P.shadow[lo:end],
                    n_params=hi - lo, running=self.metrics if metrics else None,
                    n_metrics=N_METRIC_SLOTS if metrics else 0, lr=tx.learning_rate, b1=tx.b1, b2=tx.b2,
                    eps=tx.eps, wd=tx.weight_decay, grad_scale=scale, step=o["count"], ticket=o["ticket"],
                    zero_grad=True, advance=advance)
        main.wait_stream(cs)
        self._synced = True

    def _layer_major_wpass(self, batch, P, st, seed, eo, n_mb) -> bool:
        """One stage, one pass over all rows, weight gradients deferred (cfg.wpass_streams
        = k > 1, GPU): the backward runs the input-gradient chain only and each part's
        weight-gradient GEMMs (AdamW in their epilogues) go out round-robin on k - 1 side
        streams as soon as the chain has produced that part's output gradients
        (TransformerLM.backward ``after`` hook), overlapping the rest of the chain."""
        k = int(self.cfg.wpass_streams)
        # (the opt-in layer-by-layer side-stream AdamW needs each layer's gradients final
        # as the backward passes it: the inline weight GEMMs of the plain pass)
        if (k <= 1 and self._wpass_one_ok() and hasattr(self.model, "weight_grads_of")
                and (eo is not None or self._overlapped_opt() is None)):
            return self._layer_major_one_wpass(batch, P, st, seed, eo, n_mb)
        if k <= 1 or self.dev.type != "cuda" or not hasattr(self.model, "weight_grads_of"):
            return False
        arena = self._wgrad_arena(batch.size)
        if arena is None:
            return False
        if self._mb_streams is None or len(self._mb_streams) != k - 1:
            self._mb_streams = [torch.cuda.Stream(self.dev) for _ in range(k - 1)]
        on = _MbStreams(torch.cuda.current_stream(self.dev), self._mb_streams)
        out, cache = self.model.forward(P, batch.inputs, train=True, seed=seed, offset=0, step=st.step_tensor,
                                        arena=arena, mb=0, n_mb=1)
        d = arena.head["dlog"] if self.model.has_head else torch.empty_like(out)
        self.loss_head(out, batch.labels, d, n_parts=n_mb)
        j = [0]

        def after(part):
            on.fork()   # the side streams see the chain so far
            j[0] = self.model.weight_grads_of(P, arena, part, opt=eo, on=lambda i: on(1 + i % (k - 1)), j0=j[0])

        self.model.backward(P, cache, d, dout_is_dz=True, need_dx=False, after=after)
        on.join()
        return True

    def _layer_major_one_wpass(self, batch, P, st, seed, eo, n_mb) -> bool:
        """One stage, one pass over all rows: the forward, the input-gradient chain, then
        every weight gradient of the step in ONE launch (ops.kernels.gemm_wpass, AdamW in
        the epilogues), instead of a grouped dW + dX launch per layer."""
        arena = self._wgrad_arena(batch.size)
        if arena is None:
            return False
        out, cache = self.model.forward(P, batch.inputs, train=True, seed=seed, offset=0, step=st.step_tensor,
                                        arena=arena, mb=0, n_mb=1)
        d = arena.head["dlog"] if self.model.has_head else torch.empty_like(out)
        self.loss_head(out, batch.labels, d, n_parts=n_mb)
        self.model.backward(P, cache, d, dout_is_dz=True, need_dx=False)
        with K.gemm_wpass():
            self.model.weight_grads(P, arena, opt=eo)
        return True

    def _mb_stream_ctx(self, arena, n_mb: int) -> "_MbStreams":
        """Microbatch i's passes (and the W pass's GEMM j) run on stream i % k when
        ``cfg.mb_streams`` = k > 1 applies: GPU, one stage, deferred weight gradients."""
        k = self._mb_streams_k()
        if not (k > 1 and arena is not None):
            return _MbStreams(None, None)
        if self._mb_streams is None or len(self._mb_streams) != k - 1:
            self._mb_streams = [torch.cuda.Stream(self.dev) for _ in range(k - 1)]
        return _MbStreams(torch.cuda.current_stream(self.dev), self._mb_streams)

    def _forward_mb(self, batch, P, st, seed, caches, dlogits, arena, akw, i, mb):
        n_mb = self.cfg.num_microbatches
        if self.first:
            x = batch.inputs[i * mb:(i + 1) * mb]
        else:
            x = self._recv(self.model.input_shape(mb), self.act_dtype, self.s - 1, i)
        if arena is not None:
            akw["mb"] = i
        out, cache = self.model.forward(P, x, train=True, seed=seed, offset=i << 16, step=st.step_tensor, **akw)
        caches[i] = cache
        if self.last:
            d = torch.empty_like(out) if arena is None else arena.rows(arena.head["dlog"], i, n_mb)
            self.loss_head(out, batch.labels[i * mb:(i + 1) * mb], d)
            dlogits[i] = d
        else:
            self._send(out, self.s + 1, i)

    def _wgrad_arena(self, rows: int):
        """The stage model's deferred weight-gradient buffers (models.transformer.WGradArena)
        for ``rows`` local sequences, or None (model without them, or defer_wgrad off)."""
        if not self.cfg.defer_wgrad or not hasattr(self.model, "weight_grads"):
            return None
        ar = getattr(self, "_arena", None)
        if ar is None or ar.nseq != rows:
            from ..models.transformer import WGradArena

            ar = self._arena = WGradArena(self.model, rows, self.dev)
        return ar

    @property
    def single_stage_mode(self) -> str:
        """How a pipe axis of size 1 runs its microbatches (bench JSON): "merged"
        (one pass, merged dropout stream), "layer-major" (one pass per layer, the
        loop's masks), "microbatch-loop", or "pipeline" (S > 1)."""
        if self.S > 1:
            return "pipeline"
        if self.cfg.merge_single_stage:
            return "merged"
        k = self._mb_streams_k()
        if self.cfg.layer_major_single_stage and (self.deep_engine is not None or _no_dropout(self.model)) and k <= 1:
            return "layer-major"
        return f"microbatch-loop ({k} streams)" if k > 1 else "microbatch-loop"

    def _mb_streams_k(self) -> int:
        """Streams the per-microbatch passes of a one-stage pipeline run on (1: serial);
        never more than the process's HIP hardware queues (GPU_MAX_HW_QUEUES when set:
        a 4-stream graph on 2 queues crashed the runtime in a probe,
        profiles/r3_lm_mb_streams_ab.txt)."""
        want = int(self.cfg.mb_streams)
        if want <= 0:   # auto: the layer-major pass with its one-launch W pass where it applies
            one = (self.S == 1 and self.cfg.layer_major_single_stage and _no_dropout(self.model)
                   and self.cfg.wpass_streams <= 1 and self._wpass_one_ok() and hasattr(self.model, "weight_grads_of"))
            want = 1 if one else 4
        k = min(want, self.cfg.num_microbatches, hw_queues())
        ok = (self._streams_ok() and self.cfg.defer_wgrad and hasattr(self.model, "weight_grads")
              and not self.cfg.merge_single_stage)
        return k if ok else 1

    @property
    def stage_streams(self) -> int:
        """Streams this stage's microbatch chains ran on (bench JSON)."""
        if self.stage_engine is not None:
            return self.stage_engine.n_sets
        if self.deep_engine is not None:
            return 1
        return self._mb_streams_k()

    def _streams_ok(self) -> bool:
        """Whether this stage may run its microbatch chains on concurrent streams: GPU,
        and either one stage or -- opt-in, ``cfg.multi_stage_streams`` -- every hand-off
        on the xGMI inbox kernels (per-microbatch slots, stream-ordered reuse:
        comm/csrc/p2p.hip; RCCL send / recv issued from several streams of one
        communicator could pair up out of order across ranks).  Off by default for
        S > 1: with 4 / 8 ranks sharing one GPU it measured 5x / 20x SLOWER
        (profiles/r4_pp_streams_ab.txt) -- every rank's receive kernels then spin on
        concurrent hardware queues of a time-shared GPU; a real node (one rank per GPU)
        is unmeasured."""
        if self.dev.type != "cuda":
            return False
        return self.S == 1 or (self.p2p is not None and self.cfg.multi_stage_streams)

    def invalidate(self):
        """After a checkpoint restore: drop captured graphs and the stage engine."""
        self._eo = None
        self.graph = None
        self._ahead = None
        self.multi = None
        self.stage_engine = None
        self._engine_tried = False
        self.deep_engine = None
        self._deep_tried = False
        if self.pp_kernel is not None or self.p2p is not None:
            self._handoffs_stale = True   # rebuilt (zeroed hand-off flags, new seed) at the next step

    def _single_stage_engine(self, rows: int, mb: int):
        """One stage holding the whole MLP (pipe axis of size 1): GPipe's fill/drain
        degenerates to gradient accumulation over the microbatches, so the fused deep
        kernels run all of this rank's rows layer by layer (one md_fwd / md_bwd launch
        per layer instead of one per layer AND microbatch) while every row keeps its
        microbatch's 1/mb loss weight and -- unless ``merge_single_stage`` -- its
        microbatch's own dropout stream (``mb_rows``): the same masks, hence the same
        gradient, as the microbatch loop."""
        if not self._deep_tried:
            self._deep_tried = True
            from .fused_mlp import FusedMLPDeep, supported_deep

            if (self.cfg.fused_stage and self.cfg.layer_major_single_stage and self.wgrad is None
                    and not getattr(self.model, "final_act", True)
                    and supported_deep(self.model, rows, self.dev)):
                self.deep_engine = FusedMLPDeep(self.state, self.mesh, self.cfg.data_axis, self.cfg.num_microbatches,
                                                rows, self.metrics,
                                                mb_rows=0 if self.cfg.merge_single_stage else mb)
        return self.deep_engine

    def _fused_stage(self, mb: int, seed: int):
        if not self._engine_tried:
            self._engine_tried = True
            from .fused_stage import FusedMLPStage, stage_supported

            if self.cfg.fused_stage and self.wgrad is None and stage_supported(self.model, mb, self.dev):
                # S > 1 on the inbox kernels: microbatch i on stream i % k, with its own grad
                # set (every md-kernel gradient write is a read-modify-write), merged after
                # the join -- the DP minibatch loop's scheme (FusedMLPStage n_sets)
                k = self._stage_streams_k()
                self.stage_engine = FusedMLPStage(self.model, self.state.params, self.cfg.num_microbatches, mb,
                                                  self.state.step_tensor, seed, n_sets=k)
        return self.stage_engine

    def _stage_streams_k(self) -> int:
        """Concurrent streams of a multi-stage MLP stage's microbatch chains (1: serial)."""
        if self.S == 1 or not self._streams_ok():
            return 1
        return max(1, min(int(self.cfg.mb_streams) or 4, self.cfg.num_microbatches, hw_queues()))

    def _compute_fused(self, batch: Batch, eng, n_mb: int, mb: int):
        """The same GPipe fill/drain schedule on the fused stage kernels.  With
        ``eng.n_sets`` = k > 1 (S > 1, xGMI inbox hand-offs) microbatch i's receive,
        compute and send run on stream i % k: a stage starts microbatch i as soon as it
        arrives while earlier ones still run (latency-bound ticks overlap instead of
        queueing), and the backward of one microbatch overlaps another's."""
        k = eng.n_sets
        if k > 1:
            if self._mb_streams is None or len(self._mb_streams) != k - 1:
                self._mb_streams = [torch.cuda.Stream(self.dev) for _ in range(k - 1)]
            on = _MbStreams(torch.cuda.current_stream(self.dev), self._mb_streams)
        else:
            on = _MbStreams(None, None)
        on.fork()
        for t in range(n_mb + self.S - 1):
            i = t - self.s
            if not (0 <= i < n_mb):
                continue
            with on(i):
                if self.first:
                    x = batch.inputs[i * mb:(i + 1) * mb]
                else:
                    x = self._recv(self.model.input_shape(mb), self.act_dtype, self.s - 1, i)
                out = eng.forward(i, x)
                if not self.last:
                    self._send(out, self.s + 1, i)
        for i in reversed(range(n_mb)):
            with on(i):
                if self.last:
                    dx = eng.backward(i, labels=batch.labels[i * mb:(i + 1) * mb], need_dx=not self.first)
                else:
                    dh = self._recv(self.model.output_shape(mb), self.act_dtype, self.s + 1, n_mb + i)
                    dx = eng.backward(i, dh=dh, need_dx=not self.first)
                if not self.first:
                    self._send(dx, self.s - 1, n_mb + i)
        on.join()
        if k > 1:
            eng.merge()

    def _epilogue_opt(self):
        """The in-epilogue AdamW (ops.kernels.EpilogueAdamW) for a transformer stage
        with no data axis on a GPU: weights updated in their final weight-gradient
        GEMMs, the rest by one multi-range launch in _sync_update.  JDT_LM_FUSED_OPT=0
        turns it off (A/B)."""
        if getattr(self, "_eo", None) is None:
            from ..utils.train_state import AdamW

            st, cfg = self.state, self.cfg
            ok = (self.n_dp == 1 and self.wgrad is None and isinstance(st.tx, AdamW) and st.params.master.is_cuda
                  and hasattr(self.model, "gemm_weight_names")
                  and os.environ.get("JDT_LM_FUSED_OPT", "1") != "0")
            self._eo = (K.EpilogueAdamW(st.params, st.tx, st.opt_state, 1.0 / (cfg.num_microbatches * self.n_dp),
                                        self.model.gemm_weight_names()) if ok else False)
        return self._eo or None

    def _overlapped_opt(self):
        """The layer-by-layer side-stream AdamW (one GPU, one stage, no data axis)."""
        if getattr(self, "_ov_opt", None) is None:
            from ..utils.train_state import AdamW

            st, cfg = self.state, self.cfg
            ok = (cfg.overlap_optimizer and os.environ.get("JDT_OVERLAP_OPT", "0") == "1" and self.S == 1
                  and self.n_dp == 1 and self.wgrad is None and isinstance(st.tx, AdamW)
                  and st.params.master.is_cuda)
            self._ov_opt = K.OverlappedAdamW(st.params, st.tx, st.opt_state, 1.0 / cfg.num_microbatches) if ok else False
        return self._ov_opt or None

    def _sync_update(self):
        """sync_gradients(('data','pipe')): stage params are pipe-sharded -> mean over
        'data' only; then AdamW on the local stage and the metrics fold.  The host
        step counter is advanced by the callers."""
        st, P, cfg = self.state, self.state.params, self.cfg
        if self.pp_kernel is not None:
            return   # AdamW, the metrics fold and the step advance ran inside the stage launch
        if getattr(self, "_synced", False):   # the W pass issued the sync per part (_overlapped_sync)
            self._synced = False
            return
        scale = 1.0 / (cfg.num_microbatches * self.n_dp)
        ov = getattr(self, "_ov_opt", None)
        if ov and ov.forked:   # AdamW already forked layer by layer during the backward
            ov.finish()
            with named_scope("sync_metrics"):
                K.metrics_fold_(self.metrics, P.metrics_slot, slab=self._mslab)
            return
        if self.wgrad is not None:
            self.wgrad.join()  # every weight-gradient GEMM of the step has landed
        if self.deep_engine is not None and self.deep_engine.fuse_opt:
            return  # one GPU, one stage: AdamW + metrics fold ran in the backward epilogues
        eo = self._epilogue_opt() if self.deep_engine is None and self.stage_engine is None else None
        if eo is not None:
            # weights: updated in their weight-gradient GEMM epilogues; the rest here
            # (on a side stream beside the W pass it measured slower: BENCH_NOTES round 6)
            eo.finish()
            with named_scope("sync_metrics"):
                K.metrics_fold_(self.metrics, P.metrics_slot, slab=self._mslab)
            return
        with named_scope("sync_grads"):
            if self._xg_fused_opt:
                tx, o = st.tx, st.opt_state
                self.xg.all_reduce_adamw_(
                    P.grad, p=P.master, m=o["m"], v=o["v"], shadow=P.shadow, n_params=P.numel,
                    running=self.metrics, n_metrics=N_METRIC_SLOTS, lr=tx.learning_rate, b1=tx.b1, b2=tx.b2,
                    eps=tx.eps, wd=tx.weight_decay, grad_scale=scale, step=o["count"], ticket=o["ticket"],
                    zero_grad=True)
                return  # AdamW + metrics fold ran inside the all-reduce kernel
            if self.xg is not None:
                self.xg.all_reduce_(P.grad)
            else:
                C.psum_(P.grad, self.mesh, cfg.data_axis)
        st.tx.update(P, st.opt_state, scale)
        with named_scope("sync_metrics"):
            K.metrics_fold_(self.metrics, P.metrics_slot, slab=self._mslab)

    def set_batch(self, batch: Batch):
        """New data for captured graphs (see DataParallelTrainer.set_batch)."""
        if getattr(self, "_static", None) is not None:
            load_static_batch(self._static, batch, (self.deep_engine,))

    def step(self, batch: Batch):
        if self.graph is not None:
            check_static_batch(getattr(self, "_static", None), batch)
            with replay_scope("train_step_pp"):
                self._ahead.replay(1) if getattr(self, "_ahead", None) else self.graph.replay()
        else:
            self._compute(batch)
            self._sync_update()
        self.state.step += 1

    # ------------------------------------------------------------------ hipGraph
    def capture(self, batch: Batch, steps_per_graph: int = 1):
        """Record the step (and a ``steps_per_graph``-step variant) as hipGraphs.
        Every rank of the mesh must capture; the batch must stay alive."""
        if not self.capturable:
            raise RuntimeError("pipeline step is not capturable (host-driven collectives)")
        self._static = batch
        self._drop_stale_handoffs()   # a restore since the last step: rebuild outside the capture

        def body():
            self._compute(batch)
            self._sync_update()

        from .dp import capture_graph

        g = capture_graph(body)
        if g is None:   # a collective refused stream capture: the step stays eager
            self.graph = None
            return False
        self.graph = g
        # one stage on the deep fused engine: layer 0's forward of the next step rides in
        # the layer-0 backward (run-ahead, fused_mlp.AheadGraphs: cold / primed graphs)
        eng = self.deep_engine
        self._ahead = None
        if self.S == 1 and eng is not None and getattr(eng, "ahead_ok", False):
            from .fused_mlp import AheadGraphs

            self._ahead = AheadGraphs(eng, batch, steps_per_graph, pool=g.pool())
            if steps_per_graph > 1:
                self.multi = (steps_per_graph, self._ahead.graph(steps_per_graph))
        elif steps_per_graph > 1:
            gm = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gm, pool=g.pool()):
                for _ in range(steps_per_graph):
                    body()
            self.multi = (steps_per_graph, gm)
        return True

    def run_steps(self, batch: Batch, n: int):
        if self.graph is not None:
            check_static_batch(getattr(self, "_static", None), batch)
        if self.graph is not None and self.multi is not None:
            S, gm = self.multi
            for _ in range(n // S):
                with replay_scope("train_step_pp", S):
                    self._ahead.replay(S) if self._ahead else gm.replay()
            self.state.step += (n // S) * S
            n %= S
        for _ in range(n):
            self.step(batch)

    def finalize(self):
        if self.deep_engine is not None:
            self.deep_engine.finalize()  # bf16 shadow parity of the in-epilogue AdamW
        if self.p2p is not None and self.p2p.error():
            raise RuntimeError("xgmi pipeline receive timed out on this rank (peer dead or desynchronised)")
        if self.pp_kernel is not None and self.pp_kernel.error():
            raise RuntimeError("pipeline stage kernel: an in-kernel wait timed out on this rank (peer dead or "
                               "desynchronised); results invalid")
        if self.xg is not None:
            self.xg.raise_if_error()

    def close(self):
        """Release the inboxes and the xGMI context and drop the captured graphs, so
        another trainer can be built in this process (bench.py's autotune candidates).
        Collective (runtime.dist.quiesce)."""
        from ..runtime.dist import quiesce

        quiesce(self.dev)
        for r in (self.p2p, self.xg, self.pp_kernel):
            if r is not None:
                r.close()
        self.p2p = self.xg = self.pp_kernel = None
        self.graph = self._ahead = self.multi = None

    def loss_head(self, logits, labels, dlogits, n_parts: int = 1):
        """CE of ``labels`` (``n_parts`` merged microbatches: every row keeps its
        microbatch's 1/rows weight)."""
        y = self.model.flatten_labels(labels)
        hb = self.model.head_bias_name
        K.softmax_xent(logits, y, grad_scale=n_parts / y.numel(), dlogits=dlogits,
                       dbias=self.state.params.g(hb) if hb else None, metrics=self.state.params.metrics_slot,
                       mslab=self._mslab)

    def gather_metrics(self) -> torch.Tensor:
        """Metrics live on the last stage; bring them to every pipe member."""
        m = self.metrics.clone()
        if self.mesh is not None and self.S > 1 and is_initialized():
            if not self.last:
                m.zero_()
            C.psum_(m, self.mesh, self.cfg.pipe_axis)
        return m
