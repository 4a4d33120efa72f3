"""Data parallelism with gradient accumulation (reference data_paral.py:128-277).

Reference step (data_paral.py:193-238), per device under shard_map:
    rng split -> accum_grads over 4 minibatches -> pmean(grads, 'data')
    -> adamw apply_gradients -> psum(metrics, 'data') -> metrics += step_metrics

MI355X step, per GPU process:
    for each minibatch: 2 fwd GEMMs, fused CE(+metrics, +top bias grad),
                        dW GEMM(s) with beta=1, dz GEMM(s) with fused act'/mask/db
    ONE all-reduce (RCCL, SUM) of [flat fp32 grads || 4 metric scalars]   (X03+X04)
    ONE fused AdamW kernel (grad scale 1/(n_mb * N) folded in, bf16 shadow out,
                           grad buffer zeroed)
    ONE metrics-fold kernel (running += step metrics)
The whole step is captured as a hipGraph after warmup (N=1: one graph; N>1:
compute graph + RCCL all-reduce + optimizer graph, or one graph with the
collective inside when ``capture_collectives``).

``accum="loop"`` runs the minibatches sequentially exactly like
util.accum_grads_loop; ``accum="fused"`` runs all of a device's rows in one
pass (identical gradient: each row is weighted 1/(mb*n_mb) either way; only the
dropout streams are indexed differently) -- 4x fewer launches.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field
from typing import Optional

import torch

from ..comm import collectives as C
from ..models.mlp import MLP, loss_and_grad
from ..ops import kernels as K
from ..runtime.dist import Mesh
from ..utils import rng as R
from ..utils.flat import FlatParams, N_METRIC_SLOTS
from ..utils.profiling import named_scope, replay_scope
from ..utils.train_state import AdamW, Batch, TrainState, check_static_batch, load_static_batch


def fold_rng_over_axis(rng: int, mesh: Optional[Mesh], axis_name: str) -> int:
    """data_paral.py:28-34."""
    return R.fold_rng_over_axis(rng, mesh, axis_name)


def shard_batch(batch: Batch, mesh: Optional[Mesh], axis: str) -> Batch:
    """Rows [r*B/N, (r+1)*B/N) to member r of ``axis`` (in_specs=P('data'), X10)."""
    n = C.axis_size(mesh, axis)
    if n == 1:
        return batch
    r = C.axis_index(mesh, axis)
    per = batch.size // n
    return batch.slice(r * per, per)


def init_dp(model: MLP, tx, seed: int, device, mesh: Optional[Mesh] = None, axis: str = "data") -> TrainState:
    """data_paral.py:128-168: same seed on every rank -> replicated params; rank 0
    broadcasts anyway so replication holds even if init were nondeterministic."""
    params = FlatParams(model.param_specs(), device=device)
    params.init_(seed)
    if mesh is not None and C.axis_size(mesh, axis) > 1:
        C.broadcast_(params.master, mesh, axis, 0)
        params.sync_shadow()
    return TrainState.create(apply_fn=model, params=params, tx=tx, rng=R.PRNGKey(seed))


@dataclass
class DPConfig:
    num_minibatches: int = 4
    accum: str = "loop"          # "loop" | "scan" | "fused" | "kernel" (whole-step fused kernels, parallel/fused_mlp.py)
    axis: str = "data"
    overlap: bool = True         # eager generic path: bucketed all-reduce overlapping the last backward
    bucket_mb: float = 25.0
    comm: str = "auto"           # "auto" | "xgmi" | "rccl": N>1 gradient collective (comm/xgmi.py)
    # accum "loop" on the fused per-layer kernels (parallel/fused_stage.py): the same
    # per-minibatch passes and dropout streams as the generic loop, 2 launches per
    # minibatch (env JDT_FUSED_LOOP=0: generic GEMM chain)
    fused_loop: bool = field(default_factory=lambda: os.environ.get("JDT_FUSED_LOOP", "1") == "1")
    # ... with minibatch i on stream i % loop_streams (its own grad set, merged after the
    # join: parallel.fused_stage.FusedMLPStage n_sets).  0 = auto: 2 for models of >= 3
    # layers (4-layer loop 6.4k -> 7.6-7.9k steps/s), 1 for the 2-layer classifier (no
    # gain: its per-minibatch kernels already cover the chip), never 4 (the merge of 3
    # private sets costs more than it wins) -- profiles/r3_dp_loop_streams_ab.txt
    loop_streams: int = field(default_factory=lambda: int(os.environ.get("JDT_LOOP_STREAMS", "0")))


class DataParallelTrainer:
    """Owns the step program for one rank; ``step(batch_local)`` = train_step_dp."""

    def __init__(self, state: TrainState, mesh: Optional[Mesh], cfg: DPConfig = DPConfig()):
        self.state = state
        self.mesh = mesh
        self.cfg = cfg
        self.model: MLP = state.apply_fn
        P = state.params
        self.metrics = torch.zeros(N_METRIC_SLOTS, dtype=torch.float32, device=P.master.device)
        self.world = C.axis_size(mesh, cfg.axis)
        # the step issues its gradient collective (N > 1, or a Mesh(unit_groups=True))
        self._coll = self.world > 1 or C.active(mesh, cfg.axis)
        self.graph = None
        self._ahead = None
        self._static = None
        self.fused = None
        self._capturing = False
        self.buckets = None
        self._scan = None
        self._loop_engine = None
        self._loop_tried = False
        self._loop_streams = None
        self.xg = None
        self._xg_fused_opt = False
        if self.world > 1 and P.grad.is_cuda:
            from ..comm.xgmi import create_for

            # one kernel = all-reduce of [grads || metrics] + AdamW + metrics fold
            self.xg = create_for(mesh, cfg.axis, P.grad.numel(), P.grad.device, cfg.comm)
            self._xg_fused_opt = self.xg is not None and isinstance(state.tx, AdamW)
        if self._coll and cfg.overlap and self.xg is None:
            from ..comm.buckets import GradBuckets

            self.buckets = GradBuckets(P, mesh, cfg.axis, int(cfg.bucket_mb * (1 << 20)))
        from ..utils.checkpoint import bind_trainer

        bind_trainer(state, self)

    def invalidate(self):
        """Drop state derived from the parameters (fused-engine bf16 copies, captured
        graphs): called after a checkpoint restore; rebuilt on the next step."""
        self.fused = None
        self._stage = None
        self.graph = None
        self._ahead = None
        self.multi = None
        self._scan = None
        self._capturing = False
        self._loop_engine = None
        self._loop_tried = False

    def _fused_engine(self, batch: Batch):
        if self.cfg.accum != "kernel":
            return None
        if self.fused is None:
            from .fused_mlp import make_engine

            # a step with a collective keeps the optimizer out of the backward epilogue --
            # unless the tiles exchange their gradients inside the run-ahead launch (N > 1,
            # one launch per step, _tile_exchange)
            tx, share = self._tile_exchange(batch)
            self.fused = make_engine(self.state, self.mesh, self.cfg.axis, self.cfg.num_minibatches, batch.size,
                                     self.metrics, batch.inputs.device,
                                     fuse_opt=True if tx is not None else (False if self._coll else None),
                                     tx=tx, ranks_on_gpu=share)
            if self.fused is None:
                self.cfg.accum = "fused"  # shapes outside the fused kernels' envelope
                return None
            self._setup_stage()
        return self.fused

    def _tile_exchange(self, batch: Batch):
        """(TileExchange, ranks sharing this GPU) for the N > 1 step without a separate
        collective launch, or (None, 1).  2-layer engine (AdamW / plain SGD): ONE launch per
        step; deep engine (AdamW): one backward launch per hidden layer, each exchanging
        its tiles, layer 0 running ahead.  Not deterministic, every exchanging grid
        co-resident with the grids of the ranks sharing its GPU -- agreed by all ranks
        (collective: every rank builds its engine on the same step).  JDT_DP_AHEAD=0: the
        forward / backward / xGMI all-reduce step (A/B)."""
        if not (self.world > 1 and batch.inputs.is_cuda and os.environ.get("JDT_DP_AHEAD", "1") == "1"):
            return None, 1
        from ..comm import tile_exchange as TX
        from ..runtime.dist import ranks_per_gpu
        from .fused_mlp import _is_adamw, _is_plain_sgd, deterministic, supported

        from .fused_mlp import FusedMLPDeep, supported_deep

        share = ranks_per_gpu()
        dev = batch.inputs.device
        if supported(self.model, batch.size, dev):          # 2-layer: one launch per step
            from .fused_mlp import mlp2_chunk

            K, H = self.model.dims[0], self.model.dims[1]
            # the engine's own condition for an optimizer fused into the backward epilogue
            # (JDT_FUSED_SGD=0 keeps SGD out of it: three-launch step)
            fused_sgd = _is_plain_sgd(self.state.tx) and os.environ.get("JDT_FUSED_SGD", "1") == "1"
            local = (not deterministic() and (_is_adamw(self.state.tx) or fused_sgd)
                     and TX.ahead_tx_ok(batch.size, H, share, K))
            tiles = (H // 16) * (K // mlp2_chunk(K))
        elif supported_deep(self.model, batch.size, dev):   # deep: one launch per hidden layer
            # opt-in (JDT_DP_DEEP_TX=1): measured 4 % SLOWER than md_fwd / md_bwd + the xGMI
            # all-reduce on the shared GPU (profiles/r4_one_launch_dp_ab.txt; its two-ranks-
            # per-GPU variants spill registers), one rank per GPU unmeasured
            local = (os.environ.get("JDT_DP_DEEP_TX", "0") == "1" and not deterministic()
                     and _is_adamw(self.state.tx) and os.environ.get("JDT_MLP2_AHEAD", "1") == "1"
                     and bool(_lib_md_ahead_ok(batch.size)) and TX.deep_tx_ok(batch.size, share))
            tiles = FusedMLPDeep.tx_tiles(self.model.L - 1)
        else:
            local, tiles = False, 0
        if not TX.agree(self.mesh.group(self.cfg.axis), local, dev):
            return None, 1
        # fresh buffers per engine: their flags hold epochs (optimizer step + 1), which a
        # checkpoint restore (invalidate -> new engine) may move backwards
        old = getattr(self, "_txx", None)
        if old is not None:
            torch.cuda.synchronize(batch.inputs.device)
            old.close()
        self._txx = TX.create_for(self.mesh, self.cfg.axis, dev, tiles=tiles)
        return self._txx, share

    def _setup_stage(self):
        """N > 1 with the fused xGMI all-reduce + AdamW: the backward kernel writes the
        gradient bucket straight into this rank's xGMI staging buffer, so the
        collective skips its staging copy (comm/csrc/xgmi.hip, staged)."""
        self._stage = None
        if not (self._xg_fused_opt and self.fused is not None and not self.fused.fuse_opt
                and os.environ.get("JDT_XGMI_STAGED", "1") == "1"):
            return
        plan = self.xg.stage_plan(self.state.params.grad.numel())
        if plan is None:
            return
        self.xg.stage_clear()
        self.fused.set_grad_stage(plan["base"], plan["stride"])
        self._stage = plan

    # ------------------------------------------------------------------ pieces
    def compute(self, batch: Batch):
        """accum_grads: per-minibatch fwd/CE/bwd accumulated into P.grad (beta=1)."""
        st, P, cfg = self.state, self.state.params, self.cfg
        eng = self._fused_engine(batch)
        if eng is not None:
            eng.forward_backward(batch)
            return
        rng = fold_rng_over_axis(st.rng, self.mesh, cfg.axis)
        seed = rng & 0xFFFFFFFF
        n_mb = cfg.num_minibatches
        rows = batch.size
        mb = rows // n_mb
        # overlap only on the eager path (collectives are never captured into the compute graph)
        bk = self.buckets if (self.buckets is not None and not self._capturing) else None
        if bk is not None:
            bk.begin()
        loop_eng = self._fused_loop(mb, seed) if (cfg.accum == "loop" and bk is None) else None
        if loop_eng is not None:
            # the reference's minibatch loop (util.py:41-78) on the fused per-layer
            # kernels: fwd + CE/bwd per minibatch, grads accumulated into P.grad
            k = loop_eng.n_sets
            main = torch.cuda.current_stream(P.master.device) if k > 1 else None
            if k > 1:
                if self._loop_streams is None:
                    self._loop_streams = [torch.cuda.Stream(P.master.device) for _ in range(k - 1)]
                for s_ in self._loop_streams:
                    s_.wait_stream(main)
            for i in range(n_mb):
                ctx = torch.cuda.stream(self._loop_streams[i % k - 1]) if (k > 1 and i % k) else contextlib.nullcontext()
                with ctx:
                    loop_eng.forward(i, batch.inputs[i * mb:(i + 1) * mb])
                    loop_eng.backward(i, labels=batch.labels[i * mb:(i + 1) * mb])
            if k > 1:
                for s_ in self._loop_streams:
                    main.wait_stream(s_)
                loop_eng.merge()
            return
        if cfg.accum == "fused":
            loss_and_grad(self.model, P, batch.inputs, batch.labels, train=True, seed=seed, offset=0,
                          step=st.step_tensor, grad_scale=1.0 / mb, metrics=P.metrics_slot,
                          on_ready=bk.ready if bk is not None else None)
        elif cfg.accum == "scan" and P.master.is_cuda and not self._capturing:
            self._scan_minibatches(batch, seed, mb)
        else:
            for i in range(n_mb):
                last = i == n_mb - 1  # grads are final only in the last minibatch's backward
                self._minibatch(batch.inputs[i * mb:(i + 1) * mb], batch.labels[i * mb:(i + 1) * mb], i, seed, mb,
                                on_ready=bk.ready if (bk is not None and last) else None)

    def _loop_sets(self) -> int:
        from .pipeline import hw_queues

        k = int(self.cfg.loop_streams)
        return min(k if k > 0 else (2 if self.model.L >= 3 else 1), hw_queues())

    def _fused_loop(self, mb: int, seed: int):
        """FusedMLPStage over this rank's minibatches (one stage = the whole model):
        minibatch i, layer l draws dropout stream (i << 32) + (l << 1) at counter high
        word step * n_mb -- exactly the generic loop's (_minibatch) masks."""
        if not self._loop_tried:
            self._loop_tried = True
            from .fused_stage import FusedMLPStage, stage_supported

            dev = self.state.params.master.device
            if self.cfg.fused_loop and stage_supported(self.model, mb, dev):
                # the real step counter (the kernels' parity buffers follow it), scaled by
                # n_mb for the dropout counter
                self._loop_engine = FusedMLPStage(self.model, self.state.params, self.cfg.num_minibatches, mb,
                                                  self.state.step_tensor, seed, mb_shift=32,
                                                  step_mul=self.cfg.num_minibatches,
                                                  n_sets=min(self._loop_sets(), self.cfg.num_minibatches))
        return self._loop_engine

    # ------------------------------------------------------------------ accumulation
    # Minibatch i's dropout stream is (seed, counter-hi = (step * n_mb + i) << 32): the
    # index enters through a DEVICE int (mb_step), not a captured constant, so the
    # rolled "scan" variant -- one captured minibatch step replayed n times -- draws
    # the same masks as the unrolled loop (util.py:81-137 vs 41-78: the
    # reference's scan indexes its per-minibatch rngs with the traced loop index).
    def _mb_tensors(self):
        if getattr(self, "_mbt", None) is None:
            dev = self.state.params.master.device
            self._mbt = (torch.zeros(1, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
        return self._mbt

    def _minibatch(self, x, y, i, seed: int, mb: int, on_ready=None, mb_idx: Optional[torch.Tensor] = None):
        st, P = self.state, self.state.params
        idx, mstep = self._mb_tensors()
        n_mb = self.cfg.num_minibatches
        if mb_idx is None:
            # unrolled loop: mstep = step * n_mb once per step (device op: captured,
            # replay-safe); the minibatch index is the dropout counter's constant
            # high-word addend, offset = i << 32 -- the same stream as below with one
            # launch per step instead of three per minibatch (each ~4.5 us in a graph)
            if i == 0:
                torch.mul(st.step_tensor, n_mb, out=mstep)
            off = int(i) << 32
        else:
            # scan: one captured minibatch replayed with a device index
            torch.mul(st.step_tensor, n_mb, out=mstep)
            mstep.add_(mb_idx)
            off = 0
        loss_and_grad(self.model, P, x, y, train=True, seed=seed, offset=off, step=mstep, grad_scale=1.0 / mb,
                      metrics=P.metrics_slot, on_ready=on_ready)

    def _scan_minibatches(self, batch: Batch, seed: int, mb: int):
        """accum_grads_scan on the device: ONE minibatch step captured as a hipGraph
        (input slots + the device minibatch index), replayed num_minibatches times."""
        n_mb = self.cfg.num_minibatches
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr(), seed, mb)
        if self._scan is None or self._scan[0] != key:
            xin = torch.empty((mb,) + tuple(batch.inputs.shape[1:]), dtype=batch.inputs.dtype,
                              device=batch.inputs.device)
            yin = torch.empty((mb,), dtype=batch.labels.dtype, device=batch.labels.device)
            # warm the minibatch program once eagerly on minibatch 0 (allocations), then capture it
            xin.copy_(batch.inputs[0:mb])
            yin.copy_(batch.labels[0:mb])
            self._mb_tensors()[0].fill_(0)
            self._minibatch(xin, yin, 0, seed, mb, mb_idx=self._mbt[0])
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._minibatch(xin, yin, 0, seed, mb, mb_idx=self._mbt[0])
            self._scan = (key, g, xin, yin)
            start = 1
        else:
            start = 0
        _, g, xin, yin = self._scan
        idx = self._mbt[0]
        for i in range(start, n_mb):
            xin.copy_(batch.inputs[i * mb:(i + 1) * mb])
            yin.copy_(batch.labels[i * mb:(i + 1) * mb])
            idx.fill_(i)
            g.replay()

    @property
    def one_launch(self) -> bool:
        """N > 1 step as one run-ahead launch with the in-kernel tile exchange."""
        return getattr(self.fused, "tx", None) is not None

    def sync(self):
        """pmean(grads) + psum(metrics) as SUM all-reduce(s) of the flat bucket(s); the
        1/N of the mean is applied by the optimizer."""
        P = self.state.params
        if not self._coll or self.one_launch:   # one-launch step: summed inside the backward launch
            return
        with named_scope("sync_grads"):
            if self.xg is not None:
                if self._xg_fused_opt and getattr(self, "_stage", None) is not None:
                    tx, st = self.state.tx, self.state.opt_state
                    self.xg.all_reduce_adamw_staged_(
                        self._stage, p=P.master, m=st["m"], v=st["v"], shadow=P.shadow, n_params=P.numel,
                        running=self.metrics, n_metrics=N_METRIC_SLOTS, lr=tx.learning_rate, b1=tx.b1, b2=tx.b2,
                        eps=tx.eps, wd=tx.weight_decay, grad_scale=1.0 / (self.cfg.num_minibatches * self.world),
                        step=st["count"], ticket=st["ticket"])
                elif self._xg_fused_opt:
                    tx, st = self.state.tx, self.state.opt_state
                    self.xg.all_reduce_adamw_(
                        P.grad, p=P.master, m=st["m"], v=st["v"], shadow=P.shadow, n_params=P.numel,
                        running=self.metrics, n_metrics=N_METRIC_SLOTS, lr=tx.learning_rate, b1=tx.b1, b2=tx.b2,
                        eps=tx.eps, wd=tx.weight_decay, grad_scale=1.0 / (self.cfg.num_minibatches * self.world),
                        step=st["count"], ticket=st["ticket"], zero_grad=True)
                else:
                    self.xg.all_reduce_(P.grad)
            elif self.buckets is not None and self.fused is None and not self._capturing:
                self.buckets.finish()
            else:
                C.psum_(P.grad, self.mesh, self.cfg.axis)

    def update(self):
        self.update_noncounting()
        self.state.step += 1

    def step(self, batch: Batch):
        if self.graph is not None:
            check_static_batch(self._static, batch)
            self._replay()
            return
        self.compute(batch)
        self.sync()
        self.update()

    def set_batch(self, batch: Batch):
        """New data for captured graphs: copied into the captured batch tensors (the
        run-ahead schedule's next forward, computed from the old contents, is redone)."""
        if self._static is None:
            return
        load_static_batch(self._static, batch, (self.fused,))

    # ------------------------------------------------------------------ hipGraph
    def capture(self, batch: Batch, capture_collectives: bool = False, steps_per_graph: int = 1):
        """Capture the step into hipGraph(s).  Replays then skip all host work.
        The batch tensors must stay alive and fixed (the reference also reuses
        one synthetic batch every step, data_paral.py:271-273).

        ``steps_per_graph`` > 1 (single graph mode) records that many complete,
        sequential training steps into one graph -- each with its own forward,
        backward and optimizer update (the device step counter advances inside
        the graph, so dropout masks differ per step) -- so one hipGraphLaunch
        (~10-30 us of host time) is amortised over several ~20 us steps.
        ``run_steps`` uses it; ``step`` replays the 1-step graph."""
        assert batch.inputs.is_cuda
        from ..runtime.dist import collectives_capturable

        self._static = batch
        self._capturing = True  # from now on the step's collectives are whole-buffer (no per-bucket overlap)
        # the collective inside the step graph: xGMI collectives are kernels, RCCL enqueues
        # on the capturing stream (reference: the whole step under one jit,
        # data_paral.py:241-251); only a gloo group runs it on the host between graphs
        one_graph = (not self._coll or capture_collectives or self.xg is not None or collectives_capturable())
        if one_graph:
            def body():
                self.compute(batch)
                self.sync()
                self.update_noncounting()

            g = capture_graph(body)
            if g is None:   # the collective refused capture: compute / RCCL eager / update graphs
                self._capture_split(batch)
                return
            self.graph = ("one", g)
            self.multi = None
            self._ahead = None
            # single GPU, whole-step fused engine: the S steps are ONE persistent launch
            # (opt-in mlp2_loop_kernel, grid barriers instead of kernel boundaries) or,
            # by default, one run-ahead launch per step (step t's backward + AdamW +
            # step t+1's forward).  Run-ahead graphs come in two variants: "cold" starts
            # with step t's forward, "primed" does not -- after a run-ahead launch the
            # forward of the next step is already done (FusedMLP2.ahead_primed).
            loop = self.world == 1 and getattr(self.fused, "loop_ok", False)
            ahead = (self.world == 1 or self.one_launch) and not loop and getattr(self.fused, "ahead_ok", False)
            if ahead:
                from .fused_mlp import AheadGraphs

                self._ahead = AheadGraphs(self.fused, batch, steps_per_graph, pool=g.pool())
                if steps_per_graph > 1:
                    self.multi = (steps_per_graph, self._ahead.graph(steps_per_graph))
            elif steps_per_graph > 1:
                gm = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gm, pool=g.pool()):
                    if not (loop and self.fused.run_loop(batch, steps_per_graph)):
                        for _ in range(steps_per_graph):
                            body()
                self.multi = (steps_per_graph, gm)
        else:
            self._capture_split(batch)

    def _capture_split(self, batch: Batch):
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            self.compute(batch)
        with torch.cuda.graph(g2):
            self.update_noncounting()
        self.graph = ("split", g1, g2)
        self.multi = None
        self._ahead = None

    def update_noncounting(self):
        P = self.state.params
        if self._xg_fused_opt or self.one_launch:
            return  # AdamW + metrics fold ran inside the xGMI all-reduce kernel (sync)
        if self.fused is not None:
            if self.fused.fuse_opt:
                return  # AdamW + metrics already applied inside mlp2_bwd
            self.state.tx.update(P, self.state.opt_state, 1.0 / (self.cfg.num_minibatches * self.world),
                                 zero_grad=False)
        else:
            self.state.tx.update(P, self.state.opt_state, 1.0 / (self.cfg.num_minibatches * self.world))
        with named_scope("sync_metrics"):
            K.metrics_fold_(self.metrics, P.metrics_slot)

    @property
    def xgmi_status(self) -> str:
        from ..comm.xgmi import status

        return status(self.xg, self.world, self.state.params.master.device, self.cfg.comm)

    def time_collective(self, batch: Batch, iters: int = 20) -> Optional[float]:
        """Median device time (ms) of the step's gradient collective -- ``sync``: the
        bucket all-reduce (xGMI: with the fused AdamW + metrics fold) -- bracketed by
        hipEvents in separate, untimed eager steps (complete training steps: they
        advance the state like any other).  None for N = 1 or off-GPU."""
        if not self._coll or not self.state.params.master.is_cuda or self.one_launch:
            return None   # (one-launch step: the exchange is inside the backward launch)
        ts = []
        for _ in range(iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            self.compute(batch)
            a.record()
            self.sync()
            b.record()
            self.update_noncounting()
            self.state.step += 1
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return round(ts[len(ts) // 2], 5)

    def finalize(self):
        if self.fused is not None:
            self.fused.finalize()
        if self.xg is not None:
            self.xg.raise_if_error()

    def close(self):
        """Release the IPC-mapped exchange buffers (tile exchange inboxes, xGMI context)
        and the captured graphs, so another trainer can be built in this process
        (bench.py's probes).  Collective (runtime.dist.quiesce: no rank frees buffers a
        peer's kernel may still write); the trainer is unusable afterwards."""
        from ..runtime.dist import quiesce

        quiesce(self.state.params.master.device)
        for r in (getattr(self, "_txx", None), self.xg):
            if r is not None:
                r.close()
        self._txx = self.xg = None
        self.invalidate()

    @property
    def comm_backend(self) -> str:
        if not self._coll:
            return "none"
        if self.xg is not None:
            return "xgmi"
        from ..runtime.dist import backend

        b = backend()
        return "rccl" if b == "nccl" else (b or "none")

    def run_steps(self, batch: Batch, n: int):
        """n training steps; with a multi-step graph, n // S replays of it plus
        single-step replays for the remainder."""
        multi = getattr(self, "multi", None)
        if self.graph is not None:
            check_static_batch(self._static, batch)
        if self.graph is not None and multi is not None:
            S, gm = multi
            for _ in range(n // S):
                with replay_scope("train_step_dp", S):
                    self._ahead.replay(S) if self._ahead else gm.replay()
            self.state.step += (n // S) * S
            n = n % S
        for _ in range(n):
            self.step(batch)

    def _replay(self):
        kind = self.graph[0]
        if kind == "one" and getattr(self, "_ahead", None):
            with replay_scope("train_step_dp"):
                self._ahead.replay(1)
        elif kind == "one":
            with replay_scope("train_step_dp"):
                self.graph[1].replay()
        else:
            self.graph[1].replay()
            self.sync()
            self.graph[2].replay()
        self.state.step += 1


def _lib_md_ahead_ok(rows: int) -> int:
    from ..ops import _lib

    return _lib.lib().jdt_md_ahead_ok(int(rows))


def capture_graph(body, pool=None) -> Optional[torch.cuda.CUDAGraph]:
    """``body`` recorded into a hipGraph, or None if a collective in it refused stream
    capture (the caller then keeps that collective eager).  RCCL collectives enqueue
    on the capturing stream and are recorded like kernels."""
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, pool=pool):
            body()
    except RuntimeError as e:
        import logging

        logging.getLogger(__name__).warning("step capture with the collective inside failed (%s); "
                                            "running the collective eagerly between graphs", e)
        torch.cuda.synchronize()
        return None
    return g


def train_step_dp(trainer: DataParallelTrainer, batch: Batch):
    """Functional-style alias of the reference's step (data_paral.py:193-238)."""
    trainer.step(batch)
    return trainer.state, trainer.metrics
