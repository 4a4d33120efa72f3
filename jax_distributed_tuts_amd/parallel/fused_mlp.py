"""Fused whole-step engine for the tutorial classifier (csrc/mlp_fused.hip).

One DP step = ``mlp2_fwd`` + ``mlp2_bwd`` (+ RCCL all-reduce + fused AdamW when
N > 1).  On one GPU the optimizer runs inside ``mlp2_bwd``'s epilogue, so a
step is two kernel launches -- or, in captured multi-step graphs, ONE: the
run-ahead ``mlp2_bwd`` (``run_ahead`` / ``AheadGraphs``) also computes the next
step's forward from the W1 tiles its AdamW epilogue just produced.  Mathematically identical to the reference's
4-minibatch accumulation loop: each row's loss is weighted 1/(rows per
minibatch) and the summed gradient is scaled by 1/n_minibatches (and 1/N after
the SUM all-reduce); dropout draws one Philox stream per (step, row, unit).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_longlong, c_ulonglong, c_void_p
from typing import Optional

import torch

from ..comm import collectives as C
from ..ops import _lib
from ..ops import kernels as K
from ..utils.profiling import named_scope


class Mlp2Args(ctypes.Structure):
    _fields_ = [("M", c_int), ("H", c_int), ("inv_mb", c_float), ("X", c_void_p), ("labels", c_void_p),
                ("W1s", c_void_p), ("b1s", c_void_p), ("W2s0", c_void_p), ("W2s1", c_void_p), ("b2s", c_void_p),
                ("G1", c_void_p), ("H1", c_void_p), ("logits", c_void_p),
                ("keep", c_float), ("seed", c_ulonglong), ("offset", c_ulonglong),
                ("step", c_void_p), ("ticket", c_void_p),
                ("gW1", c_void_p), ("gb1", c_void_p), ("gW2", c_void_p), ("gb2", c_void_p), ("mslot", c_void_p),
                ("fuse_opt", c_int),
                ("pW1", c_void_p), ("pb1", c_void_p), ("pW2", c_void_p), ("pb2", c_void_p),
                ("mW1", c_void_p), ("mb1", c_void_p), ("mW2", c_void_p), ("mb2", c_void_p),
                ("vW1", c_void_p), ("vb1", c_void_p), ("vW2", c_void_p), ("vb2", c_void_p),
                ("sW1", c_void_p), ("sb1", c_void_p), ("sW2_0", c_void_p), ("sW2_1", c_void_p), ("sb2", c_void_p),
                ("lr", c_float), ("beta1", c_float), ("beta2", c_float), ("eps", c_float), ("wd", c_float),
                ("gscale", c_float), ("running", c_void_p), ("stamps", c_void_p),
                ("W1T", c_void_p), ("ldw1t", c_int), ("XT", c_void_p), ("ldxt", c_int),
                ("step_copy", c_void_p), ("W2snap", c_void_p), ("stage_stride", ctypes.c_long),
                ("det_logits", c_void_p),
                ("XR", c_void_p), ("zslab", c_void_p), ("ztick", c_void_p), ("hand", c_void_p), ("lg3", c_int),
                ("opt_sgd", c_int), ("smap", c_void_p), ("wt", c_int), ("tx", c_void_p), ("tx_fsdp", c_int)]


class StageLeaf(ctypes.Structure):
    """Mirror of ``jdt::StageLeaf`` (ops/csrc/common.h)."""

    _fields_ = [("off", ctypes.c_long), ("dim", c_int), ("per", c_int), ("cols", c_int), ("pad", c_int)]


class StageMap(ctypes.Structure):
    """Mirror of ``jdt::StageMap``: where a mode-0 producer writes each gradient element
    of its leaves (W, b, head W, head b, metrics) in the fused FSDP collective's packed
    staging layout (comm/csrc/xgmi.hip xg_fsdp_kernel, staged)."""

    _fields_ = [("base", c_void_p), ("half", ctypes.c_long), ("slice", ctypes.c_long), ("W", c_int),
                ("nleaf", c_int), ("leaf", StageLeaf * 5)]


_lib.declare("jdt_stage_map_size", c_int, [])


def stage_map_tensor(base: int, half: int, slice_: int, world: int, leaves, device) -> torch.Tensor:
    """A device copy of a StageMap; ``leaves`` = 5 (off, dim, per, cols) tuples (None =
    unused slot).  The engines pass its address as ``smap``."""
    if _lib.lib().jdt_stage_map_size() != ctypes.sizeof(StageMap):
        raise RuntimeError("StageMap layout mismatch")
    m = StageMap()
    m.base, m.half, m.slice, m.W, m.nleaf = base, half, slice_, world, 5
    for k, lf in enumerate(leaves):
        if lf is not None:
            m.leaf[k] = StageLeaf(int(lf[0]), int(lf[1]), int(lf[2]), int(lf[3]), 0)
    raw = torch.frombuffer(bytearray(bytes(m)), dtype=torch.uint8)
    return raw.to(device)


_lib.declare("jdt_mlp2", c_int, [ctypes.POINTER(Mlp2Args), c_int, c_int, c_int, c_void_p])
_lib.declare("jdt_mlp2_set_p3s", None, [c_int])
_lib.declare("jdt_mlp2_args_size", c_int, [])
_lib.declare("jdt_mlp2_ahead_ok", c_int, [c_int, c_int, c_int])
_lib.declare("jdt_mlp2_chunk", c_int, [c_int])
_lib.declare("jdt_mlp2_set_rows", None, [c_int])
_lib.declare("jdt_mlp2_loop", c_int, [ctypes.POINTER(Mlp2Args), c_int, c_void_p, c_void_p, c_void_p, ctypes.c_longlong,
                                      c_void_p, c_void_p])

_lib.declare("jdt_mlp2_loop_ok", c_int, [c_int, c_int])
_lib.declare("jdt_mlp2_pst_ok", c_int, [c_int, c_int, c_int])
_lib.declare("jdt_mlp2_pst_tx_ok", c_int, [c_int, c_int, c_int, c_int, c_int])
_lib.declare("jdt_mlp2_pst_set_share", None, [c_int])
_lib.declare("jdt_mlp2_pst_set_cbw", None, [c_int])
_lib.declare("jdt_mlp2_pst", c_int, [ctypes.POINTER(Mlp2Args), c_int, c_int, c_void_p, c_longlong, c_void_p])
PST_BARRIER_TIMEOUT_S = 0.02   # persistent run-ahead grid barrier bound (x runtime.dist.spin_timeout_s sharing)

LOOP_BARRIER_TIMEOUT_TICKS = 20_000_000   # 0.2 s of s_memrealtime (100 MHz) per grid barrier


def deterministic() -> bool:
    """JDT_DETERMINISTIC=1 (entry scripts' --deterministic): fixed-order reductions."""
    return os.environ.get("JDT_DETERMINISTIC", "0") == "1"


def _is_adamw(tx) -> bool:
    from ..utils.train_state import AdamW

    return isinstance(tx, AdamW)


def _is_plain_sgd(tx) -> bool:
    """SGD without momentum: the 2-layer engine fuses it into its backward epilogue."""
    from ..utils.train_state import SGD

    return isinstance(tx, SGD) and not tx.momentum


def set_forward_rows(rb: int):
    """mlp2_fwd rows per workgroup: 16 (default, 256 workgroups at 128 rows) or 32
    (A/B comparisons; env ``JDT_MLP2_RB`` sets it at engine construction)."""
    _lib.lib().jdt_mlp2_set_rows(int(rb))


def mlp2_chunk(k_in: int) -> int:
    """Input rows of W1 per backward workgroup (csrc/mlp_fused.hip mlp2_kc): 112 for the
    tutorial's 784 inputs, 64 for 1024; 0 for a width the kernels are not built for."""
    return int(_lib.lib().jdt_mlp2_chunk(int(k_in)))


def supported(model, rows: int, device) -> bool:
    """The 2-layer fused engine's envelope: K_IN in the instantiated widths (784, 1024),
    10 classes, hidden a multiple of 16 with one hidden block per input chunk (the
    forward writes X^T chunk y from hidden block y), <= 128 rows, SiLU."""
    from ..models.mlp import MLP

    if not (torch.device(device).type == "cuda" and isinstance(model, MLP) and model.L == 2):
        return False
    k, h = model.dims[0], model.dims[1]
    kc = mlp2_chunk(k)
    return (kc > 0 and model.dims[2] == 10 and h % 16 == 0 and h // 16 >= k // kc and 0 < rows <= 128
            and model.act == "silu" and not model.final_act)


class FusedMLP2:
    """``params`` (default ``state.params``) supplies the bf16 shadow the kernels read
    and the fp32 grad views mode 0 writes -- FSDP passes its gathered full buffer
    (grads then reduce-scattered), with ``mslot`` its local metric slots."""

    def __init__(self, state, mesh, axis: str, num_minibatches: int, rows: int, metrics: torch.Tensor,
                 params=None, mslot: Optional[torch.Tensor] = None, fuse_opt: Optional[bool] = None,
                 tx=None, ranks_on_gpu: int = 1, opt_params=None):
        """``tx`` (comm.tile_exchange.TileExchange, N > 1): every step is ONE run-ahead
        launch whose tiles all-reduce their gradients with the other ranks' launches
        before the fused optimizer (``ranks_on_gpu``: ranks sharing this GPU, for the
        co-residency check).  ``opt_params`` (FSDP, with ``tx``): the rank's LOCAL shard
        buffer holding the fp32 masters the sharded AdamW updates (``params`` is then the
        gathered full buffer whose bf16 shadow the kernels read and write)."""
        P = params if params is not None else state.params
        self.tx = tx
        self.fsdp_tx = tx is not None and opt_params is not None
        self.OP = opt_params if opt_params is not None else P
        self.P = P
        self.mslot = mslot if mslot is not None else P.metrics_slot
        self.state, self.mesh, self.axis = state, mesh, axis
        self.world = C.axis_size(mesh, axis)
        self.n_mb = num_minibatches
        self.model = state.apply_fn
        H = self.model.dims[1]
        dev = P.master.device
        self.rows = rows
        # input width and its backward chunk (csrc/mlp_fused.hip is instantiated for 784 / 1024)
        self.K = K = self.model.dims[0]
        self.kc = mlp2_chunk(K)
        self.nch = K // self.kc
        # silu'(Z1) * mask / keep in 4-row groups ([Mp/4][H][4] fp32), mlp2_fwd -> mlp2_bwd
        self.G1 = torch.zeros((rows + 31) // 32 * 32 * H, dtype=torch.float32, device=dev)
        # H = dropout(silu(Z1)) bf16, same 4-row group layout as G1
        self.H1 = torch.zeros((rows + 31) // 32 * 32 * H, dtype=torch.bfloat16, device=dev)
        # logits accumulators: [0:2] by step parity (two launches per step), [2:5] by
        # step % 3 (run-ahead steps); run_ahead zeroes all five first
        self.logits_all = torch.zeros(5, rows, 10, dtype=torch.float32, device=dev)
        self.logits = self.logits_all[:2]
        self.step_copy = torch.zeros(1, dtype=torch.int32, device=dev)  # mlp2_fwd -> mlp2_bwd
        # second parity buffer of W2's bf16 shadow (single-GPU fused-optimizer mode)
        self.W2s1 = P.s("output_dense/kernel").clone()
        self.metrics = metrics
        if fuse_opt is None:
            fuse_opt = self.world == 1 and os.environ.get("JDT_FUSED_OPT", "1") == "1"
        # mode 1 fuses AdamW (or momentum-free SGD) into the backward epilogue; any other
        # optimizer runs mode 0 (plain-stored grads) + its own kernel
        # (JDT_FUSED_SGD=0: SGD through mode 0 + the standalone SGD kernel, for A/B)
        self.opt_sgd = _is_plain_sgd(state.tx) and os.environ.get("JDT_FUSED_SGD", "1") == "1"
        self.fuse_opt = (bool(fuse_opt) and (params is None or self.fsdp_tx)
                         and (_is_adamw(state.tx) or (self.opt_sgd and not self.fsdp_tx)))
        # K-contiguous bf16 operand copies (zero K padding): X^T written by mlp2_fwd for
        # mlp2_bwd; W1^T written by mlp2_bwd's AdamW epilogue for the next mlp2_fwd
        self.Mp = (rows + 31) // 32 * 32
        self.XT = torch.zeros(K, self.Mp, dtype=torch.bfloat16, device=dev)  # sample tail stays zero
        if os.environ.get("JDT_MLP2_RB"):
            set_forward_rows(int(os.environ["JDT_MLP2_RB"]))
        self.W1T = None
        if self.fuse_opt:
            self.ldw1t = (K + 31) // 32 * 32   # K padded to whole 32-deep MFMA steps (zero tail)
            self.W1T = torch.zeros(H, self.ldw1t, dtype=torch.bfloat16, device=dev)
            self.W1T[:, :K].copy_(P.s("input_dense/kernel").t())
        # persistent n-step kernel (mlp2_loop_kernel): W2 snapshot + barrier words
        # [arrival counter, its base at the next launch, error flag, pad]
        self.W2snap = torch.zeros(H * 10, dtype=torch.float32, device=dev)
        self.loop_ws = torch.zeros(4, dtype=torch.int32, device=dev)
        # Opt-in (JDT_MLP2_LOOP=1): measured SLOWER than two launches per step on MI355X
        # (29.3 vs 16.3 us/step, tools/stamp_loop.py: each 256-workgroup grid barrier
        # costs ~8 us against a 2.4 us kernel boundary), kept as the tested reference
        # design for in-launch sc1 hand-offs.
        self.loop_ok = (self.fuse_opt and K == 784 and os.environ.get("JDT_MLP2_LOOP", "0") == "1"
                        and bool(_lib.lib().jdt_mlp2_loop_ok(rows, H)))
        if _lib.lib().jdt_mlp2_args_size() != ctypes.sizeof(Mlp2Args):
            raise RuntimeError("Mlp2Args layout mismatch")
        if os.environ.get("JDT_MLP2_P3S"):   # A/B: the one-GPU run-ahead with the N > 1 phase-3 order
            _lib.lib().jdt_mlp2_set_p3s(int(os.environ["JDT_MLP2_P3S"]))
        self._args = None
        self._key = None
        self.grad_stage = None   # (staging base pointer, half stride in floats): set_grad_stage
        # deterministic mode: per-column-block partial logits instead of fp32 atomics, summed
        # in block order (one set per step % 3 for the run-ahead / persistent step, which
        # then runs in this mode too: the benchmarked kernel, bitwise reproducible)
        self.det_logits = (torch.zeros(3, H // 16, rows, 10, dtype=torch.float32, device=dev)
                           if deterministic() else None)
        # run-ahead steps (one launch per step: step t's backward + AdamW + step t+1's
        # forward, csrc/mlp_fused.hip mlp2_bwd AHEAD); single GPU, fused AdamW only.
        # JDT_MLP2_AHEAD=0 turns it off (A/B)
        self.ahead_ok = (self.fuse_opt and self.W1T is not None
                         and os.environ.get("JDT_MLP2_AHEAD", "1") == "1"
                         and bool(_lib.lib().jdt_mlp2_ahead_ok(rows, H, K)))
        if tx is not None:
            from ..comm.tile_exchange import ahead_tx_ok

            self.ahead_ok = self.fuse_opt and self.W1T is not None and ahead_tx_ok(rows, H, ranks_on_gpu, K)
        self._ahead_args = None
        # host-side: the last launch on this engine was a run-ahead backward (set by
        # run_ahead / DataParallelTrainer after replaying a run-ahead graph)
        self.ahead_primed = False
        if self.ahead_ok:
            nch = self.nch
            self.XR = torch.zeros(rows, K, dtype=torch.bfloat16, device=dev)
            self.zslab = torch.zeros(H // 16 * nch * 128 * 16, dtype=torch.float32, device=dev)
            # 128-byte lines: [step ticket, error word (1: tile map, 2: barrier timeout),
            # launch counter], one column-barrier counter line per hidden block, one
            # per-tile launch counter line per XCD (csrc/mlp_fused.hip Mlp2Args.ztick)
            tpx = H // 16 * nch // 8
            self.ztick = torch.zeros(32 * (1 + H // 16) + 8 * 32 * ((tpx + 31) // 32), dtype=torch.int32, device=dev)
            self.hand = torch.zeros(H + H * 10 + 10, dtype=torch.float32, device=dev)
        # persistent run-ahead (csrc/mlp_fused.hip mlp2_pst_kernel): n >= 2 steps of a
        # run-ahead call in ONE launch, the AdamW state in registers across them and an
        # XCD-hierarchical grid barrier between steps; one GPU only.  JDT_MLP2_PST=0: one
        # launch per step (A/B).  pst_ws: the barrier's counter lines, zeroed once.
        # N > 1 (one-launch step, ``tx``): the same persistent launch with the tile
        # exchange inside every step (mlp2_pst_kernel TX; FSDP: the owner exchange FX, the
        # owned shard's AdamW state in registers), so a replay's n steps are one launch per
        # rank; JDT_DP_PST=0 / JDT_FSDP_PST=0 keep one run-ahead launch per step (bench.py's
        # autotune validates and times both).
        if tx is None:
            self.pst_ok = (self.ahead_ok and os.environ.get("JDT_MLP2_PST", "1") == "1"
                           and bool(_lib.lib().jdt_mlp2_pst_ok(rows, H, K)))
        else:
            env = "JDT_FSDP_PST" if self.fsdp_tx else "JDT_DP_PST"
            self.pst_ok = (self.ahead_ok and os.environ.get(env, "1") == "1"
                           and bool(_lib.lib().jdt_mlp2_pst_tx_ok(rows, H, K, int(ranks_on_gpu), int(self.fsdp_tx))))
            if self.pst_ok:
                _lib.lib().jdt_mlp2_pst_set_share(int(ranks_on_gpu))
        if self.pst_ok:
            from ..runtime.dist import spin_timeout_s

            # [generation, CBW base] line, barrier counter lines, then one completion-counter
            # line per column block (CBW, csrc/mlp_fused.hip cb_wait)
            self.pst_ws = torch.zeros(32 * (18 + 64), dtype=torch.int32, device=dev)
            # between-step synchronisation: JDT_MLP2_PST_SYNC=barrier (XCD-hierarchical grid
            # barrier) or colblk (column-block completion counters), one GPU only
            _lib.lib().jdt_mlp2_pst_set_cbw(int(tx is None and os.environ.get("JDT_MLP2_PST_SYNC", "barrier") == "colblk"))
            # s_memrealtime ticks (100 MHz); grows with the ranks sharing the GPU like the
            # other in-kernel waits
            self.pst_timeout = int(spin_timeout_s(PST_BARRIER_TIMEOUT_S) * 1e8)
            if tx is not None:
                # N > 1: a workgroup reaches the grid barrier only after its tile's exchange,
                # which waits for the peers' launches (not started in lockstep): the barrier
                # gets the exchange's bound
                self.pst_timeout = max(self.pst_timeout, int(tx.timeout_s * 1e8))
        self._pst_warm = False

    def set_grad_stage(self, base: int, stride: int):
        """Mode 0: write the gradient bucket into the xGMI staging buffer at ``base``
        (+ (step & 1) * ``stride`` floats) instead of P.grad (comm/xgmi.py staged)."""
        assert not self.fuse_opt
        self.grad_stage = (int(base), int(stride))
        self._args = None

    def set_fsdp_stage(self, layout: dict, base: int, half: int, slice_: int, world: int):
        """Mode 0, FSDP N > 1: write the gradients and metric slots straight into the
        fused FSDP collective's staging buffer (``layout``: leaf name -> (packed offset,
        dim, per, cols), "metrics" included; XgmiComm.fsdp_stage_layout)."""
        assert not self.fuse_opt
        names = ["input_dense/kernel", "input_dense/bias", "output_dense/kernel", "output_dense/bias", "metrics"]
        self.smap_t = stage_map_tensor(base, half, slice_, world, [layout[n] for n in names], self.P.master.device)
        self._args = None

    def _build_args(self, batch) -> Mlp2Args:
        st, P = self.state, self.P
        o = st.opt_state
        a = Mlp2Args()
        a.M, a.H = self.rows, self.model.dims[1]
        mb = self.rows // self.n_mb
        a.inv_mb = 1.0 / mb
        a.X, a.labels = batch.inputs.data_ptr(), batch.labels.data_ptr()
        a.W1s, a.b1s = P.s("input_dense/kernel").data_ptr(), P.s("input_dense/bias").data_ptr()
        a.W2s0 = P.s("output_dense/kernel").data_ptr()
        a.W2s1 = self.W2s1.data_ptr() if self.fuse_opt else a.W2s0
        a.b2s = P.s("output_dense/bias").data_ptr()
        a.G1, a.H1, a.logits = self.G1.data_ptr(), self.H1.data_ptr(), self.logits.data_ptr()
        a.keep = 1.0 - self.model.dropout_rate
        from ..utils import rng as R

        a.seed = R.fold_rng_over_axis(st.rng, self.mesh, self.axis) & 0xFFFFFFFF
        a.offset = 0
        a.step, a.ticket = o["count"].data_ptr(), o["ticket"].data_ptr()
        names = ["input_dense/kernel", "input_dense/bias", "output_dense/kernel", "output_dense/bias"]
        a.gW1, a.gb1, a.gW2, a.gb2 = (P.g(n).data_ptr() for n in names)
        a.mslot = self.mslot.data_ptr()
        if self.grad_stage is not None:
            # N > 1: the bucket is written straight into the xGMI staging buffer (same
            # flat layout as P.grad, half selected in-kernel by the step parity)
            base, stride = self.grad_stage
            a.gW1, a.gb1, a.gW2, a.gb2 = (base + 4 * P.offsets[n][0] for n in names)
            a.mslot = base + 4 * P.metric_off
            a.stage_stride = stride
        if getattr(self, "smap_t", None) is not None:
            a.smap = self.smap_t.data_ptr()
        a.fuse_opt = int(self.fuse_opt)
        # run-ahead: the W1 AdamW state and W1^T stored write-through (+1.0 % steps/s,
        # profiles/r4_write_through_ab.txt; 3 = also the Z1 partials and G1: no gain)
        a.wt = int(os.environ.get("JDT_MLP2_WT", "1"))
        a.XT, a.ldxt = self.XT.data_ptr(), self.Mp
        a.step_copy = self.step_copy.data_ptr()
        a.W2snap = self.W2snap.data_ptr()
        if self.W1T is not None:
            a.W1T, a.ldw1t = self.W1T.data_ptr(), self.ldw1t
        if self.det_logits is not None:
            a.det_logits = self.det_logits.data_ptr()
        tx = st.tx
        if self.fuse_opt:
            OP = self.OP   # the optimizer's masters (FSDP one-launch: this rank's local shards)
            off = {n: OP.offsets[n][0] for n in names}
            a.pW1, a.pb1, a.pW2, a.pb2 = (OP.p(n).data_ptr() for n in names)
            a.tx_fsdp = int(self.fsdp_tx)
            if self.opt_sgd:   # no moment buffers: m / v alias p (the kernel neither uses nor writes them)
                a.mW1, a.mb1, a.mW2, a.mb2 = a.pW1, a.pb1, a.pW2, a.pb2
                a.vW1, a.vb1, a.vW2, a.vb2 = a.pW1, a.pb1, a.pW2, a.pb2
                a.opt_sgd = 1
            else:
                m, v = o["m"], o["v"]
                a.mW1, a.mb1, a.mW2, a.mb2 = (m[off[n]:].data_ptr() for n in names)
                a.vW1, a.vb1, a.vW2, a.vb2 = (v[off[n]:].data_ptr() for n in names)
            a.sW1, a.sb1 = P.s(names[0]).data_ptr(), P.s(names[1]).data_ptr()
            a.sW2_0, a.sW2_1 = P.s(names[2]).data_ptr(), self.W2s1.data_ptr()
            a.sb2 = P.s(names[3]).data_ptr()
            if self.opt_sgd:
                a.lr, a.beta1, a.beta2, a.eps, a.wd = tx.learning_rate, 0.0, 0.0, 0.0, tx.weight_decay
            else:
                a.lr, a.beta1, a.beta2, a.eps, a.wd = tx.learning_rate, tx.b1, tx.b2, tx.eps, tx.weight_decay
            # N > 1 one-launch step: the kernel sums the ranks' gradients, 1/N in the scale
            a.gscale = 1.0 / (self.n_mb * (self.world if self.tx is not None else 1))
            a.running = self.metrics.data_ptr()
        return a

    def forward_backward(self, batch):
        if self.tx is not None:
            # N > 1 with the tile exchange: a step is a run-ahead launch (the two-launch pair
            # would apply AdamW to this rank's local gradients)
            self.run_ahead(batch, 1, prologue=not self.ahead_primed)
            return
        if not torch.cuda.is_current_stream_capturing():
            self.ahead_primed = False   # the run-ahead buffers no longer hold the next forward
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr(), self.state.rng)
        if self._args is None or self._key != key:
            self._args, self._key = self._build_args(batch), key
        L = _lib.lib()
        s = _lib.stream_ptr()
        _lib.check(L.jdt_mlp2(ctypes.byref(self._args), 0, self.K, 10, s), "mlp2_fwd")
        _lib.check(L.jdt_mlp2(ctypes.byref(self._args), 1, self.K, 10, s), "mlp2_bwd")

    def run_ahead(self, batch, n: int, prologue: bool = True):
        """n complete training steps as n run-ahead backward launches, launch i = step
        i's CE, backward and AdamW plus step i+1's forward (n >= 2 with ``pst_ok``: ONE
        persistent launch of the n steps -- equal to the per-step launches up to the
        arrival order of the logits' fp32 atomics); ``prologue`` first runs the
        first step's forward (``mlp2_fwd``), needed unless the previous launch on this
        engine was a run-ahead backward (``ahead_primed``: step t's G1, H1 and logits
        (t % 3) are then already there).  Same maths as n two-launch steps except the
        fp32 summation order of Z1 (7 input-chunk partials instead of 8 wave
        partials)."""
        assert self.ahead_ok
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr(), self.state.rng)
        if self._args is None or self._key != key:
            self._args, self._key = self._build_args(batch), key
            self._ahead_args = None
        if self._ahead_args is None:
            self._make_ahead_args()
        L = _lib.lib()
        s = _lib.stream_ptr()
        if prologue:
            self.logits_all.zero_()
            _lib.check(L.jdt_mlp2(ctypes.byref(self._ahead_args), 0, self.K, 10, s), "mlp2_fwd")
        elif not torch.cuda.is_current_stream_capturing():
            assert self.ahead_primed, "run_ahead(prologue=False) needs a run-ahead launch just before"
        if self.pst_ok and n >= 2:
            if not torch.cuda.is_current_stream_capturing():
                self.pst_warm()
            _lib.check(L.jdt_mlp2_pst(ctypes.byref(self._ahead_args), int(n), self.K, self.pst_ws.data_ptr(),
                                      self.pst_timeout, s), "mlp2_pst")
        else:
            for _ in range(n):
                _lib.check(L.jdt_mlp2(ctypes.byref(self._ahead_args), 2, self.K, 10, s), "mlp2_bwd_ahead")
        if not torch.cuda.is_current_stream_capturing():
            self.ahead_primed = True

    def _make_ahead_args(self):
        b = Mlp2Args.from_buffer_copy(self._args)
        b.logits = self.logits_all[2:].data_ptr()
        b.lg3 = 1
        b.XR, b.zslab, b.ztick, b.hand = (t.data_ptr() for t in (self.XR, self.zslab, self.ztick, self.hand))
        if self.tx is not None:
            b.tx = self.tx.args_ptr
        self._ahead_args = b

    def pst_warm(self):
        """One no-op dispatch of the persistent kernel (n = 0), once, outside any capture:
        its first-dispatch setup (private segment) lands here, not in a timed replay."""
        if self.pst_ok and not self._pst_warm and self._ahead_args is not None:
            _lib.check(_lib.lib().jdt_mlp2_pst(ctypes.byref(self._ahead_args), 0, self.K, self.pst_ws.data_ptr(),
                                               self.pst_timeout, _lib.stream_ptr()), "mlp2_pst warm")
            self._pst_warm = True

    def run_loop(self, batch, n: int, stamps: Optional[torch.Tensor] = None) -> bool:
        """n complete steps (forward, backward, AdamW) in ONE persistent launch.
        False (nothing launched) if the loop kernel is unavailable for this engine
        or its grid cannot be fully resident; the caller then runs n two-launch steps."""
        if not self.loop_ok:
            return False
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr(), self.state.rng)
        if self._args is None or self._key != key:
            self._args, self._key = self._build_args(batch), key
        w = self.loop_ws
        rc = _lib.lib().jdt_mlp2_loop(ctypes.byref(self._args), int(n), w[0:].data_ptr(), w[1:].data_ptr(),
                                      w[2:].data_ptr(), LOOP_BARRIER_TIMEOUT_TICKS,
                                      stamps.data_ptr() if stamps is not None else None, _lib.stream_ptr())
        if rc == -4:
            self.loop_ok = False
            return False
        _lib.check(rc, "mlp2_loop")
        return True

    def loop_error(self) -> bool:
        return bool(int(self.loop_ws[2].item()))

    def step(self, batch):
        self.forward_backward(batch)
        if not self.fuse_opt:
            P = self.state.params
            with named_scope("sync_grads"):
                C.psum_(P.grad, self.mesh, self.axis)
            self.state.tx.update(P, self.state.opt_state, 1.0 / (self.n_mb * self.world), zero_grad=False)
            with named_scope("sync_metrics"):
                K.metrics_fold_(self.metrics, P.metrics_slot)

    def finalize(self):
        """Bring the generic bf16 shadows up to date: W2's parity buffer in use, and
        W1's (mlp2_bwd keeps only the K-contiguous W1^T copy current)."""
        if self.loop_error():
            raise RuntimeError("mlp2_loop_kernel: a grid barrier timed out (not every workgroup was resident)")
        if self.ahead_ok and int(self.ztick[1].item()) != 0:
            if self.pst_ok and int(self.ztick[1].item()) & 8:
                # a persistent launch left its grid barrier early: the XCD / top counters
                # moved without the generation word, so every later launch would be out of
                # step -- re-zero them (the engine stays unusable until the error is cleared)
                self.pst_ws.zero_()
            raise RuntimeError("mlp2_bwd run-ahead: tile map, column barrier or tile exchange failed (error "
                               f"word {int(self.ztick[1].item())}: 1 tile map, 2 column barrier, 4 exchange "
                               "timeout, 8 persistent grid barrier); results invalid")
        P = self.P   # the buffer whose bf16 shadow the kernels read (FSDP: the gathered full one)
        if self.fuse_opt and int(self.state.opt_state["count"].item()) % 2 == 1:
            P.s("output_dense/kernel").copy_(self.W2s1)
        if self.W1T is not None:
            P.s("input_dense/kernel").copy_(self.W1T[:, :self.K].t())


class AheadGraphs:
    """hipGraphs of run-ahead steps for a single-GPU FusedMLP2 engine (DP and FSDP at
    N = 1): for S in {1, steps_per_graph}, a "cold" graph (step t's forward first)
    and a "primed" one (no forward: the previous replay's last launch already ran
    it).  ``replay(S)`` picks the variant from the engine's host-side state."""

    def __init__(self, eng: "FusedMLP2", batch, steps_per_graph: int, pool=None):
        self.eng = eng
        self._checked = False
        self.graphs = {}
        if int(steps_per_graph) >= 2 and getattr(eng, "pst_ok", False):
            if eng._ahead_args is None:   # the arguments are built by the first run-ahead call
                eng._args, eng._key = eng._build_args(batch), (batch.inputs.data_ptr(), batch.labels.data_ptr(),
                                                              eng.state.rng)
                eng._ahead_args = None
                eng._make_ahead_args()
            eng.pst_warm()
        for S in sorted({1, int(steps_per_graph)}):
            for primed in (False, True):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    eng.run_ahead(batch, S, prologue=not primed)
                self.graphs[(S, primed)] = g
                pool = g.pool() if pool is None else pool

    def graph(self, S: int, primed: bool = False):
        return self.graphs[(S, primed)]

    def replay(self, S: int):
        # (the persistent kernel's S steps are one graph node; launching it directly instead
        # measured slower in bench.py's driver form, 81.6k vs 85.0k steps/s: profiles/r5_pst_headline.txt)
        self.graphs[(S, bool(self.eng.ahead_primed))].replay()
        self.eng.ahead_primed = True
        if not self._checked:
            # the first replay (warmup) checks the run-ahead error word once, so a tile
            # map or column barrier that failed on this device stops the run here
            # instead of at finalize() after a whole run on wrong weights
            self._checked = True
            err = int(self.eng.ztick[1].item())
            tx = getattr(self.eng, "tx", None)
            if tx is not None and tx.error():
                err |= 4
            dz = self.eng.dzs_error() if hasattr(self.eng, "dzs_error") else 0
            if dz:
                raise RuntimeError("md_bwd dZ split: a column-block barrier timed out on the first replay "
                                   "(not every workgroup resident); rerun with JDT_MD_DZS=0")
            if err:
                raise RuntimeError(f"run-ahead step failed on its first replay (error word {err}: "
                                   "1 = tile map, 2 = column barrier timeout, 4 = tile exchange timeout); "
                                   "rerun with JDT_MLP2_AHEAD=0 (JDT_DP_AHEAD=0 at N > 1)")


# ----------------------------------------------------------------------------- deep MLPs (csrc/mlp_deep.hip)
class MdArgs(ctypes.Structure):
    """Mirror of ``jdt::MdArgs`` (field order and types must match)."""

    _fields_ = [("M", c_int), ("K", c_int), ("N", c_int), ("C", c_int), ("inv_mb", c_float),
                ("X", c_void_p), ("Ws0", c_void_p), ("Ws1", c_void_p), ("WT", c_void_p), ("ldwt", c_int),
                ("bs", c_void_p), ("G", c_void_p), ("Hout", c_void_p), ("INT", c_void_p), ("ldint", c_int),
                ("Wh0", c_void_p), ("Wh1", c_void_p), ("bh", c_void_p), ("logits", c_void_p), ("labels", c_void_p),
                ("keep", c_float), ("seed", c_ulonglong), ("offset", c_ulonglong),
                ("step", c_void_p), ("ticket", c_void_p), ("advance_step", c_int),
                ("dZn", c_void_p), ("Wn0", c_void_p), ("Wn1", c_void_p), ("dZout", c_void_p),
                ("fuse_opt", c_int),
                ("gW", c_void_p), ("gb", c_void_p), ("gWh", c_void_p), ("gbh", c_void_p), ("mslot", c_void_p),
                ("pW", c_void_p), ("mW", c_void_p), ("vW", c_void_p),
                ("pb", c_void_p), ("mb", c_void_p), ("vb", c_void_p),
                ("sb", c_void_p), ("WTout", c_void_p),
                ("pWh", c_void_p), ("mWh", c_void_p), ("vWh", c_void_p),
                ("pbh", c_void_p), ("mbh", c_void_p), ("vbh", c_void_p), ("sbh", c_void_p),
                ("lr", c_float), ("beta1", c_float), ("beta2", c_float), ("eps", c_float), ("wd", c_float),
                ("gscale", c_float), ("running", c_void_p), ("stamps", c_void_p),
                ("accumulate", c_int), ("dH", c_void_p), ("mb_rows", c_int), ("mb_stride", c_ulonglong),
                ("stage_stride", ctypes.c_long), ("det_logits", c_void_p), ("step_mul", c_int),
                ("XR", c_void_p), ("zslab", c_void_p), ("ztick", c_void_p), ("hand", c_void_p),
                ("dzx", c_void_p), ("dzc", c_void_p), ("dzs", c_int), ("smap", c_void_p), ("wt", c_int),
                ("tx", c_void_p), ("tx_base", c_int), ("tx_shared", c_int), ("tx_fsdp", c_int)]


_lib.declare("jdt_md_layer", c_int, [ctypes.POINTER(MdArgs), c_int, c_int, c_void_p])
_lib.declare("jdt_md_dzs_ok", c_int, [c_int])
_lib.declare("jdt_md_args_size", c_int, [])
_lib.declare("jdt_md_ahead_ok", c_int, [c_int])
_lib.declare("jdt_md_fx_ok", c_int, [c_int, c_int])
_lib.declare("jdt_md_fwd2_ok", c_int, [c_int])
_lib.declare("jdt_md_fwd2", c_int, [ctypes.POINTER(MdArgs), ctypes.POINTER(MdArgs), c_void_p, c_void_p])

DEEP_H = 512


def supported_deep(model, rows: int, device) -> bool:
    """784 -> 512 x (L-1) -> 10 MLPs with L >= 3 (the 4-layer MLP of BASELINE configs #2/#3)."""
    from ..models.mlp import MLP

    return (torch.device(device).type == "cuda" and isinstance(model, MLP) and model.L >= 3
            and model.dims[0] == 784 and all(d == DEEP_H for d in model.dims[1:-1]) and model.dims[-1] == 10
            and 0 < rows <= 128 and model.act == "silu" and not model.final_act)


class FusedMLPDeep:
    """One forward and one backward launch per hidden layer (csrc/mlp_deep.hip);
    same interface as :class:`FusedMLP2`."""

    def __init__(self, state, mesh, axis: str, num_minibatches: int, rows: int, metrics: torch.Tensor,
                 params=None, mslot: Optional[torch.Tensor] = None, fuse_opt: Optional[bool] = None,
                 mb_rows: int = 0, mb_stride: int = 1 << 16, tx=None, ranks_on_gpu: int = 1, opt_params=None):
        """``tx`` (comm.tile_exchange.TileExchange, N > 1): every hidden layer's backward
        all-reduces its gradient tiles with the other ranks' launches before the fused
        AdamW (layer i's tiles at exchange offset ``tx_base(i)``), layer 0 running ahead --
        no separate collective launch (FusedMLP2 ``tx``).  ``opt_params`` (FSDP, with
        ``tx``): the rank's LOCAL shards -- each gradient element goes to the rank owning
        its row, which applies the sharded AdamW and hands the value back (md_bwd FX)."""
        P = params if params is not None else state.params
        self.P = P
        self.tx = tx
        self.fsdp_tx = tx is not None and opt_params is not None
        self.OP = opt_params if opt_params is not None else P
        self.tx_shared = int(ranks_on_gpu > 1)
        self.mslot = mslot if mslot is not None else P.metrics_slot
        self.state, self.mesh, self.axis = state, mesh, axis
        self.world = C.axis_size(mesh, axis)
        self.n_mb = num_minibatches
        # mb_rows > 0: dropout masks drawn per microbatch of mb_rows rows (stream offset +
        # i * mb_stride), as the per-microbatch loop draws them (GPipe, one stage)
        self.mb_rows, self.mb_stride = int(mb_rows), int(mb_stride)
        self.model = m = state.apply_fn
        self.metrics = metrics
        self.rows = rows
        dev = P.master.device
        H, L = DEEP_H, m.L
        self.nh = L - 1                                    # hidden layers
        bf = dict(dtype=torch.bfloat16, device=dev)
        # backward factors silu'(Z) * mask/keep, fp32 [row groups of 4][H][4], padded to the
        # forward's 16-row blocks
        self.G = [torch.zeros((rows + 15) // 16 * 4, H, 4, dtype=torch.float32, device=dev)
                  for _ in range(self.nh)]
        self.Hs = [torch.empty(rows, H, **bf) for _ in range(self.nh)]
        self.dZ = [None] + [torch.empty(rows, H, **bf) for _ in range(1, self.nh)]
        self.Mp = (rows + 31) // 32 * 32
        self.INT = [torch.zeros(m.dims[i], self.Mp, **bf) for i in range(self.nh)]
        self.logits = torch.zeros(2, rows, 10, dtype=torch.float32, device=dev)
        if fuse_opt is None:
            fuse_opt = self.world == 1 and os.environ.get("JDT_FUSED_OPT", "1") == "1"
        self.fuse_opt = bool(fuse_opt) and (params is None or self.fsdp_tx) and _is_adamw(state.tx)
        kn = [f"{n}/kernel" for n in m.names]
        self.kn, self.bn = kn, [f"{n}/bias" for n in m.names]
        # second step-parity copy of the row-major shadows read after being updated in
        # the same step: hidden layers >= 1 (by the previous layer's backward) and the head
        self.par = {}
        self.WT = [None] * self.nh
        if self.fuse_opt:
            for i in list(range(1, self.nh)) + [L - 1]:
                self.par[i] = P.s(kn[i]).clone()
            for i in range(self.nh):
                kp = (m.dims[i] + 31) // 32 * 32
                self.WT[i] = torch.zeros(H, kp, **bf)
                self.WT[i][:, : m.dims[i]].copy_(P.s(kn[i]).t())
        if _lib.lib().jdt_md_args_size() != ctypes.sizeof(MdArgs):
            raise RuntimeError("MdArgs layout mismatch")
        self._args = None
        self._key = None
        self.grad_stage = None
        self.det_logits = (torch.zeros(DEEP_H // 16, rows, 10, dtype=torch.float32, device=dev)
                           if deterministic() else None)
        # run-ahead (one GPU, fused AdamW): the layer-0 backward of step t also runs
        # layer 0's forward of step t+1 (csrc/mlp_deep.hip md_bwd AHEAD, per-microbatch
        # dropout streams included), one launch less per step; buffers / checks as FusedMLP2
        # Per-microbatch dropout streams (mb_rows > 0, one-stage GPipe) are opt-in
        # (JDT_MLP2_AHEAD_MB=1): its kernel path passes the H_0 / G_0 check against md_fwd,
        # but a 330-step 8-layer run ended at a different loss than the plain schedule
        # (0.066 vs 0.089, BENCH_NOTES) and that was not explained this round.
        self.ahead_ok = (self.fuse_opt and (self.world == 1 or tx is not None) and self.det_logits is None
                         and (self.mb_rows == 0 or os.environ.get("JDT_MLP2_AHEAD_MB", "0") == "1")
                         and m.dims[0] == 784 and os.environ.get("JDT_MLP2_AHEAD", "1") == "1"
                         and bool(_lib.lib().jdt_md_ahead_ok(rows)))
        self.ahead_primed = False
        self._ahead_args = None
        # dZ split (one GPU): the K-chunk workgroups of a column block share the dZ_i rows
        # instead of each recomputing all of them from the whole dZ_{i+1}
        # (csrc/mlp_deep.hip MdArgs::dzs); JDT_MD_DZS=0 turns it off (A/B: +3 % on the 3- / 4-layer and
        # 8-layer GPipe steps, profiles/r3_dz_split_ab.txt)
        self.dzs_ok = (self.world == 1 and self.nh >= 2 and os.environ.get("JDT_MD_DZS", "1") == "1"
                       and bool(_lib.lib().jdt_md_dzs_ok(rows)))
        if self.dzs_ok:
            self.dzx = [torch.zeros(H // 16 * 16 * 128, **bf) for _ in range(self.nh - 1)]
            self.dzc = [torch.zeros(32 * (1 + H // 16), dtype=torch.int32, device=dev) for _ in range(self.nh - 1)]
        # the last two hidden layers' forwards in ONE launch (csrc/mlp_deep.hip md_fwd2_kernel:
        # a row of layer i+1 needs only that row of layer i, so the launch boundary becomes a
        # per-row-block arrival counter) -- the run-ahead schedule's whole forward when
        # L = 4.  Opt-in (JDT_MD_FWD2=1): 23.6k vs 24.0k steps/s, the counter wait costs what the
        # boundary did (BENCH_NOTES round 6)
        self.fwd2_ok = (self.ahead_ok and self.world == 1 and tx is None and self.nh >= 3
                        and os.environ.get("JDT_MD_FWD2", "0") == "1" and bool(_lib.lib().jdt_md_fwd2_ok(rows)))
        if self.fwd2_ok:
            self.rowc = torch.zeros(32 * (1 + (rows + 15) // 16), dtype=torch.int32, device=dev)
        if self.ahead_ok:
            nch, tpx = 784 // 112, H // 16 * (784 // 112) // 8
            self.XR = torch.zeros(rows, 784, **bf)
            self.zslab = torch.zeros(H // 16 * nch * 128 * 16, dtype=torch.float32, device=dev)
            self.ztick = torch.zeros(32 * (1 + H // 16) + 8 * 32 * ((tpx + 31) // 32), dtype=torch.int32, device=dev)
            self.hand = torch.zeros(H, dtype=torch.float32, device=dev)

    def set_grad_stage(self, base: int, stride: int):
        """See FusedMLP2.set_grad_stage."""
        assert not self.fuse_opt
        self.grad_stage = (int(base), int(stride))
        self._args = None

    def set_fsdp_stage(self, layout: dict, base: int, half: int, slice_: int, world: int):
        """See FusedMLP2.set_fsdp_stage: one StageMap per hidden layer (its W / b, the
        head's W / b, the metric slots)."""
        assert not self.fuse_opt
        L = self.model.L
        dev = self.P.master.device
        self.smap_t = [stage_map_tensor(base, half, slice_, world,
                                        [layout[self.kn[i]], layout[self.bn[i]], layout[self.kn[L - 1]],
                                         layout[self.bn[L - 1]], layout["metrics"]], dev)
                       for i in range(self.nh)]
        self._args = None

    def _shadow_pair(self, i):
        s0 = self.P.s(self.kn[i]).data_ptr()
        return s0, (self.par[i].data_ptr() if i in self.par else s0)

    def _layer(self, batch, i: int, phase: int) -> MdArgs:
        st, P, m = self.state, self.P, self.model
        o = st.opt_state
        L = m.L
        top = i == self.nh - 1
        a = MdArgs()
        a.M, a.K, a.N, a.C = self.rows, m.dims[i], DEEP_H, 10
        a.inv_mb = 1.0 / (self.rows // self.n_mb)
        a.X = batch.inputs.data_ptr() if i == 0 else self.Hs[i - 1].data_ptr()
        a.Ws0, a.Ws1 = self._shadow_pair(i)
        if self.WT[i] is not None:
            if phase == 0:
                a.WT = self.WT[i].data_ptr()
            else:
                a.WTout = self.WT[i].data_ptr()
            a.ldwt = self.WT[i].shape[1]
        a.bs = P.s(self.bn[i]).data_ptr()
        a.G, a.Hout = self.G[i].data_ptr(), self.Hs[i].data_ptr()
        a.INT, a.ldint = self.INT[i].data_ptr(), self.Mp
        a.Wh0, a.Wh1 = self._shadow_pair(L - 1)
        a.bh = P.s(self.bn[L - 1]).data_ptr()
        a.logits, a.labels = self.logits.data_ptr(), batch.labels.data_ptr()
        a.keep = 1.0 - m.dropout_rate
        from ..utils import rng as R

        a.seed = R.fold_rng_over_axis(st.rng, self.mesh, self.axis) & 0xFFFFFFFF
        a.offset = (m.layer_id_base + i) << 1
        a.mb_rows, a.mb_stride = self.mb_rows, self.mb_stride
        if self.ahead_ok and i == 0 and phase == 0:
            a.XR = self.XR.data_ptr()   # the run-ahead backward's operand for the next forward
        if self.det_logits is not None:
            a.det_logits = self.det_logits.data_ptr()
        a.step, a.ticket = o["count"].data_ptr(), o["ticket"].data_ptr()
        a.advance_step = int(self.fuse_opt and phase == 1 and i == 0)
        if not top:
            a.dZn = self.dZ[i + 1].data_ptr()
            a.Wn0, a.Wn1 = self._shadow_pair(i + 1)
            if phase == 1 and self.dzs_ok:
                a.dzx, a.dzc, a.dzs = self.dzx[i].data_ptr(), self.dzc[i].data_ptr(), 1
        if i >= 1:
            a.dZout = self.dZ[i].data_ptr()
        a.fuse_opt = int(self.fuse_opt)
        a.wt = int(os.environ.get("JDT_MD_WT", "1"))   # write-through AdamW state (+3 %, r4_write_through_ab.txt)
        if self.tx is not None and phase == 1:
            a.tx, a.tx_base, a.tx_shared = self.tx.args_ptr, self.tx_base(i), self.tx_shared
            # FSDP: 1 = W row-sharded (dim 0), 2 = column-sharded (dim 1: the reference
            # rule's choice for the square hidden kernels)
            a.tx_fsdp = (0 if not self.fsdp_tx else
                         2 if tuple(self.OP.p(self.kn[i]).shape)[1] != DEEP_H else 1)
        a.gW, a.gb = P.g(self.kn[i]).data_ptr(), P.g(self.bn[i]).data_ptr()
        a.gWh, a.gbh = P.g(self.kn[L - 1]).data_ptr(), P.g(self.bn[L - 1]).data_ptr()
        a.mslot = self.mslot.data_ptr()
        if self.grad_stage is not None:
            base, stride = self.grad_stage
            a.gW, a.gb = base + 4 * P.offsets[self.kn[i]][0], base + 4 * P.offsets[self.bn[i]][0]
            a.gWh, a.gbh = base + 4 * P.offsets[self.kn[L - 1]][0], base + 4 * P.offsets[self.bn[L - 1]][0]
            a.mslot = base + 4 * P.metric_off
            a.stage_stride = stride
        if getattr(self, "smap_t", None) is not None and phase == 1:
            a.smap = self.smap_t[i].data_ptr()
        if self.fuse_opt:
            # AdamW state: the whole leaves, or (FSDP FX) this rank's local shards, whose
            # optimizer state is laid out like the local flat buffer
            mm, vv, OP = o["m"], o["v"], self.OP

            def trio(name):
                off = OP.offsets[name][0]
                return OP.p(name).data_ptr(), mm[off:].data_ptr(), vv[off:].data_ptr()

            a.pW, a.mW, a.vW = trio(self.kn[i])
            a.pb, a.mb, a.vb = trio(self.bn[i])
            a.sb = P.s(self.bn[i]).data_ptr()
            a.pWh, a.mWh, a.vWh = trio(self.kn[L - 1])
            a.pbh, a.mbh, a.vbh = trio(self.bn[L - 1])
            a.sbh = P.s(self.bn[L - 1]).data_ptr()
            tx = st.tx
            a.lr, a.beta1, a.beta2, a.eps, a.wd = tx.learning_rate, tx.b1, tx.b2, tx.eps, tx.weight_decay
            # N > 1 with the tile exchange: the kernels sum the ranks' gradients, 1/N here
            a.gscale = 1.0 / (self.n_mb * (self.world if self.tx is not None else 1))
            a.running = self.metrics.data_ptr()
        return a

    def _ensure_args(self, batch):
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr(), self.state.rng)
        if self._args is None or self._key != key:
            fwd = [self._layer(batch, i, 0) for i in range(self.nh)]
            bwd = [self._layer(batch, i, 1) for i in reversed(range(self.nh))]
            self._args, self._key = (fwd, bwd), key
            self._ahead_args = None

    def run_ahead(self, batch, n: int, prologue: bool = True):
        """n complete steps, the layer-0 backward of each also running layer 0's forward
        of the next step (2 * hidden - 1 launches per step); ``prologue`` first runs
        layer 0's forward of the first step (see FusedMLP2.run_ahead)."""
        assert self.ahead_ok
        self._ensure_args(batch)
        fwd, bwd = self._args
        if self._ahead_args is None:
            b = MdArgs.from_buffer_copy(bwd[-1])   # layer 0's backward
            b.XR, b.zslab, b.ztick, b.hand = (t.data_ptr() for t in (self.XR, self.zslab, self.ztick, self.hand))
            self._ahead_args = b
        Lb = _lib.lib()
        s = _lib.stream_ptr()
        if prologue:
            _lib.check(Lb.jdt_md_layer(ctypes.byref(fwd[0]), 0, int(self.nh == 1), s), "md_fwd")
        elif not torch.cuda.is_current_stream_capturing():
            assert self.ahead_primed, "run_ahead(prologue=False) needs a run-ahead launch just before"
        for _ in range(n):
            last = self.nh - 2 if self.fwd2_ok else self.nh
            for i in range(1, last):
                _lib.check(Lb.jdt_md_layer(ctypes.byref(fwd[i]), 0, int(i == self.nh - 1), s), "md_fwd")
            if self.fwd2_ok:
                _lib.check(Lb.jdt_md_fwd2(ctypes.byref(fwd[-2]), ctypes.byref(fwd[-1]), self.rowc.data_ptr(), s),
                           "md_fwd2")
            for j, a in enumerate(bwd[:-1]):
                _lib.check(Lb.jdt_md_layer(ctypes.byref(a), 1, int(j == 0), s), "md_bwd")
            _lib.check(Lb.jdt_md_layer(ctypes.byref(self._ahead_args), 2, 0, s), "md_bwd_ahead")
        if not torch.cuda.is_current_stream_capturing():
            self.ahead_primed = True

    @staticmethod
    def tx_tiles(nh: int) -> int:
        """Exchange tiles of one step: layer 0's backward 32 x 7, every other 32 x 8."""
        return 224 + 256 * (nh - 1)

    def tx_base(self, i: int) -> int:
        return 0 if i == 0 else 224 + 256 * (i - 1)

    def forward_backward(self, batch):
        if self.tx is not None:
            # N > 1 with the tile exchange: a step is the run-ahead schedule (layer 0's
            # exchanging backward exists only as the run-ahead launch)
            self.run_ahead(batch, 1, prologue=not self.ahead_primed)
            return
        if not torch.cuda.is_current_stream_capturing():
            self.ahead_primed = False
        self._ensure_args(batch)
        Lb = _lib.lib()
        s = _lib.stream_ptr()
        fwd, bwd = self._args
        for i, a in enumerate(fwd):
            _lib.check(Lb.jdt_md_layer(ctypes.byref(a), 0, int(i == self.nh - 1), s), "md_fwd")
        for j, a in enumerate(bwd):
            _lib.check(Lb.jdt_md_layer(ctypes.byref(a), 1, int(j == 0), s), "md_bwd")

    def step(self, batch):
        self.forward_backward(batch)
        if not self.fuse_opt:
            P = self.state.params
            with named_scope("sync_grads"):
                C.psum_(P.grad, self.mesh, self.axis)
            self.state.tx.update(P, self.state.opt_state, 1.0 / (self.n_mb * self.world), zero_grad=False)
            with named_scope("sync_metrics"):
                K.metrics_fold_(self.metrics, P.metrics_slot)

    def dzs_error(self) -> int:
        """Nonzero if a dZ-split block barrier timed out (a block-mate never ran)."""
        return max((int(t[0].item()) for t in self.dzc), default=0) if self.dzs_ok else 0

    def finalize(self):
        """Bring the generic bf16 shadows up to date (parity copies in use on odd steps)."""
        if self.dzs_error():
            raise RuntimeError("md_bwd dZ split: a column-block barrier timed out (not every workgroup "
                               "resident); results invalid -- rerun with JDT_MD_DZS=0")
        if self.ahead_ok and int(self.ztick[1].item()) != 0:
            raise RuntimeError("md_bwd run-ahead: tile map or column barrier failed (error word "
                               f"{int(self.ztick[1].item())}); results invalid")
        if self.tx is not None and self.tx.error():
            raise RuntimeError(f"md_bwd tile exchange: a wait timed out (error word {self.tx.error()}); "
                               "results invalid -- rerun with JDT_DP_AHEAD=0")
        if self.fwd2_ok and int(self.rowc[0].item()) != 0:
            raise RuntimeError("md_fwd2: a row-block wait timed out (not every workgroup resident); results "
                               "invalid -- rerun with JDT_MD_FWD2=0")
        if self.fuse_opt and int(self.state.opt_state["count"].item()) % 2 == 1:
            for i, t in self.par.items():
                self.P.s(self.kn[i]).copy_(t)


def make_engine(state, mesh, axis: str, num_minibatches: int, rows: int, metrics: torch.Tensor, device,
                params=None, mslot: Optional[torch.Tensor] = None, fuse_opt: Optional[bool] = None,
                tx=None, ranks_on_gpu: int = 1, opt_params=None):
    """The whole-step fused engine for ``state.apply_fn`` (2-layer or deep), or None
    if the model/shape is outside the fused kernels' envelope.  ``tx``: the one-launch
    (2-layer) / one-launch-per-layer (deep) N > 1 step; ``opt_params``: FSDP's local shards."""
    model = state.apply_fn
    if supported(model, rows, device):
        return FusedMLP2(state, mesh, axis, num_minibatches, rows, metrics, params=params, mslot=mslot,
                         fuse_opt=fuse_opt, tx=tx, ranks_on_gpu=ranks_on_gpu, opt_params=opt_params)
    if supported_deep(model, rows, device):
        return FusedMLPDeep(state, mesh, axis, num_minibatches, rows, metrics, params=params, mslot=mslot,
                            fuse_opt=fuse_opt, tx=tx, ranks_on_gpu=ranks_on_gpu, opt_params=opt_params)
    return None
