"""Fused whole-step engine for the tutorial classifier (csrc/mlp_fused.hip).

One DP step = ``mlp2_fwd`` + ``mlp2_bwd`` (+ RCCL all-reduce + fused AdamW when
N > 1).  On one GPU the optimizer runs inside ``mlp2_bwd``'s epilogue, so a
step is two kernel launches.  Mathematically identical to the reference's
4-minibatch accumulation loop: each row's loss is weighted 1/(rows per
minibatch) and the summed gradient is scaled by 1/n_minibatches (and 1/N after
the SUM all-reduce); dropout draws one Philox stream per (step, row, unit).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_ulonglong, c_void_p
from typing import Optional

import torch

from ..comm import collectives as C
from ..ops import _lib
from ..ops import kernels as K
from ..utils.profiling import named_scope


class Mlp2Args(ctypes.Structure):
    _fields_ = [("M", c_int), ("H", c_int), ("inv_mb", c_float), ("X", c_void_p), ("labels", c_void_p),
                ("W1s", c_void_p), ("b1s", c_void_p), ("W2s0", c_void_p), ("W2s1", c_void_p), ("b2s", c_void_p),
                ("Z1", c_void_p), ("H1", c_void_p), ("logits", c_void_p),
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
                ("W1T", c_void_p), ("ldw1t", c_int), ("XT", c_void_p), ("ldxt", c_int)]


_lib.declare("jdt_mlp2", c_int, [ctypes.POINTER(Mlp2Args), c_int, c_int, c_int, c_void_p])
_lib.declare("jdt_mlp2_args_size", c_int, [])


def supported(model, rows: int, device) -> bool:
    from ..models.mlp import MLP

    return (torch.device(device).type == "cuda" and isinstance(model, MLP) and model.L == 2 and model.dims[0] == 784
            and model.dims[2] == 10 and model.dims[1] % 16 == 0 and 0 < rows <= 128 and model.act == "silu"
            and not model.final_act)


class FusedMLP2:
    """``params`` (default ``state.params``) supplies the bf16 shadow the kernels read
    and the fp32 grad views mode 0 writes -- FSDP passes its gathered full buffer
    (grads then reduce-scattered), with ``mslot`` its local metric slots."""

    def __init__(self, state, mesh, axis: str, num_minibatches: int, rows: int, metrics: torch.Tensor,
                 params=None, mslot: Optional[torch.Tensor] = None, fuse_opt: Optional[bool] = None):
        P = params if params is not None else state.params
        self.P = P
        self.mslot = mslot if mslot is not None else P.metrics_slot
        self.state, self.mesh, self.axis = state, mesh, axis
        self.world = C.axis_size(mesh, axis)
        self.n_mb = num_minibatches
        self.model = state.apply_fn
        H = self.model.dims[1]
        dev = P.master.device
        self.rows = rows
        self.Z1 = torch.empty(rows, H, dtype=torch.bfloat16, device=dev)
        self.H1 = torch.empty(rows, H, dtype=torch.bfloat16, device=dev)
        self.logits = torch.zeros(2, rows, 10, dtype=torch.float32, device=dev)
        # second parity buffer of W2's bf16 shadow (single-GPU fused-optimizer mode)
        self.W2s1 = P.s("output_dense/kernel").clone()
        self.metrics = metrics
        if fuse_opt is None:
            fuse_opt = self.world == 1 and os.environ.get("JDT_FUSED_OPT", "1") == "1"
        self.fuse_opt = bool(fuse_opt) and params is None
        # K-contiguous bf16 operand copies (zero K padding): X^T written by mlp2_fwd for
        # mlp2_bwd; W1^T written by mlp2_bwd's AdamW epilogue for the next mlp2_fwd
        self.Mp = (rows + 31) // 32 * 32
        self.XT = torch.zeros(784, self.Mp, dtype=torch.bfloat16, device=dev)
        self.W1T = None
        if self.fuse_opt:
            self.W1T = torch.zeros(H, 800, dtype=torch.bfloat16, device=dev)
            self.W1T[:, :784].copy_(P.s("input_dense/kernel").t())
        if _lib.lib().jdt_mlp2_args_size() != ctypes.sizeof(Mlp2Args):
            raise RuntimeError("Mlp2Args layout mismatch")
        self._args = None
        self._key = None

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
        a.Z1, a.H1, a.logits = self.Z1.data_ptr(), self.H1.data_ptr(), self.logits.data_ptr()
        a.keep = 1.0 - self.model.dropout_rate
        from ..utils import rng as R

        a.seed = R.fold_rng_over_axis(st.rng, self.mesh, self.axis) & 0xFFFFFFFF
        a.offset = 0
        a.step, a.ticket = o["count"].data_ptr(), o["ticket"].data_ptr()
        names = ["input_dense/kernel", "input_dense/bias", "output_dense/kernel", "output_dense/bias"]
        a.gW1, a.gb1, a.gW2, a.gb2 = (P.g(n).data_ptr() for n in names)
        a.mslot = self.mslot.data_ptr()
        a.fuse_opt = int(self.fuse_opt)
        a.XT, a.ldxt = self.XT.data_ptr(), self.Mp
        if self.W1T is not None:
            a.W1T, a.ldw1t = self.W1T.data_ptr(), 800
        tx = st.tx
        if self.fuse_opt:
            off = {n: P.offsets[n][0] for n in names}
            m, v = o["m"], o["v"]
            a.pW1, a.pb1, a.pW2, a.pb2 = (P.p(n).data_ptr() for n in names)
            a.mW1, a.mb1, a.mW2, a.mb2 = (m[off[n]:].data_ptr() for n in names)
            a.vW1, a.vb1, a.vW2, a.vb2 = (v[off[n]:].data_ptr() for n in names)
            a.sW1, a.sb1 = P.s(names[0]).data_ptr(), P.s(names[1]).data_ptr()
            a.sW2_0, a.sW2_1 = P.s(names[2]).data_ptr(), self.W2s1.data_ptr()
            a.sb2 = P.s(names[3]).data_ptr()
            a.lr, a.beta1, a.beta2, a.eps, a.wd = tx.learning_rate, tx.b1, tx.b2, tx.eps, tx.weight_decay
            a.gscale = 1.0 / self.n_mb
            a.running = self.metrics.data_ptr()
        return a

    def forward_backward(self, batch):
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr(), self.state.rng)
        if self._args is None or self._key != key:
            self._args, self._key = self._build_args(batch), key
        L = _lib.lib()
        s = _lib.stream_ptr()
        _lib.check(L.jdt_mlp2(ctypes.byref(self._args), 0, 784, 10, s), "mlp2_fwd")
        _lib.check(L.jdt_mlp2(ctypes.byref(self._args), 1, 784, 10, s), "mlp2_bwd")

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
        """Bring the generic bf16 shadow of W2 up to date (parity buffer in use)."""
        P = self.state.params
        if self.fuse_opt and int(self.state.opt_state["count"].item()) % 2 == 1:
            P.s("output_dense/kernel").copy_(self.W2s1)
