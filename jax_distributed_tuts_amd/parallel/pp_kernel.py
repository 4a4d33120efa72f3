"""A GPipe stage's whole step as ONE persistent launch per rank (csrc/pp_stage.hip).

For an MLP pipeline with one 512-wide SiLU/dropout layer per stage (stage 0's takes the
784 inputs, the last stage also carries the 10-class head) -- BASELINE config #4, the
8-stage MLP -- the per-tick schedule of parallel/pipeline.py (a receive, the md layer
kernel, a dX GEMM and a send per microbatch and direction: 3-4 launches per tick)
becomes one launch of 32 workgroups per rank per step: every tick's wait is an in-kernel
poll of the producer stage's inbox flags, every hand-off a system-scope store straight
into the consumer's inbox, the weight gradients stay in registers over the
microbatches and AdamW runs at the end of the same launch.

The engine applies when every rank of the pipe axis can run it (agreed collectively):
a GPU, no data axis (the data-axis all-reduce needs the gradients in memory: the
per-tick path keeps it), AdamW, one layer per stage, microbatches of 16..64 rows
(multiple of 16), all 32 workgroups of every rank sharing the GPU co-resident.
``JDT_PP_KERNEL=0`` turns it off (A/B; bench.py's autotune times both).

Reference: the intended GPipe of /root/reference/pipeline_parallel.py:37-38
(SURVEY §3.5), the tutorial MLP layer of data_paral.py:86-100.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_long, c_longlong, c_ulonglong, c_void_p
from typing import Optional

import torch

from ..ops import _lib

NB = 32          # workgroups per rank (512 / 16 columns)
H = 512
C_HEAD = 10


class PsArgs(ctypes.Structure):
    """Mirror of ``jdt::PsArgs`` (ops/csrc/pp_stage.hip)."""

    _fields_ = [("n_mb", c_int), ("mb", c_int), ("K", c_int), ("gid", c_int), ("mb_shift", c_int),
                ("keep", c_float), ("seed", c_ulonglong),
                ("p", c_void_p), ("m", c_void_p), ("v", c_void_p), ("sW", c_void_p),
                ("pb", c_void_p), ("mbv", c_void_p), ("vb", c_void_p), ("sb", c_void_p),
                ("ph", c_void_p), ("mh", c_void_p), ("vh", c_void_p), ("sh", c_void_p),
                ("phb", c_void_p), ("mhb", c_void_p), ("vhb", c_void_p), ("shb", c_void_p),
                ("X", c_void_p), ("labels", c_void_p),
                ("in_mine", c_void_p), ("flag_mine", c_void_p), ("in_prev", c_void_p), ("flag_prev", c_void_p),
                ("in_next", c_void_p), ("flag_next", c_void_p), ("slot_bytes", c_long), ("err", c_void_p),
                ("timeout", c_longlong),
                ("XT", c_void_p), ("w_mine", c_void_p), ("wflag_mine", c_void_p), ("w_prev", c_void_p),
                ("wflag_prev", c_void_p), ("logits", c_void_p), ("ctr", c_void_p),
                ("gpart", c_void_p), ("gstride", c_long), ("step", c_void_p), ("ticket", c_void_p),
                ("lr", c_float), ("b1", c_float), ("b2", c_float), ("eps", c_float), ("wd", c_float),
                ("gscale", c_float), ("mslot", c_void_p), ("running", c_void_p), ("stamps", c_void_p)]


_lib.declare("jdt_pp_stage_args_size", c_int, [])
_lib.declare("jdt_pp_stage_gstride", c_long, [c_int])
_lib.declare("jdt_pp_stage_ok", c_int, [c_int, c_int, c_int, c_int])
_lib.declare("jdt_pp_stage", c_int, [ctypes.POINTER(PsArgs), c_int, c_int, c_void_p])
_lib.declare("jdt_p2p_max_slots", c_int, [])
_lib.declare("jdt_p2p_peer", c_int, [c_void_p, c_int, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p),
                                     ctypes.POINTER(c_void_p)])


W_BYTES = H * H * 2   # a stage's bf16 weight image (ops/csrc/pp_stage.hip PS_WBYTES)


def _fill_params(a: "PsArgs", P, o, layer: str, head: Optional[str]):
    """Layer ``layer``'s (and the head's) fp32 master / Adam moments / bf16 shadow pointers."""
    def trio(name):
        off = P.offsets[name][0]
        return P.p(name).data_ptr(), o["m"][off:].data_ptr(), o["v"][off:].data_ptr()

    kn, bn = f"{layer}/kernel", f"{layer}/bias"
    a.p, a.m, a.v = trio(kn)
    a.sW = P.s(kn).data_ptr()
    a.pb, a.mbv, a.vb = trio(bn)
    a.sb = P.s(bn).data_ptr()
    if head is not None:
        hk, hb = f"{head}/kernel", f"{head}/bias"
        a.ph, a.mh, a.vh = trio(hk)
        a.sh = P.s(hk).data_ptr()
        a.phb, a.mhb, a.vhb = trio(hb)
        a.shb = P.s(hb).data_ptr()


def slot_bytes(mb: int) -> int:
    """Inbox slot: H [mb][512] then H^T [512][mbp] (bf16)."""
    mbp = (mb + 31) // 32 * 32
    return mb * H * 2 + H * mbp * 2


def stage_fits(model, first: bool, last: bool) -> bool:
    """One 512-wide SiLU layer per stage (784 inputs on stage 0), the head on the last."""
    from ..models.mlp import MLP

    if not isinstance(model, MLP) or model.act != "silu":
        return False
    k0 = 784 if first else H
    if last:
        return model.L == 2 and list(model.dims) == [k0, H, C_HEAD] and not model.final_act
    return model.L == 1 and list(model.dims) == [k0, H] and model.final_act


def local_ok(trainer, mb: int) -> bool:
    """This rank's view of whether the stage kernel applies (not collective)."""
    from ..utils.train_state import AdamW

    n_mb = trainer.cfg.num_microbatches
    if os.environ.get("JDT_PP_KERNEL", "1") == "0" or trainer.dev.type != "cuda":
        return False
    if trainer.S < 2 or trainer.n_dp != 1 or not isinstance(trainer.state.tx, AdamW):
        return False
    # 32 or 64 rows: two row halves of whole 16-row MFMA tiles per column block
    if not (mb in (32, 64) and n_mb * mb == 128):
        return False
    if 2 * n_mb > int(_lib.lib().jdt_p2p_max_slots()):
        return False
    if not stage_fits(trainer.model, trainer.first, trainer.last):
        return False
    from ..runtime.dist import ranks_per_gpu

    # JDT_PP_STAGE_SPARE=0: ranks sharing the GPU may fill every workgroup slot with stage
    # workgroups (tests: the 8-stage protocol on one GPU); default: keep half free
    spare = 0 if os.environ.get("JDT_PP_STAGE_SPARE") == "0" else 1
    return bool(_lib.lib().jdt_pp_stage_ok(int(trainer.first), int(trainer.last), ranks_per_gpu(), spare))


class PPStageKernel:
    """One rank's stage of the in-kernel GPipe step (collective construction over the
    pipe axis: every stage builds its engine at the same point)."""

    def __init__(self, trainer, mb: int, seed: int):
        from ..comm.p2p import TICKS_PER_S, XgmiP2P
        from ..runtime.dist import spin_timeout_s

        if _lib.lib().jdt_pp_stage_args_size() != ctypes.sizeof(PsArgs):
            raise RuntimeError("PsArgs layout mismatch")
        tr = self.tr = trainer
        self.mb, self.n_mb = mb, trainer.cfg.num_microbatches
        self.first, self.last = trainer.first, trainer.last
        dev = self.dev = trainer.dev
        S, s = trainer.S, trainer.s
        timeout_s = spin_timeout_s(30.0)
        self.p2p = XgmiP2P(trainer.mesh.group(trainer.cfg.pipe_axis), s, S, slot_bytes(mb), 2 * self.n_mb, dev,
                           timeout_s=timeout_s)
        # weight boxes: two slots (step parity) of a 512 x 512 bf16 image, written by the
        # successor at its step start, read by this stage's backward (dH = dZ_next W_next^T)
        self.wbox = XgmiP2P(trainer.mesh.group(trainer.cfg.pipe_axis), s, S, W_BYTES, 2, dev, timeout_s=timeout_s)
        self.ok = self.p2p.ok and self.wbox.ok
        if not self.ok:
            return
        L = _lib.lib()

        def peer(box, q):
            ib, fl, er = c_void_p(), c_void_p(), c_void_p()
            _lib.check(L.jdt_p2p_peer(box.ctx, int(q), ctypes.byref(ib), ctypes.byref(fl), ctypes.byref(er)),
                       "jdt_p2p_peer")
            return ib.value, fl.value, er.value

        mine = peer(self.p2p, s)
        prev = peer(self.p2p, s - 1) if s > 0 else (None, None, None)
        nxt = peer(self.p2p, s + 1) if s < S - 1 else (None, None, None)
        w_mine = peer(self.wbox, s) if s < S - 1 else (None, None, None)
        w_prev = peer(self.wbox, s - 1) if s > 0 else (None, None, None)
        P, st, model = trainer.state.params, trainer.state, trainer.model
        o = st.opt_state
        bf = dict(dtype=torch.bfloat16, device=dev)
        # scratch: stage 0's per-microbatch X^T blocks [n_mb][784][mb] (the dW operand,
        # written by the kernel's pre-pass); the two row halves' partial gradients, summed
        # by the AdamW launch that follows the stage launch
        self.XT = torch.zeros(128 * 784, **bf) if self.first else None
        self.gstride = int(L.jdt_pp_stage_gstride(int(model.dims[0])))
        self.gpart = torch.zeros(2 * self.gstride, dtype=torch.float32, device=dev)
        self.logits = torch.zeros(2, 128, C_HEAD, dtype=torch.float32, device=dev) if self.last else None
        self.ctr = torch.zeros(64 * 32, dtype=torch.int32, device=dev)
        self.stamps = None

        a = PsArgs()
        a.n_mb, a.mb, a.K = self.n_mb, mb, model.dims[0]
        a.gid = int(model.layer_id_base)
        a.mb_shift = 16
        a.keep = 1.0 - float(model.dropout_rate)
        a.seed = int(seed) & 0xFFFFFFFF
        _fill_params(a, P, o, model.names[0], model.names[1] if self.last else None)
        if self.last:
            a.logits = self.logits.data_ptr()
            a.mslot, a.running = P.metrics_slot.data_ptr(), trainer.metrics.data_ptr()
        a.in_mine, a.flag_mine, a.err = mine
        a.in_prev, a.flag_prev, _ = prev
        a.in_next, a.flag_next, _ = nxt
        a.slot_bytes = int(self.p2p.slot_bytes)
        a.timeout = int(timeout_s * TICKS_PER_S)
        a.XT = self.XT.data_ptr() if self.XT is not None else None
        a.w_mine, a.wflag_mine, _ = w_mine
        a.w_prev, a.wflag_prev, _ = w_prev
        a.ctr = self.ctr.data_ptr()
        a.gpart, a.gstride = self.gpart.data_ptr(), self.gstride
        a.step, a.ticket = o["count"].data_ptr(), o["ticket"].data_ptr()
        tx = st.tx
        a.lr, a.b1, a.b2, a.eps, a.wd = tx.learning_rate, tx.b1, tx.b2, tx.eps, tx.weight_decay
        a.gscale = 1.0 / self.n_mb
        self.args = a
        self._key = None

    def set_stamps(self, stamps: Optional[torch.Tensor]):
        """Diagnostic: [32 * 32] int64 s_memrealtime per workgroup (tools/stamp_pp.py)."""
        self.stamps = stamps
        self.args.stamps = stamps.data_ptr() if stamps is not None else None

    def step(self, batch, seed: Optional[int] = None):
        a = self.args
        if seed is not None:
            a.seed = int(seed) & 0xFFFFFFFF   # the trainer's dropout stream (changes on restore)
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr())
        if key != self._key:
            if self.first:
                assert batch.inputs.dtype == torch.float32 and batch.inputs.is_contiguous()
                assert batch.inputs.shape == (self.n_mb * self.mb, 784)
                a.X = batch.inputs.data_ptr()
            if self.last:
                assert batch.labels.dtype == torch.int32 and batch.labels.numel() == self.n_mb * self.mb
                a.labels = batch.labels.data_ptr()
            self._key = key
        _lib.check(_lib.lib().jdt_pp_stage(ctypes.byref(a), int(self.first), int(self.last), c_void_p(_lib.stream_ptr())),
                   "pp_stage")

    def error(self) -> int:
        return self.p2p.error() if self.p2p is not None else 0

    def close(self):
        for box in ("p2p", "wbox"):
            if getattr(self, box, None) is not None:
                getattr(self, box).close()
                setattr(self, box, None)


_lib.declare("jdt_pp_chain_ok", c_int, [c_int])
_lib.declare("jdt_pp_chain_max", c_int, [])
_lib.declare("jdt_pp_chain", c_int, [c_void_p, c_int, c_void_p])


def chain_ok(trainer, mb: int) -> bool:
    """A pipe axis of size 1 holding the whole 784 -> 512 x L -> 10 MLP (2 <= L <= 8),
    AdamW, no data axis, 32- or 64-row microbatches: the one-GPU chain launch applies.
    Opt-in (JDT_PP_CHAIN=1): it measured SLOWER than the layer-by-layer full-chip
    kernels it replaces -- 8 layers 131.7 vs 115.3 us, 4 layers 85.2 vs 61.0 us per step
    (BENCH_NOTES round 5): 32 workgroups per layer leave each tick latency-bound, and the
    AdamW of every layer waits for the whole chain, where the multi-rank stages overlap it."""
    from ..models.mlp import MLP
    from ..utils.train_state import AdamW

    m = trainer.model
    if os.environ.get("JDT_PP_CHAIN", "0") != "1" or trainer.dev.type != "cuda" or trainer.S != 1:
        return False
    if trainer.n_dp != 1 or not isinstance(trainer.state.tx, AdamW) or not isinstance(m, MLP) or m.act != "silu":
        return False
    dims = list(m.dims)
    L = len(dims) - 2
    if not (2 <= L <= int(_lib.lib().jdt_pp_chain_max()) and dims[0] == 784 and dims[-1] == C_HEAD
            and all(d == H for d in dims[1:-1]) and not m.final_act):
        return False
    if not (mb in (32, 64) and trainer.cfg.num_microbatches * mb == 128):
        return False
    return bool(_lib.lib().jdt_pp_chain_ok(L))


class PPChainKernel:
    """One GPU, the whole GPipe step of an L-layer MLP as ONE launch: hidden layer i is
    stage i of the chain (32 workgroups each, all resident), the stages hand off through
    local inboxes with the protocol of the per-rank stage launch (csrc/pp_stage.hip
    pp_chain_kernel), then one AdamW launch over the chip for every layer.  Replaces the
    one-stage GPipe's layer-by-layer launches (2 per layer)."""

    def __init__(self, trainer, mb: int, seed: int):
        from ..comm.p2p import TICKS_PER_S
        from ..runtime.dist import spin_timeout_s

        if _lib.lib().jdt_pp_stage_args_size() != ctypes.sizeof(PsArgs):
            raise RuntimeError("PsArgs layout mismatch")
        L_ = _lib.lib()
        tr = self.tr = trainer
        model = trainer.model
        self.mb, self.n_mb = mb, trainer.cfg.num_microbatches
        dev = self.dev = trainer.dev
        self.L = L = len(model.dims) - 2
        P, st = trainer.state.params, trainer.state
        o = st.opt_state
        bf = dict(dtype=torch.bfloat16, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        sb = slot_bytes(mb)
        n_slots = 2 * self.n_mb
        # per stage: activation / gradient inbox, its flags [64][32], the weight box (two
        # 512 x 512 bf16 images by step parity) and its flags; one error word for all
        self.inbox = [torch.zeros(n_slots * sb, dtype=torch.uint8, device=dev) for _ in range(L)]
        self.flags = [torch.zeros(64 * 32, **i32) for _ in range(L)]
        self.wbox = [torch.zeros(2 * W_BYTES, dtype=torch.uint8, device=dev) for _ in range(L)]
        self.wflags = [torch.zeros(64 * 32, **i32) for _ in range(L)]
        self.err = torch.zeros(1, **i32)
        self.ctr = [torch.zeros(64 * 32, **i32) for _ in range(L)]
        self.gpart = [torch.zeros(2 * int(L_.jdt_pp_stage_gstride(int(model.dims[i]))), dtype=torch.float32,
                                  device=dev) for i in range(L)]
        self.XT = torch.zeros(128 * 784, **bf)
        self.logits = torch.zeros(2, 128, C_HEAD, dtype=torch.float32, device=dev)
        timeout = int(spin_timeout_s(30.0) * TICKS_PER_S)
        tx = st.tx
        self.args = (PsArgs * L)()
        for i in range(L):
            a = self.args[i]
            first, last = i == 0, i == L - 1
            a.n_mb, a.mb, a.K = self.n_mb, mb, model.dims[i]
            a.gid = int(model.layer_id_base) + i
            a.mb_shift = 16
            a.keep = 1.0 - float(model.dropout_rate)
            a.seed = int(seed) & 0xFFFFFFFF
            _fill_params(a, P, o, model.names[i], model.names[L] if last else None)
            if last:
                a.logits = self.logits.data_ptr()
                a.mslot, a.running = P.metrics_slot.data_ptr(), trainer.metrics.data_ptr()
            a.in_mine, a.flag_mine = self.inbox[i].data_ptr(), self.flags[i].data_ptr()
            if not first:
                a.in_prev, a.flag_prev = self.inbox[i - 1].data_ptr(), self.flags[i - 1].data_ptr()
                a.w_prev, a.wflag_prev = self.wbox[i - 1].data_ptr(), self.wflags[i - 1].data_ptr()
            if not last:
                a.in_next, a.flag_next = self.inbox[i + 1].data_ptr(), self.flags[i + 1].data_ptr()
                a.w_mine, a.wflag_mine = self.wbox[i].data_ptr(), self.wflags[i].data_ptr()
            a.slot_bytes = sb
            a.err = self.err.data_ptr()
            a.timeout = timeout
            a.XT = self.XT.data_ptr() if first else None
            a.ctr = self.ctr[i].data_ptr()
            a.gpart, a.gstride = self.gpart[i].data_ptr(), self.gpart[i].numel() // 2
            a.step, a.ticket = o["count"].data_ptr(), o["ticket"].data_ptr()
            a.lr, a.b1, a.b2, a.eps, a.wd = tx.learning_rate, tx.b1, tx.b2, tx.eps, tx.weight_decay
            a.gscale = 1.0 / self.n_mb
        self._key = None
        self.ok = True

    def step(self, batch, seed: Optional[int] = None):
        if seed is not None:
            for i in range(self.L):
                self.args[i].seed = int(seed) & 0xFFFFFFFF
        key = (batch.inputs.data_ptr(), batch.labels.data_ptr())
        if key != self._key:
            assert batch.inputs.dtype == torch.float32 and batch.inputs.is_contiguous()
            assert batch.inputs.shape == (self.n_mb * self.mb, 784)
            assert batch.labels.dtype == torch.int32 and batch.labels.numel() == self.n_mb * self.mb
            self.args[0].X = batch.inputs.data_ptr()
            self.args[self.L - 1].labels = batch.labels.data_ptr()
            self._key = key
        _lib.check(_lib.lib().jdt_pp_chain(ctypes.cast(self.args, c_void_p), self.L, c_void_p(_lib.stream_ptr())),
                   "pp_chain")

    def error(self) -> int:
        return int(self.err.item())

    def close(self):
        pass
