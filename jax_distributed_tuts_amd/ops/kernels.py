"""Python entry points of the gfx950 kernels, with pure-torch CPU references.

Dispatch rule: CUDA (ROCm) tensors ALWAYS run the hand-written HIP kernels from
``ops/lib/libjdt_kernels.so`` (an error is raised if the library cannot be
loaded); CPU tensors run the torch reference below.  The CPU path is what the
gloo-simulated multi-device mode (``util.sim_multiCPU_dev``) executes and is the
fp32 oracle the GPU numerics tests compare against.

Numerics contract: matmul operands are rounded to bf16, products
accumulate in fp32, activations are stored bf16, master params / grads /
optimizer state are fp32.
"""
from __future__ import annotations

import contextlib
import math
import os
import ctypes
from typing import Optional

import numpy as np
import torch

from . import _lib

ACT = {"none": 0, "silu": 1, "gelu": 2, "relu": 3}


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _is_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


_WS = {}
WS_FLOATS = 8 << 20      # 32 MiB split-K slab workspace per device
N_COUNTERS = 1 << 16


def workspace(device):
    """Per-(device, stream) split-K workspace (fp32 slabs) + zeroed arrival
    counters.  The counters are re-armed to 0 by each tile's last arriver, so one
    allocation serves every GEMM on its stream (kernels on one stream never
    overlap; a side stream -- WGradStream -- gets its own)."""
    key = (device.type, device.index, torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0)
    w = _WS.get(key)
    if w is None:
        w = (torch.empty(WS_FLOATS, dtype=torch.float32, device=device),
             torch.zeros(N_COUNTERS, dtype=torch.int32, device=device))
        _WS[key] = w
    if device.type == "cuda" and not torch.cuda.is_current_stream_capturing():
        _capture_workspace(device)
    return w


def _capture_workspace(device):
    """The workspace of torch's default graph-capture stream, made (and its counters
    zeroed) eagerly: created during a capture instead, the counters' zero-fill kernel
    would be RECORDED into that graph and run at every replay (4.6 us per LM step)."""
    cls = torch.cuda.graphs.graph
    if cls.default_capture_stream is None:
        cls.default_capture_stream = torch.cuda.Stream()   # what torch.cuda.graph would create
    s = cls.default_capture_stream
    key = (device.type, device.index, s.cuda_stream)
    if key not in _WS and s.device == device:
        cur = torch.cuda.current_stream(device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            _WS[key] = (torch.empty(WS_FLOATS, dtype=torch.float32, device=device),
                        torch.zeros(N_COUNTERS, dtype=torch.int32, device=device))
        cur.wait_stream(s)


class WGradStream:
    """Weight-gradient GEMMs on a side HIP stream.

    In an explicit backward the dW = h^T dz GEMMs are off the critical path (only
    the dX chain feeds the next layer / the previous pipeline stage), so
    ``run(fn, *tensors)`` forks them onto a second stream after the work queued
    so far, and ``join()`` makes the caller's stream wait before the optimizer.
    The many small GEMMs of a microbatch-sized step then overlap instead of
    queueing behind each other; inside hipGraph capture the fork/join become
    parallel graph branches.  ``tensors`` (the GEMM operands) are kept alive
    until the join so the caching allocator cannot hand their memory to the
    main stream while the side stream still reads it."""

    def __init__(self, device):
        self.s = torch.cuda.Stream(device)
        self.keep: list = []
        self.pending = False

    def run(self, fn, *tensors):
        ev = torch.cuda.Event()
        ev.record()
        self.s.wait_event(ev)
        with torch.cuda.stream(self.s):
            fn()
        self.keep.extend(tensors)
        self.pending = True

    def join(self):
        if self.pending:
            torch.cuda.current_stream().wait_stream(self.s)
            self.keep.clear()
            self.pending = False


class OverlappedAdamW:
    """AdamW applied layer by layer on a side stream while the backward pass
    continues: an explicit backward reports parameters whose gradients are final
    (``on_ready(names)``, output side first); each report forks AdamW over those
    parameters' contiguous range of the flat buffers onto the side stream (no
    step advance), ``finish()`` covers anything unreported, advances the device
    step once (after every range has read it: one stream, in order) and makes the
    caller's stream wait.  The bandwidth-bound optimizer pass then runs under the
    lower layers' GEMMs instead of after them.  Inside hipGraph capture the
    fork / join become graph branches."""

    def __init__(self, P, tx, opt_state, grad_scale: float):
        self.P, self.tx, self.o, self.scale = P, tx, opt_state, float(grad_scale)
        self.s = torch.cuda.Stream(P.master.device)
        self.done: set = set()
        self.forked = False

    def _range(self, names):
        offs = [self.P.offsets[n] for n in names]
        lo = min(o for o, _ in offs)
        hi = max(o + _align4(int(np.prod(sh))) for o, sh in offs)
        return lo, hi

    def _launch(self, lo: int, hi: int):
        P, tx, o = self.P, self.tx, self.o
        adamw_step(P.master[lo:hi], P.grad[lo:hi], o["m"][lo:hi], o["v"][lo:hi],
                   P.shadow[lo:hi] if P.shadow is not None else None, lr=tx.learning_rate, b1=tx.b1, b2=tx.b2,
                   eps=tx.eps, wd=tx.weight_decay, grad_scale=self.scale, step=o["count"], ticket=None)

    def ready(self, names):
        names = [n for n in names if n in self.P.offsets and n not in self.done]
        if not names:
            return
        ev = torch.cuda.Event()
        ev.record()
        self.s.wait_event(ev)
        with torch.cuda.stream(self.s):
            lo, hi = self._range(names)
            self._launch(lo, hi)
        self.done.update(names)
        self.forked = True

    def finish(self):
        rest = [s.name for s in self.P.specs if s.name not in self.done]
        if rest:
            self.ready(rest)
        with torch.cuda.stream(self.s):
            self.o["count"].add_(1)
        torch.cuda.current_stream().wait_stream(self.s)
        self.done.clear()
        self.forked = False


def _align4(n: int) -> int:
    from ..utils.flat import _align

    return _align(n)


def dw_gemm(wgrad: Optional["WGradStream"], h, dz, out, opt: Optional["EpilogueAdamW"] = None, name: str = "",
            **kw):
    """``out += h^T dz`` (a_layout "km", b_layout "kn", fp32 accumulate), on the
    side stream when ``wgrad`` is given (GPU), inline otherwise.  With ``opt`` (an
    :class:`EpilogueAdamW` covering ``name``) this is the weight's final gradient of
    the step and AdamW runs in the GEMM epilogue instead (see GemmArgs::opt_*)."""
    acc = True
    if opt is not None and opt.covers(name):
        kw["opt"] = opt.views(name)
        acc = not opt.only_contribution
    if wgrad is None or not h.is_cuda:
        return gemm(h, dz, a_layout="km", b_layout="kn", out=out, accumulate=acc, **kw)
    wgrad.run(lambda: gemm(h, dz, a_layout="km", b_layout="kn", out=out, accumulate=acc, **kw), h, dz)
    return out


class EpilogueAdamW:
    """AdamW for one stage's step with the weight matrices updated in the epilogues of
    their final weight-gradient GEMMs (the fp32 gradient of a fused weight never goes
    to HBM when it has a single contribution) and every other parameter (biases,
    LayerNorm, embeddings) by ONE multi-range launch (``finish``), which also advances
    the device step counter -- instead of an AdamW pass over the whole flat buffer
    (read p, g, m, v; write p, m, v, bf16 shadow, zeroed g: 34 B per parameter).
    ``only_contribution``: the backward pass carrying it is the weights' sole gradient
    contribution of the step (layer-major single pass) -> no read-modify-write of the
    gradient buffer; otherwise (last of several microbatches) the epilogue adds the
    accumulated gradient and re-zeroes it."""

    def __init__(self, P, tx, opt_state, grad_scale: float, fused_names):
        self.P, self.tx, self.o, self.grad_scale = P, tx, opt_state, float(grad_scale)
        self.fused = [n for n in fused_names if n in P.offsets]
        self.only_contribution = True
        from ..utils.flat import _align

        rest = sorted((P.offsets[n][0], _align(int(math.prod(P.offsets[n][1])))) for n in P.names()
                      if n not in self.fused)
        merged = []
        for st_, ln in rest:
            if merged and merged[-1][0] + merged[-1][1] == st_:
                merged[-1][1] += ln
            else:
                merged.append([st_, ln])
        starts = [m_[0] for m_ in merged]
        pref, acc = [], 0
        for _, ln in merged:
            pref.append(acc)
            acc += ln
        dev = P.master.device
        self.nr, self.total = len(merged), acc
        self.start = torch.tensor(starts, dtype=torch.int64, device=dev)
        self.prefix = torch.tensor(pref, dtype=torch.int64, device=dev)

    def covers(self, name: str) -> bool:
        return name in self.fused

    def views(self, name: str):
        off, shape = self.P.offsets[name]
        n = int(math.prod(shape))
        return (self.P.p(name), self.o["m"][off:off + n].view(shape), self.o["v"][off:off + n].view(shape),
                self.P.s(name), self)

    def finish(self):
        """AdamW over every parameter not fused into a GEMM epilogue; advances the step."""
        P, tx, o = self.P, self.tx, self.o
        rc = _lib.lib().jdt_adamw_ranges(_ptr(P.master), _ptr(P.grad), _ptr(o["m"]), _ptr(o["v"]), _ptr(P.shadow),
                                         _ptr(self.start), _ptr(self.prefix), self.nr, self.total,
                                         float(tx.learning_rate), float(tx.b1), float(tx.b2), float(tx.eps),
                                         float(tx.weight_decay), self.grad_scale, _ptr(o["count"]), _ptr(o["ticket"]),
                                         _lib.stream_ptr())
        _lib.check(rc, "jdt_adamw_ranges")


# ----------------------------------------------------------------------------- philox (CPU mirror)
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox_uniform(seed: int, offset: int, idx: np.ndarray, word: int | np.ndarray = 0) -> np.ndarray:
    """Bit-exact numpy mirror of ``jdt::philox4x32``; output word ``word`` -> U[0,1) with 24 bits."""
    idx = idx.astype(np.uint64)
    c0 = idx & _MASK32
    c1 = idx >> np.uint64(32)
    c2 = np.full_like(c0, np.uint64(offset) & _MASK32)
    c3 = np.full_like(c0, (np.uint64(offset) >> np.uint64(32)) & _MASK32)
    k0 = np.uint64(seed) & _MASK32
    k1 = (np.uint64(seed) >> np.uint64(32)) & _MASK32
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0
            p1 = _M1 * c2
            hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
            hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
            n0 = hi1 ^ c1 ^ k0
            n2 = hi0 ^ c3 ^ k1
            c0, c1, c2, c3 = n0, lo1, n2, lo0
            k0 = (k0 + _W0) & _MASK32
            k1 = (k1 + _W1) & _MASK32
    words = np.stack([c0, c1, c2, c3], 0)
    word = np.broadcast_to(np.asarray(word, dtype=np.int64), c0.shape)
    sel = np.take_along_axis(words, word[None], 0)[0]
    return (sel >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)


def dropout_mask(seed: int, offset: int, shape, keep_prob: float) -> torch.Tensor:
    """Mirror of the kernels' grouped mask (common.h ``dropout_group``): element
    (z, r, c) of a [Z.., M, N] tensor keeps iff word (r & 3) of
    philox(seed, (z * ceil(M/4) + r // 4) * N + c, offset) is < keep_prob."""
    shape = tuple(shape)
    M, N = shape[-2], shape[-1]
    Z = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    z = np.arange(Z, dtype=np.uint64)[:, None, None]
    r = np.arange(M, dtype=np.uint64)[None, :, None]
    c = np.arange(N, dtype=np.uint64)[None, None, :]
    grp = (z * np.uint64((M + 3) // 4) + (r >> np.uint64(2))) * np.uint64(N) + c
    word = np.broadcast_to((r & np.uint64(3)).astype(np.int64), grp.shape)
    u = philox_uniform(seed, offset, grp.reshape(-1), word.reshape(-1))
    return torch.from_numpy(u < keep_prob).reshape(shape)


# ----------------------------------------------------------------------------- activations (torch)
def act_fwd_t(act: str, z: torch.Tensor) -> torch.Tensor:
    if act == "silu":
        return z * torch.sigmoid(z)
    if act == "gelu":
        return torch.nn.functional.gelu(z, approximate="tanh")
    if act == "relu":
        return torch.relu(z)
    return z


def act_grad_t(act: str, z: torch.Tensor) -> torch.Tensor:
    if act == "silu":
        s = torch.sigmoid(z)
        return s * (1 + z * (1 - s))
    if act == "gelu":
        k = 0.7978845608028654
        u = k * (z + 0.044715 * z ** 3)
        t = torch.tanh(u)
        return 0.5 * (1 + t) + 0.5 * z * (1 - t * t) * k * (1 + 3 * 0.044715 * z * z)
    if act == "relu":
        return (z > 0).to(z.dtype)
    return torch.ones_like(z)


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


# ----------------------------------------------------------------------------- GEMM
def gemm(a: torch.Tensor, b: torch.Tensor, *, a_layout: str = "mk", b_layout: str = "kn",
         out: Optional[torch.Tensor] = None, out_dtype=torch.bfloat16, accumulate: bool = False,
         alpha: float = 1.0, bias: Optional[torch.Tensor] = None, act: str = "none",
         z_out: Optional[torch.Tensor] = None, z_in: Optional[torch.Tensor] = None, act_bwd: str = "none",
         keep_prob: float = 1.0, seed: int = 0, offset: int = 0, resid: Optional[torch.Tensor] = None,
         dbias: Optional[torch.Tensor] = None, step: Optional[torch.Tensor] = None,
         cfg: int = -1, splits: int = -1, opt=None, seed_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C = epilogue(alpha * A @ B).

    ``a`` holds logical A[M,K] as ``[M,K]`` (``a_layout="mk"``) or ``[K,M]`` ("km");
    ``b`` holds logical B[K,N] as ``[K,N]`` ("kn", a flax ``[in,out]`` kernel) or
    ``[N,K]`` ("nk").  Optional leading batch dim on every operand.
    Epilogue order: +bias -> (store z_out) -> *act'(z_in) -> act -> dropout -> +resid
    -> store/accumulate; ``dbias += colsum(result)``.  Dropout uses Philox stream
    (seed, offset + (step[0] << 32)) when a device step counter is given;
    ``seed_dev`` (device int64[1]) replaces ``seed`` by a value read in the kernel.
    """
    batched = a.dim() == 3
    if a_layout == "mk":
        M, K = a.shape[-2], a.shape[-1]
    else:
        K, M = a.shape[-2], a.shape[-1]
    N = b.shape[-1] if b_layout == "kn" else b.shape[-2]
    Kb = b.shape[-2] if b_layout == "kn" else b.shape[-1]
    assert Kb == K, f"gemm K mismatch {K} vs {Kb}"
    lead = (a.shape[0],) if batched else ()
    if out is None:
        out = (torch.zeros if accumulate else torch.empty)(*lead, M, N, dtype=out_dtype, device=a.device)
    if not _is_gpu(a):
        assert opt is None, "epilogue AdamW is a GPU path"
        if step is not None and keep_prob < 1.0:
            offset = int(offset) + (int(step.item()) << 32)
        if seed_dev is not None:
            seed = int(seed_dev.item())
        return _gemm_ref(a, b, a_layout, b_layout, out, accumulate, alpha, bias, act, z_out, z_in, act_bwd,
                         keep_prob, seed, offset, resid, dbias)
    for t in (a, b, out, z_out, z_in, resid):
        if t is not None:
            assert t.stride(-1) == 1, "gemm operands must be contiguous in the last dim"
            assert t.dtype in (torch.bfloat16, torch.float32)
    g = _lib.GemmArgs()
    g.A, g.lda, g.a_f32, g.a_trans = a.data_ptr(), a.stride(-2), int(a.dtype == torch.float32), int(a_layout == "km")
    g.B, g.ldb, g.b_f32, g.b_trans = b.data_ptr(), b.stride(-2), int(b.dtype == torch.float32), int(b_layout == "kn")
    g.sA = a.stride(0) if batched else 0
    g.sB = (b.stride(0) if b.dim() == 3 else 0) if batched else 0
    g.M, g.N, g.K, g.alpha = M, N, K, float(alpha)
    if bias is not None:
        assert bias.is_contiguous()
        g.bias, g.bias_f32 = bias.data_ptr(), int(bias.dtype == torch.float32)
    g.act = ACT[act]
    if z_out is not None:
        assert z_out.dtype == torch.bfloat16
        g.Zout, g.ldz, g.sZ = z_out.data_ptr(), z_out.stride(-2), (z_out.stride(0) if batched else 0)
    if z_in is not None:
        assert z_in.dtype == torch.bfloat16
        g.Zin, g.ldzin, g.sZin = z_in.data_ptr(), z_in.stride(-2), (z_in.stride(0) if batched else 0)
        g.act_bwd = ACT[act_bwd]
    g.keep_prob, g.seed, g.offset = float(keep_prob), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1)
    if resid is not None:
        assert resid.dtype == torch.bfloat16
        g.resid, g.ldr, g.sR = resid.data_ptr(), resid.stride(-2), (resid.stride(0) if batched else 0)
    if dbias is not None:
        assert dbias.dtype == torch.float32 and dbias.is_contiguous()
        g.dbias = dbias.data_ptr()
    g.C, g.ldc, g.sC = out.data_ptr(), out.stride(-2), (out.stride(0) if batched else 0)
    g.c_f32, g.accumulate = int(out.dtype == torch.float32), int(accumulate)
    if step is not None:
        assert step.dtype == torch.int32
        g.step_ptr = step.data_ptr()
    if seed_dev is not None:
        assert seed_dev.dtype == torch.int64 and seed_dev.is_cuda
        g.seed_ptr = seed_dev.data_ptr()
    if opt is not None:   # (p, m, v, shadow views shaped like out, EpilogueAdamW): AdamW in the epilogue
        pv, mv, vv, sv, eo = opt
        assert out.dtype == torch.float32 and not batched
        for t in (pv, mv, vv, sv):
            assert t.shape == out.shape and t.is_contiguous() and out.is_contiguous()
        g.opt_p, g.opt_m, g.opt_v, g.opt_s = pv.data_ptr(), mv.data_ptr(), vv.data_ptr(), sv.data_ptr()
        g.opt_step = eo.o["count"].data_ptr()
        tx = eo.tx
        g.opt_lr, g.opt_b1, g.opt_b2, g.opt_eps, g.opt_wd, g.opt_gs = (float(tx.learning_rate), float(tx.b1),
                                                                       float(tx.b2), float(tx.eps),
                                                                       float(tx.weight_decay), eo.grad_scale)
    if _WPASS and not batched and cfg < 0 and splits < 0:
        _WPASS[-1].append((g, a.device, (a, b, out, bias, z_out, z_in, resid, dbias, step, seed_dev)))
        return out
    if _GROUP and not batched and cfg < 0 and splits < 0:
        _GROUP[-1].append((g, a.device, (a, b, out, bias, z_out, z_in, resid, dbias, step, seed_dev)))
        return out
    _launch_gemm(g, int(a.shape[0]) if batched else 1, cfg, splits, a.device)
    return out


def _launch_gemm(g, batch: int, cfg: int, splits: int, device):
    ws, ctr = workspace(device)
    rc = _lib.lib().jdt_gemm(ctypes.byref(g), int(batch), int(cfg), int(splits),
                             ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(ctr.data_ptr()),
                             ctr.numel(), _lib.stream_ptr())
    _lib.check(rc, "jdt_gemm")


_GROUP: list = []
_WPASS: list = []
_WPASS_PLANS: dict = {}
# tile config of the one-launch W pass (csrc/gemm.hip jdt_gemm_wpass_launch): 4 = 64 x 128
# tiles of 32x32x16 MFMAs, two workgroups per CU (one's AdamW epilogue under the other's
# main loop) -- 109 us alone vs 126 (cfg 2, 128 x 128) and 143 (cfg 0, 64 x 64); LM step
# 0.879 vs 0.906 ms (profiles/r6_s6_floor_wpass.txt)
WPASS_CFG = int(os.environ.get("JDT_WPASS_CFG", "4"))


@contextlib.contextmanager
def gemm_wpass(cfg: Optional[int] = None):
    """GPU GEMMs issued inside the block -- a stage's deferred weight-gradient GEMMs
    dW (+)= A^T dZ, both operands token-major, AdamW in their epilogues -- run at its end as
    ONE launch (csrc/gemm.hip ``gemm_wpass_kernel``: every problem's tiles in one grid,
    problems picked from a prefix table in device memory).  The table is planned and
    uploaded on the first (eager) use of a problem set and reused by later calls and graph
    replays; a set first seen inside a stream capture, or outside the kernel's envelope,
    launches problem by problem (same results)."""
    _WPASS.append([])
    try:
        yield
    finally:
        items = _WPASS.pop()
        if items:
            _launch_wpass(items, WPASS_CFG if cfg is None else int(cfg))


def _launch_wpass(items, cfg: int):
    L = _lib.lib()
    dev = items[0][1]
    arr = (_lib.GemmArgs * len(items))(*[it[0] for it in items])
    # (the plan embeds the planning stream's split-K workspace; a W pass runs on one
    # stream at a time, and a graph capture replays the eager plan)
    key = (bytes(arr), cfg)
    plan = _WPASS_PLANS.get(key)
    if plan is None and not torch.cuda.is_current_stream_capturing():
        ws, ctr = workspace(dev)
        host = (ctypes.c_char * int(L.jdt_gemm_wpass_table_bytes()))()
        total = int(L.jdt_gemm_wpass_plan(arr, len(items), int(cfg), host, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                          ctypes.c_void_p(ctr.data_ptr()), ctr.numel()))
        table = None
        if total > 0:
            table = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
        plan = _WPASS_PLANS[key] = (table, total)
    if plan is None or plan[0] is None:
        for g, d, _refs in items:
            _launch_gemm(g, 1, -1, -1, d)
        return
    table, total = plan
    _lib.check(L.jdt_gemm_wpass_launch(ctypes.c_void_p(table.data_ptr()), total, int(cfg), _lib.stream_ptr()),
               "jdt_gemm_wpass")


@contextlib.contextmanager
def gemm_group():
    """GPU GEMMs issued inside the block (unbatched, default config) are launched
    together at its end as ONE grouped kernel (csrc/gemm.hip
    ``gemm_dma_group_kernel``) -- e.g. a layer's weight- and input-gradient
    GEMMs, which both only need dz.  Outputs are allocated at call time but
    written at the end of the block, so nothing inside may read them.  Shapes
    outside the grouped kernel's envelope are launched one by one."""
    _GROUP.append([])
    try:
        yield
    finally:
        items = _GROUP.pop()
        if items:
            if len(items) > 1:
                arr = (_lib.GemmArgs * len(items))(*[it[0] for it in items])
                ws, ctr = workspace(items[0][1])
                rc = _lib.lib().jdt_gemm_group(arr, len(items), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                               ctypes.c_void_p(ctr.data_ptr()), ctr.numel(), _lib.stream_ptr())
                if rc != 1:
                    _lib.check(rc, "jdt_gemm_group")
                    items = []
            for g, dev, _refs in items:
                _launch_gemm(g, 1, -1, -1, dev)


def _gemm_ref(a, b, a_layout, b_layout, out, accumulate, alpha, bias, act, z_out, z_in, act_bwd, keep_prob, seed,
              offset, resid, dbias):
    A = _bf(a.float())
    B = _bf(b.float())
    if a_layout == "km":
        A = A.transpose(-1, -2)
    if b_layout == "nk":
        B = B.transpose(-1, -2)
    v = alpha * torch.matmul(A, B)
    if bias is not None:
        v = v + bias.float()
    if z_out is not None:
        z_out.copy_(v.to(torch.bfloat16))
        if act != "none":
            v = _bf(v)
    if z_in is not None:
        v = v * act_grad_t(act_bwd, z_in.float())
    v = act_fwd_t(act, v)
    if keep_prob < 1.0:
        M, N = v.shape[-2], v.shape[-1]
        mask = dropout_mask(seed, offset, v.shape, keep_prob).to(v.device)
        del M, N
        v = torch.where(mask, v / keep_prob, torch.zeros_like(v))
    if resid is not None:
        v = v + resid.float()
    if out.dtype == torch.float32:
        if accumulate:
            out.add_(v)
        else:
            out.copy_(v)
        contrib = v
    else:
        if accumulate:
            out.copy_((out.float() + v).to(out.dtype))
            contrib = v
        else:
            out.copy_(v.to(out.dtype))
            contrib = out.float()
    if dbias is not None:
        dbias.add_(contrib.reshape(-1, contrib.shape[-1]).sum(0))
    return out


# ----------------------------------------------------------------------------- cross-entropy
def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, *, grad_scale: float = 1.0,
                 dlogits: Optional[torch.Tensor] = None, dbias: Optional[torch.Tensor] = None,
                 metrics: Optional[torch.Tensor] = None, row_loss: Optional[torch.Tensor] = None,
                 mslab: Optional[torch.Tensor] = None):
    """Fused softmax-CE fwd+bwd.  Writes dlogits = (softmax - onehot) * grad_scale (bf16),
    adds colsum(dlogits) into dbias, adds [loss_sum, n, correct, n] into metrics (fp32[4]).
    ``mslab`` (GPU, fp32 [rows, 4], zero): the metric sums may instead go to one row per
    workgroup (no same-address atomics); the caller then folds with
    ``metrics_fold_(..., slab=mslab)``, which adds slot and slab."""
    M, C = logits.shape
    if not _is_gpu(logits):
        z = logits.float()
        valid = (labels >= 0) & (labels < C)
        lab = labels.clamp(0, C - 1).long()
        lse = torch.logsumexp(z, dim=-1)
        loss = torch.where(valid, lse - z.gather(1, lab[:, None])[:, 0], torch.zeros_like(lse))
        if row_loss is not None:
            row_loss.copy_(loss)
        if dlogits is not None:
            p = torch.softmax(z, dim=-1)
            g = (p - torch.nn.functional.one_hot(lab, C).float()) * grad_scale
            g = torch.where(valid[:, None], g, torch.zeros_like(g))
            dlogits.copy_(g.to(dlogits.dtype))
            if dbias is not None:
                dbias.add_(dlogits.float()[valid].sum(0))
        if metrics is not None:
            correct = ((z.argmax(-1) == lab) & valid).float().sum()
            n = valid.float().sum()
            metrics.add_(torch.stack([loss.sum(), n, correct, n]).to(metrics.device))
        return loss
    assert labels.dtype == torch.int32 and labels.is_contiguous() and logits.stride(-1) == 1
    if dlogits is not None:
        assert dlogits.dtype == torch.bfloat16 and dlogits.stride(-1) == 1
    if mslab is not None and metrics is not None:
        assert mslab.is_cuda and mslab.dtype == torch.float32 and mslab.shape[-1] == 4 and mslab.is_contiguous()
        rc = _lib.lib().jdt_xent_slab(_ptr(logits), int(logits.dtype == torch.float32), logits.stride(0),
                                      _ptr(labels), M, C, float(grad_scale), _ptr(dlogits),
                                      dlogits.stride(0) if dlogits is not None else 0, _ptr(dbias), _ptr(metrics),
                                      _ptr(row_loss), _ptr(mslab), int(mslab.shape[0]), _lib.stream_ptr())
        _lib.check(min(rc, 0), "jdt_xent_slab")   # 1: the slab took the sums, 0: the slot did
        return row_loss
    rc = _lib.lib().jdt_xent(_ptr(logits), int(logits.dtype == torch.float32), logits.stride(0), _ptr(labels), M, C,
                             float(grad_scale), _ptr(dlogits), dlogits.stride(0) if dlogits is not None else 0,
                             _ptr(dbias), _ptr(metrics), _ptr(row_loss), _lib.stream_ptr())
    _lib.check(rc, "jdt_xent")
    return row_loss


# ----------------------------------------------------------------------------- optimizers
def adamw_step(p, g, m, v, shadow, *, lr, b1=0.9, b2=0.999, eps=1e-8, wd=1e-4, grad_scale=1.0, step, ticket,
               zero_grad=True):
    """Fused AdamW over flat fp32 buffers; ``step`` is a device int32[1] counter advanced in-kernel."""
    if not _is_gpu(p):
        t = int(step.item()) + 1
        gr = g * grad_scale
        m.mul_(b1).add_(gr, alpha=1 - b1)
        v.mul_(b2).addcmul_(gr, gr, value=1 - b2)
        mh = m / (1 - b1 ** t)
        vh = v / (1 - b2 ** t)
        p.sub_(lr * (mh / (vh.sqrt() + eps) + wd * p))
        if zero_grad:
            g.zero_()
        if shadow is not None:
            shadow.copy_(p.to(shadow.dtype))
        if ticket is not None:   # no ticket: one range of a split step, the caller advances it
            step.add_(1)
        return
    rc = _lib.lib().jdt_adamw(_ptr(p), _ptr(g), _ptr(m), _ptr(v), _ptr(shadow), p.numel(), float(lr), float(b1),
                              float(b2), float(eps), float(wd), float(grad_scale), _ptr(step), _ptr(ticket),
                              int(zero_grad), _lib.stream_ptr())
    _lib.check(rc, "jdt_adamw")


def sgd_step(p, g, buf, shadow, *, lr, momentum=0.0, wd=0.0, grad_scale=1.0, step=None, ticket=None,
             zero_grad=True):
    if not _is_gpu(p):
        gr = g * grad_scale + wd * p
        if buf is not None:
            buf.mul_(momentum).add_(gr)
            gr = buf
        p.sub_(lr * gr)
        if zero_grad:
            g.zero_()
        if shadow is not None:
            shadow.copy_(p.to(shadow.dtype))
        if step is not None:
            step.add_(1)
        return
    rc = _lib.lib().jdt_sgd(_ptr(p), _ptr(g), _ptr(buf), _ptr(shadow), p.numel(), float(lr), float(momentum),
                            float(wd), float(grad_scale), _ptr(step), _ptr(ticket), int(zero_grad),
                            _lib.stream_ptr())
    _lib.check(rc, "jdt_sgd")


def cast_bf16_(src: torch.Tensor, dst: torch.Tensor):
    if not _is_gpu(src):
        dst.copy_(src.to(torch.bfloat16))
        return dst
    rc = _lib.lib().jdt_cast_f32_bf16(_ptr(src), _ptr(dst), src.numel(), _lib.stream_ptr())
    _lib.check(rc, "jdt_cast_f32_bf16")
    return dst


# ----------------------------------------------------------------------------- elementwise
def act_bwd(dh: torch.Tensor, z: Optional[torch.Tensor], act: str, *, keep_prob: float = 1.0, seed: int = 0,
            offset: int = 0, step: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
            dbias: Optional[torch.Tensor] = None, seed_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dz = dh * dropout_mask/keep * act'(z); dbias += colsum(dz).  [M,N] bf16.
    ``seed_dev``: device int64[1] dropout seed (replaces ``seed``, see :func:`gemm`)."""
    M, N = dh.shape
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dh.device)
    if not _is_gpu(dh):
        v = dh.float()
        if z is not None:
            v = v * act_grad_t(act, z.float())
        if keep_prob < 1.0:
            off = int(offset) + ((int(step.item()) << 32) if step is not None else 0)
            mask = dropout_mask(int(seed_dev.item()) if seed_dev is not None else seed, off, (M, N), keep_prob)
            v = torch.where(mask, v / keep_prob, torch.zeros_like(v))
        out.copy_(v.to(out.dtype))
        if dbias is not None:
            dbias.add_(out.float().sum(0))
        return out
    assert dh.is_contiguous() and out.is_contiguous() and (z is None or z.is_contiguous())
    rc = _lib.lib().jdt_act_bwd(_ptr(dh), _ptr(z), ACT[act] if z is not None else 0, float(keep_prob),
                                int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), _ptr(step), _ptr(seed_dev), M, N,
                                _ptr(out),
                                _ptr(dbias), _lib.stream_ptr())
    _lib.check(rc, "jdt_act_bwd")
    return out


def metrics_fold_(running: torch.Tensor, slot: torch.Tensor, slab: Optional[torch.Tensor] = None,
                  step: Optional[torch.Tensor] = None):
    """running += slot ; slot = 0 (one tiny kernel, graph-capturable).  ``slab`` (fp32
    [rows, 4], softmax_xent's per-workgroup metric rows): its row sums are added as
    {loss, n, correct, n} and it is re-zeroed; ``step`` (device int32[1]): advanced by
    one in the same launch."""
    if not _is_gpu(running):
        running.add_(slot)
        slot.zero_()
        if slab is not None:
            t = slab.sum(0)
            running[:4].add_(torch.stack([t[0], t[1], t[2], t[1]]))
            slab.zero_()
        if step is not None:
            step.add_(1)
        return
    if slab is not None or step is not None:
        cap = int(slab.shape[0]) if slab is not None else 0
        rc = _lib.lib().jdt_metrics_fold_slab(_ptr(running), _ptr(slot), int(slot.numel()), _ptr(slab), cap,
                                              _ptr(step), _lib.stream_ptr())
        _lib.check(rc, "jdt_metrics_fold_slab")
        return
    rc = _lib.lib().jdt_metrics_fold(_ptr(running), _ptr(slot), int(slot.numel()), _lib.stream_ptr())
    _lib.check(rc, "jdt_metrics_fold")


# ----------------------------------------------------------------------------- raw GEMM (strided batches)
def _gemm_raw(*, A, lda, B, ldb, C, ldc, M, N, K, a_trans=False, b_kn=False, a_f32=False, b_f32=False,
              c_f32=False, alpha=1.0, batch=1, zin=1, sA=0, sA2=0, sB=0, sB2=0, sC=0, sC2=0, accumulate=False):
    """Launch jdt_gemm on raw (ptr, ld, stride) descriptors -- used where operands are
    interleaved views (per-head Q/K/V inside the fused [T, 3d] QKV activation)."""
    g = _lib.GemmArgs()
    g.A, g.lda, g.a_f32, g.a_trans, g.sA, g.sA2 = A, lda, int(a_f32), int(a_trans), sA, sA2
    g.B, g.ldb, g.b_f32, g.b_trans, g.sB, g.sB2 = B, ldb, int(b_f32), int(b_kn), sB, sB2
    g.M, g.N, g.K, g.alpha = M, N, K, float(alpha)
    g.keep_prob = 1.0
    g.C, g.ldc, g.sC, g.sC2, g.c_f32, g.accumulate = C, ldc, sC, sC2, int(c_f32), int(accumulate)
    g.zin = zin
    ws, ctr = workspace(torch.device("cuda", torch.cuda.current_device()))
    rc = _lib.lib().jdt_gemm(ctypes.byref(g), batch, -1, -1, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                             ctypes.c_void_p(ctr.data_ptr()), ctr.numel(), _lib.stream_ptr())
    _lib.check(rc, "jdt_gemm(raw)")


# ----------------------------------------------------------------------------- attention
def attention_fwd(qkv: torch.Tensor, B: int, S: int, H: int, causal: bool = True, impl: Optional[str] = None,
                  o_out: Optional[torch.Tensor] = None):
    """qkv [B*S, 3*H*Dh] bf16 (q | k | v column blocks, heads contiguous) ->
    (o [B*S, H*Dh] bf16, aux saved for backward).

    GPU, Dh = 64: fused flash kernel (csrc/flash_attn.hip), aux = LSE [B*H, S] fp32.
    ``impl="composed"`` (or other head dims): MFMA GEMM -> softmax kernel -> GEMM,
    aux = P [B*H, S, S] bf16.  CPU: torch reference, aux = P."""
    T, d3 = qkv.shape
    d = d3 // 3
    Dh = d // H
    scale = 1.0 / (Dh ** 0.5)
    if not _is_gpu(qkv):
        q, k, v = _bf(qkv.float()).view(B, S, 3, H, Dh).permute(2, 0, 3, 1, 4)
        s = torch.matmul(q, k.transpose(-1, -2)) * scale
        if causal:
            s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float("-inf"))
        p = torch.softmax(s, dim=-1).to(torch.bfloat16)
        o = torch.matmul(p.float(), v).permute(0, 2, 1, 3).reshape(T, d).to(torch.bfloat16)
        if o_out is not None:
            o = o_out.copy_(o)
        return o, p.reshape(B * H, S, S)
    assert qkv.is_contiguous()
    dev = qkv.device
    if Dh == 64 and impl != "composed":
        # flash-style fused kernel: returns the per-row LSE instead of P
        o = torch.empty(T, d, dtype=torch.bfloat16, device=dev) if o_out is None else o_out
        assert o.is_contiguous() and o.shape == (T, d)
        lse = torch.empty(B * H, S, dtype=torch.float32, device=dev)
        rc = _lib.lib().jdt_flash_fwd(_ptr(qkv), _ptr(o), _ptr(lse), B, S, H, float(scale), int(causal),
                                      _lib.stream_ptr())
        _lib.check(rc, "jdt_flash_fwd")
        return o, lse
    Sc = torch.empty(B * H, S, S, dtype=torch.float32, device=dev)
    P = torch.empty(B * H, S, S, dtype=torch.bfloat16, device=dev)
    o = torch.empty(T, d, dtype=torch.bfloat16, device=dev) if o_out is None else o_out
    base, e2 = qkv.data_ptr(), 2
    _gemm_raw(A=base, lda=d3, sA=S * d3, sA2=Dh, B=base + d * e2, ldb=d3, sB=S * d3, sB2=Dh, b_kn=False,
              C=Sc.data_ptr(), ldc=S, sC=H * S * S, sC2=S * S, c_f32=True, M=S, N=S, K=Dh, alpha=scale,
              batch=B * H, zin=H)
    rc = _lib.lib().jdt_attn_softmax_fwd(_ptr(Sc), _ptr(P), B * H * S, S, S, int(causal), _lib.stream_ptr())
    _lib.check(rc, "jdt_attn_softmax_fwd")
    _gemm_raw(A=P.data_ptr(), lda=S, sA=H * S * S, sA2=S * S, B=base + 2 * d * e2, ldb=d3, sB=S * d3, sB2=Dh,
              b_kn=True, C=o.data_ptr(), ldc=d, sC=S * d, sC2=Dh, M=S, N=Dh, K=S, batch=B * H, zin=H)
    return o, P


_FLASH_WS: dict = {}


def _flash_workspace(device, n: int, bh: int):
    """Persistent zeroed dQ accumulator + per-(batch, head) tickets for jdt_flash_bwd
    (the kernel leaves both zero again, so one allocation serves every call, eager
    or graph-replayed; the framework issues all compute on one stream per device)."""
    key = str(device)
    ws = _FLASH_WS.get(key)
    if ws is None or ws[0].numel() < n or ws[1].numel() < bh:
        ws = (torch.zeros(max(n, ws[0].numel() if ws else 0), dtype=torch.float32, device=device),
              torch.zeros(max(bh, ws[1].numel() if ws else 0), dtype=torch.int32, device=device))
        _FLASH_WS[key] = ws
    return ws


def attention_bwd(do: torch.Tensor, qkv: torch.Tensor, P: torch.Tensor, B: int, S: int, H: int,
                  dqkv: Optional[torch.Tensor] = None, o: Optional[torch.Tensor] = None,
                  causal: bool = True, dbias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Gradient of attention_fwd w.r.t. qkv ([B*S, 3d] bf16).  ``P`` is attention_fwd's
    aux: the LSE (flash path; then ``o`` is required) or the probabilities.
    ``dbias`` (fp32 [3d]) += colsum(dqkv): the QKV projection's bias gradient,
    fused into the flash kernel (a colsum pass on the other paths)."""
    T, d3 = qkv.shape
    d = d3 // 3
    Dh = d // H
    scale = 1.0 / (Dh ** 0.5)
    if dqkv is None:
        dqkv = torch.empty_like(qkv)
    if _is_gpu(qkv) and P.dim() == 2:
        assert o is not None and do.is_contiguous() and o.is_contiguous() and dqkv.is_contiguous()
        dq_acc, tickets = _flash_workspace(qkv.device, T * d, B * H)
        rc = _lib.lib().jdt_flash_bwd(_ptr(qkv), _ptr(o), _ptr(do), _ptr(P), _ptr(dq_acc), _ptr(tickets), _ptr(dqkv),
                                      _ptr(dbias), B, S, H, float(scale), int(causal), _lib.stream_ptr())
        _lib.check(rc, "jdt_flash_bwd")
        return dqkv
    if not _is_gpu(qkv):
        q, k, v = _bf(qkv.float()).view(B, S, 3, H, Dh).permute(2, 0, 3, 1, 4)
        p = P.float().view(B, H, S, S)
        dO = _bf(do.float()).view(B, S, H, Dh).permute(0, 2, 1, 3)
        dv = torch.matmul(p.transpose(-1, -2), dO)
        dp = torch.matmul(dO, v.transpose(-1, -2))
        ds = _bf(p * (dp - (p * dp).sum(-1, keepdim=True)))
        dq = torch.matmul(ds, k) * scale
        dk = torch.matmul(ds.transpose(-1, -2), q) * scale
        out = torch.stack([dq, dk, dv], 0).permute(1, 3, 0, 2, 4).reshape(T, d3)
        dqkv.copy_(out.to(dqkv.dtype))
        if dbias is not None:
            dbias.add_(dqkv.float().sum(0))
        return dqkv
    dev = qkv.device
    base, gb, dob, e2 = qkv.data_ptr(), dqkv.data_ptr(), do.data_ptr(), 2
    assert do.is_contiguous() and dqkv.is_contiguous()
    # dV = P^T dO
    _gemm_raw(A=P.data_ptr(), lda=S, sA=H * S * S, sA2=S * S, a_trans=True, B=dob, ldb=d, sB=S * d, sB2=Dh, b_kn=True,
              C=gb + 2 * d * e2, ldc=d3, sC=S * d3, sC2=Dh, M=S, N=Dh, K=S, batch=B * H, zin=H)
    # dP = dO V^T
    dP = torch.empty(B * H, S, S, dtype=torch.float32, device=dev)
    _gemm_raw(A=dob, lda=d, sA=S * d, sA2=Dh, B=base + 2 * d * e2, ldb=d3, sB=S * d3, sB2=Dh, b_kn=False,
              C=dP.data_ptr(), ldc=S, sC=H * S * S, sC2=S * S, c_f32=True, M=S, N=S, K=Dh, batch=B * H, zin=H)
    dS = torch.empty(B * H, S, S, dtype=torch.bfloat16, device=dev)
    rc = _lib.lib().jdt_attn_softmax_bwd(_ptr(P), _ptr(dP), _ptr(dS), B * H * S, S, _lib.stream_ptr())
    _lib.check(rc, "jdt_attn_softmax_bwd")
    # dQ = scale dS K ; dK = scale dS^T Q
    _gemm_raw(A=dS.data_ptr(), lda=S, sA=H * S * S, sA2=S * S, B=base + d * e2, ldb=d3, sB=S * d3, sB2=Dh, b_kn=True,
              C=gb, ldc=d3, sC=S * d3, sC2=Dh, M=S, N=Dh, K=S, alpha=scale, batch=B * H, zin=H)
    _gemm_raw(A=dS.data_ptr(), lda=S, sA=H * S * S, sA2=S * S, a_trans=True, B=base, ldb=d3, sB=S * d3, sB2=Dh,
              b_kn=True, C=gb + d * e2, ldc=d3, sC=S * d3, sC2=Dh, M=S, N=Dh, K=S, alpha=scale, batch=B * H, zin=H)
    if dbias is not None:
        colsum_(dqkv, dbias)
    return dqkv


# ----------------------------------------------------------------------------- layernorm / embedding / colsum
def layernorm_fwd(x, gamma, beta, eps=1e-6, y_out=None, embed=None):
    """flax nn.LayerNorm (eps 1e-6); returns (y bf16, mean f32 [T], rstd f32 [T]).
    ``y_out``: preallocated y (e.g. rows of a deferred-weight-gradient arena).
    ``embed`` = (tok, wte, wpe, S): ``x`` is an output -- it receives the token +
    position embedding (``embed_fwd``'s values) and y = LN(x); on the GPU one launch
    (csrc/layernorm.hip ``jdt_ln_fwd_embed``)."""
    T, d = x.shape
    if embed is not None and _is_gpu(x):
        tok, wte, wpe, S = embed
        assert tok.dtype == torch.int32 and tok.shape == (T,) and wte.shape[1] == d == wpe.shape[1]
        assert x.is_contiguous() and wte.is_contiguous() and wpe.is_contiguous() and tok.is_contiguous()
        y = torch.empty_like(x) if y_out is None else y_out
        assert y.stride(1) == 1 and y.shape == x.shape and y.stride(0) == d
        mean = torch.empty(T, dtype=torch.float32, device=x.device)
        rstd = torch.empty(T, dtype=torch.float32, device=x.device)
        rc = _lib.lib().jdt_ln_fwd_embed(_ptr(tok), _ptr(wte), _ptr(wpe), int(S), _ptr(x), _ptr(gamma), _ptr(beta),
                                         _ptr(y), _ptr(mean), _ptr(rstd), T, d, float(eps), _lib.stream_ptr())
        _lib.check(rc, "jdt_ln_fwd_embed")
        return y, mean, rstd
    if embed is not None:
        embed_fwd(*embed, out=x)
    if not _is_gpu(x):
        xf = x.float()
        mean = xf.mean(-1)
        rstd = torch.rsqrt(((xf - mean[:, None]) ** 2).mean(-1) + eps)
        y = ((xf - mean[:, None]) * rstd[:, None] * gamma.float() + beta.float()).to(torch.bfloat16)
        if y_out is not None:
            y = y_out.copy_(y)
        return y, mean, rstd
    y = torch.empty_like(x) if y_out is None else y_out
    assert y.stride(1) == 1 and y.shape == x.shape
    mean = torch.empty(T, dtype=torch.float32, device=x.device)
    rstd = torch.empty(T, dtype=torch.float32, device=x.device)
    rc = _lib.lib().jdt_ln_fwd(_ptr(x), _ptr(gamma), _ptr(beta), _ptr(y), _ptr(mean), _ptr(rstd), T, d, float(eps),
                               _lib.stream_ptr())
    _lib.check(rc, "jdt_ln_fwd")
    return y, mean, rstd


_LN_GEMM = os.environ.get("JDT_LN_GEMM", "1") != "0"


def ln_gemm(x, gamma, beta, w, *, eps=1e-6, bias=None, act: str = "none", z_out=None, keep_prob: float = 1.0,
            seed: int = 0, offset: int = 0, step=None, y_out=None, out=None, embed=None):
    """``gemm(LN(x), w, ...)`` with the LayerNorm fused into the GEMM's A operand
    (csrc/gemm.hip ``gemm_ln_kernel``): returns (C, y = LN(x) bf16, mean, rstd) --
    the same values as ``layernorm_fwd`` followed by ``gemm`` (bit-identical y),
    one launch instead of two.  ``w`` is the [K, N] ("kn") bf16 weight.  Shapes
    outside the fused kernel's envelope (or JDT_LN_GEMM=0, or CPU) run the two ops.
    ``y_out`` / ``out``: preallocated LN(x) / C (deferred weight-gradient arena rows).
    ``embed`` = (tok, wte, wpe, S): ``x`` is an output that receives the embedding
    first (the model's first block): folded into the LayerNorm launch where the LN
    runs apart (``layernorm_fwd(embed=)``), a separate ``embed_fwd`` before the fused
    kernel."""
    T, d = x.shape
    N = w.shape[-1]
    if _is_gpu(x) and _LN_GEMM and w.dtype == torch.bfloat16 and x.dtype == torch.bfloat16:
        y = torch.empty_like(x) if y_out is None else y_out
        mean = torch.empty(T, dtype=torch.float32, device=x.device)
        rstd = torch.empty(T, dtype=torch.float32, device=x.device)
        if out is None:
            out = torch.empty(T, N, dtype=torch.bfloat16, device=x.device)
        assert y.shape == x.shape and out.shape == (T, N) and out.dtype == torch.bfloat16
        g = _lib.GemmArgs()
        g.A, g.lda = y.data_ptr(), y.stride(0)
        g.B, g.ldb, g.b_trans = w.data_ptr(), w.stride(0), 1
        g.M, g.N, g.K, g.alpha = T, N, d, 1.0
        if bias is not None:
            assert bias.is_contiguous()
            g.bias, g.bias_f32 = bias.data_ptr(), int(bias.dtype == torch.float32)
        g.act = ACT[act]
        if z_out is not None:
            assert z_out.dtype == torch.bfloat16 and z_out.stride(-1) == 1
            g.Zout, g.ldz = z_out.data_ptr(), z_out.stride(0)
        g.keep_prob, g.seed, g.offset = float(keep_prob), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1)
        g.C, g.ldc = out.data_ptr(), out.stride(0)
        if step is not None:
            assert step.dtype == torch.int32
            g.step_ptr = step.data_ptr()
        L = _lib.LnArgs()
        L.X, L.ldx = x.data_ptr(), x.stride(0)
        L.gamma, L.beta, L.eps = gamma.data_ptr(), beta.data_ptr(), float(eps)
        L.Y, L.ldy, L.mean, L.rstd = y.data_ptr(), y.stride(0), mean.data_ptr(), rstd.data_ptr()
        assert x.stride(1) == 1 and w.stride(1) == 1 and gamma.dtype == beta.dtype == torch.float32
        fused = _lib.lib().jdt_gemm_ln_eligible(ctypes.byref(g), ctypes.byref(L))
        if fused and embed is not None:
            embed_fwd(*embed, out=x)
            embed = None
        rc = _lib.lib().jdt_gemm_ln(ctypes.byref(g), ctypes.byref(L), _lib.stream_ptr()) if fused else -2
        if rc != -2:
            _lib.check(rc, "jdt_gemm_ln")
            return out, y, mean, rstd
    y, mean, rstd = layernorm_fwd(x, gamma, beta, eps, y_out=y_out, embed=embed)
    out = gemm(y, w, bias=bias, act=act, z_out=z_out, keep_prob=keep_prob, seed=seed, offset=offset, step=step,
               out=out)
    return out, y, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, dres=None, dsum=None, dx_out=None):
    """dx = dres + LN'(dy); dgamma/dbeta accumulate (fp32); ``dsum += colsum(dx)``
    (the bias grad of the residual-stream Dense that produced x, fused here).
    ``dx_out``: preallocated dx (deferred weight-gradient arena rows)."""
    T, d = x.shape
    if not _is_gpu(x):
        xh = (x.float() - mean[:, None]) * rstd[:, None]
        g = dy.float() * gamma.float()
        dx = rstd[:, None] * (g - g.mean(-1, keepdim=True) - xh * (g * xh).mean(-1, keepdim=True))
        if dres is not None:
            dx = dx + dres.float()
        if dgamma is not None:
            dgamma.add_((dy.float() * xh).sum(0))
        if dbeta is not None:
            dbeta.add_(dy.float().sum(0))
        dx = dx.to(torch.bfloat16)
        if dx_out is not None:
            dx = dx_out.copy_(dx)
        if dsum is not None:
            dsum.add_(dx.float().sum(0))
        return dx
    dx = torch.empty_like(x) if dx_out is None else dx_out
    assert dx.is_contiguous() and dx.shape == x.shape
    rc = _lib.lib().jdt_ln_bwd(_ptr(dy), _ptr(x), _ptr(mean), _ptr(rstd), _ptr(gamma), _ptr(dres), _ptr(dx),
                               _ptr(dgamma), _ptr(dbeta), _ptr(dsum), T, d, _lib.stream_ptr())
    _lib.check(rc, "jdt_ln_bwd")
    return dx


def embed_fwd(tok, wte, wpe, S, out=None):
    T = tok.shape[0]
    d = wte.shape[1]
    if not _is_gpu(tok):
        pos = torch.arange(T) % S
        e = (wte.float()[tok.long()] + wpe.float()[pos]).to(torch.bfloat16)
        return e if out is None else out.copy_(e)
    if out is None:
        out = torch.empty(T, d, dtype=torch.bfloat16, device=tok.device)
    assert out.shape == (T, d) and out.is_contiguous() and out.dtype == torch.bfloat16
    rc = _lib.lib().jdt_embed_fwd(_ptr(tok), _ptr(wte), _ptr(wpe), _ptr(out), T, S, d, _lib.stream_ptr())
    _lib.check(rc, "jdt_embed_fwd")
    return out


def embed_bwd(dout, tok, dwte, dwpe, S):
    T, d = dout.shape
    if not _is_gpu(dout):
        dwte.index_add_(0, tok.long(), dout.float())
        if dwpe is not None:
            dwpe.index_add_(0, torch.arange(T) % S, dout.float())
        return
    rc = _lib.lib().jdt_embed_bwd(_ptr(dout), _ptr(tok), _ptr(dwte), _ptr(dwpe), T, S, d, _lib.stream_ptr())
    _lib.check(rc, "jdt_embed_bwd")


def colsum_(x, out):
    """out += x.sum(0) (bias gradients)."""
    if not _is_gpu(x):
        out.add_(x.float().sum(0))
        return out
    rc = _lib.lib().jdt_colsum(_ptr(x), x.stride(0), x.shape[0], x.shape[1], _ptr(out), _lib.stream_ptr())
    _lib.check(rc, "jdt_colsum")
    return out
