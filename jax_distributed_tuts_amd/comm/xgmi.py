"""Direct xGMI peer-to-peer collectives (comm/csrc/xgmi.hip) for one node.

``XgmiComm(mesh, axis, cap_floats)`` gives the ranks of one mesh axis a
private set of IPC-shared device buffers (exported with hipIpcGetMemHandle,
exchanged once over the process group, mapped with hipIpcOpenMemHandle), then
runs the collectives as ordinary kernels on the current stream:

* ``all_reduce_(t)``      -- SUM in place (two-shot: direct reduce-scatter +
                             direct all-gather, every peer on its own link);
* ``all_reduce_adamw_()`` -- the same all-reduce whose gather phase applies
                             AdamW to the parameters and folds the metric slots
                             (the whole DP "sync_grads + apply_gradients +
                             sync_metrics" tail, data_paral.py:206-236, in ONE
                             kernel);
* ``reduce_scatter`` / ``all_gather`` -- tiled along a flat dim-0 layout
                             (FSDP X05/X06).

Being kernels rather than RCCL calls, they are captured into hipGraphs with
the rest of the step, so a multi-GPU step is a single graph replay.

Construction runs a self-test on the real hardware (``_self_test``: 32
skewed-arrival all-reduces over three sizes and both buffer parities, RS / AG,
the segmented FSDP kernels and the fused-AdamW variant, all exact, and
bit-compared with RCCL when the group is nccl) and all ranks agree on the
outcome; ``comm.ok`` is False (and the trainers fall back to RCCL) if the IPC
mapping or the self-test fails on any rank.  Every in-kernel wait has a
timeout, so a dead peer turns into an error flag (``error()``) instead of a
hung GPU.
"""
from __future__ import annotations

import ctypes
import logging
import os
from ctypes import c_float, c_int, c_long, c_longlong, c_void_p
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _lib

log = logging.getLogger(__name__)

HANDLE_BYTES = 64
TICKS_PER_S = 100_000_000  # s_memrealtime


def xg_wt() -> int:
    """JDT_XG_WT: the fused AdamW of the xGMI kernels stores p / m / v / shadow
    write-through (1) or plain (0) -- the kernel boundary then has fewer dirty L2 lines
    to write back (the md_bwd / run-ahead mlp2_bwd switch, profiles/r4_write_through_ab.txt)."""
    return int(os.environ.get("JDT_XG_WT", "0"))


class XgAdam(ctypes.Structure):
    """Mirror of ``jdt::XgAdam`` (comm/csrc/xgmi.hip)."""

    _fields_ = [
        ("p", c_void_p), ("m", c_void_p), ("v", c_void_p), ("shadow", c_void_p),
        ("n_params", c_long), ("running", c_void_p), ("n_metrics", c_int),
        ("lr", c_float), ("b1", c_float), ("b2", c_float), ("eps", c_float), ("wd", c_float),
        ("grad_scale", c_float), ("step", c_void_p), ("ticket", c_void_p), ("zero", c_void_p),
        ("hold", c_int), ("wt", c_int),
    ]


class XgSeg(ctypes.Structure):
    _fields_ = [("full", c_void_p), ("part", c_void_p), ("s", c_long), ("off", c_long), ("nfull", c_long),
                ("bcast", c_long), ("rows", c_long), ("ld", c_long), ("qoff", c_long)]


MAX_SEGS = 16


class XgSegs(ctypes.Structure):
    """Mirror of ``jdt::XgSegs``: up to 16 (full, part) tensors per launch."""

    _fields_ = [("seg", XgSeg * MAX_SEGS), ("n", c_int), ("S", c_long)]


class XgFsdp(ctypes.Structure):
    """Mirror of ``jdt::XgFsdp``: local AdamW buffers + per-segment kind / bf16 full shadow."""

    _fields_ = [("A", XgAdam), ("grad", c_void_p), ("kind", c_int * MAX_SEGS), ("full_shadow", c_void_p * MAX_SEGS),
                ("stamps", c_void_p), ("staged", c_int)]


FSDP_SHARD, FSDP_REPL, FSDP_METRIC = 0, 1, 2

_lib.declare("jdt_xgmi_fsdp_size", c_int, [])
_lib.declare("jdt_xgmi_fsdp_step", c_int, [c_void_p, ctypes.POINTER(XgSegs), ctypes.POINTER(XgFsdp), c_longlong,
                                           c_void_p])
_lib.declare("jdt_xgmi_create", c_int, [c_int, c_int, c_long, ctypes.POINTER(c_void_p), c_void_p])
_lib.declare("jdt_xgmi_open", c_int, [c_void_p, c_void_p])
_lib.declare("jdt_xgmi_allreduce", c_int, [c_void_p, c_void_p, c_void_p, c_long, ctypes.POINTER(XgAdam), c_longlong,
                                           c_void_p])
_lib.declare("jdt_xgmi_set_oneshot_bytes", None, [c_long])
_lib.declare("jdt_xgmi_oneshot_bytes", c_long, [])
_lib.declare("jdt_xgmi_reduce_scatter", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_long, c_longlong, c_void_p])
_lib.declare("jdt_xgmi_all_gather", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_long, c_longlong, c_void_p])
_lib.declare("jdt_xgmi_segments", c_int, [c_void_p, ctypes.POINTER(XgSegs), c_int, c_int, c_longlong, c_void_p])
_lib.declare("jdt_xgmi_segs_size", c_int, [])
_lib.declare("jdt_xgmi_capacity", c_long, [c_void_p])
_lib.declare("jdt_xgmi_adam_size", c_int, [])
_lib.declare("jdt_xgmi_error", c_int, [c_void_p])
_lib.declare("jdt_xgmi_error_info", c_int, [c_void_p, c_void_p])
_lib.declare("jdt_xgmi_stage_part", c_long, [c_void_p, c_long])
_lib.declare("jdt_xgmi_stage_base", c_void_p, [c_void_p])
_lib.declare("jdt_xgmi_stage_write", c_int, [c_void_p, c_int, c_void_p, c_long, c_void_p])
_lib.declare("jdt_xgmi_stage_clear", c_int, [c_void_p, c_void_p])
_lib.declare("jdt_xgmi_allreduce_staged", c_int, [c_void_p, c_long, c_long, ctypes.POINTER(XgAdam), c_longlong,
                                                  c_void_p])
_lib.declare("jdt_xgmi_destroy", c_int, [c_void_p])
_lib.declare("jdt_xgmi_unmap", c_int, [c_void_p])


def ipc_teardown_barrier(group):
    """The barrier between the two phases of a comm context's teardown: every rank of
    ``group`` has closed its mappings of the peers' buffers before any rank releases its
    own (a gloo group's barrier runs on the host; nccl's on the device)."""
    if group is None or not dist.is_initialized():
        return
    if dist.get_backend(group) == "nccl":
        from ..runtime.dist import device

        dist.barrier(group=group, device_ids=[device().index])
    else:
        dist.barrier(group=group)
_lib.declare("jdt_xgmi_seg_slice", c_long, [c_long])
_lib.declare("jdt_ipc_pool_stats", None, [c_void_p])


def ipc_pool_stats() -> dict:
    """Census of this process's pool of IPC-exported buffers (comm/csrc/ipc_pool.hip):
    every comm context (xGMI, p2p inboxes, tile exchange) takes its exported buffers
    from it and returns them there, never to the driver."""
    out = (ctypes.c_long * 3)()
    _lib.lib().jdt_ipc_pool_stats(out)
    return {"buffers": int(out[0]), "bytes": int(out[1]), "in_use": int(out[2])}


def _ptr(t: Optional[torch.Tensor]):
    return c_void_p(t.data_ptr()) if t is not None else c_void_p(0)


def part_len(n: int, world: int) -> int:
    """Per-rank part of an n-float all-reduce (multiple of 4 floats)."""
    return ((n + world - 1) // world + 3) // 4 * 4


XG_MAX_BLOCKS, XG_THREADS = 96, 256   # comm/csrc/xgmi.hip
_lib.declare("jdt_xgmi_set_max_blocks", None, [c_int])
_lib.declare("jdt_xgmi_max_blocks", c_int, [])


def max_blocks() -> int:
    """The kernels' current grid cap (``xg_geometry``; lowered when ranks share a GPU)."""
    return int(_lib.lib().jdt_xgmi_max_blocks())


def set_max_blocks(b: int) -> None:
    _lib.lib().jdt_xgmi_set_max_blocks(int(b))


def size_grids_for_sharing(device: torch.device) -> int:
    """With k ranks time-sharing this GPU, cap every spinning xGMI grid at
    CUs / (2 k) workgroups (>= 8): k ranks' waiting collectives then occupy at most half
    the CUs' workgroup slots, so a peer's non-spinning kernels (md_fwd / md_bwd, GEMMs)
    always find room to run and reach the barrier (tests at 8 shared ranks).  One rank
    per GPU keeps the full 96.  Collective (ranks_per_gpu); returns the cap."""
    from ..runtime.dist import ranks_per_gpu

    k = ranks_per_gpu()
    if k > 1:
        cus = torch.cuda.get_device_properties(device).multi_processor_count
        set_max_blocks(max(8, min(XG_MAX_BLOCKS, cus // (2 * k))))
    return max_blocks()


def geometry(s: int) -> tuple:
    """(blocks, chunk) of a launch over s floats per rank part: mirror of
    ``xg_geometry`` in comm/csrc/xgmi.hip (the host checks ``blocks*chunk*W <= cap``)."""
    g = min(max((s + 4 * XG_THREADS - 1) // (4 * XG_THREADS), 8), max_blocks())
    return g, ((s + g - 1) // g + 3) // 4 * 4


def allreduce_fits(n: int, world: int, cap: int) -> dict:
    """Which all-reduce kernels can take an n-float vector on a context of ``cap``
    floats per buffer half: {"oneshot": bool, "twoshot": bool} (the same launch
    checks as ``xg_oneshot`` / ``xg_launch`` in comm/csrc/xgmi.hip)."""
    n4 = (n + 3) // 4 * 4
    g1, c1 = geometry(n4)
    g2, c2 = geometry(part_len(n, world))
    return {"oneshot": n > 0 and g1 * c1 <= cap, "twoshot": n > 0 and g2 * c2 * world <= cap}


def stage_layout(S: "XgSegs", leaves, world: int) -> dict:
    """{leaf name: (packed offset, dim, per, cols)} + "metrics" -- the common.h StageMap
    leaves of a fused FSDP plan's segment table ``S`` (sharded leaves, replicated leaves,
    then the metric slots): dim 0 = row shards of ``per`` rows, 1 = column shards of
    ``per`` columns, 2 = the whole leaf in every peer slot."""
    out = {}
    for k, (name, shape, d) in enumerate(leaves):
        g = S.seg[k]
        cols = int(shape[-1]) if len(shape) == 2 else 1
        if d is None:
            out[name] = (int(g.off), 2, 1, cols)
        elif d == 0:
            out[name] = (int(g.off), 0, int(shape[0]) // world, cols)
        else:
            out[name] = (int(g.off), 1, int(shape[1]) // world, cols)
    out["metrics"] = (int(S.seg[len(leaves)].off), 2, 1, 1)
    return out


def requested(mode: str, world: int, device: torch.device) -> bool:
    """Whether a trainer should try the xGMI path: ``mode`` in {"auto","xgmi","rccl"}
    (env ``JDT_COMM`` overrides "auto")."""
    if mode == "auto":
        mode = os.environ.get("JDT_COMM", "auto")
    if mode == "rccl" or world < 2 or world > 8 or device.type != "cuda":
        return False
    return True


class XgmiComm:
    _serial = 0   # contexts created in this process (self-test failure logs)

    def __init__(self, group, rank: int, world: int, cap_floats: int, device: torch.device,
                 timeout_s: float = 30.0, self_test: bool = True):
        XgmiComm._serial += 1
        self.group, self.rank, self.world, self.device = group, rank, world, device
        self.timeout = c_longlong(int(timeout_s * TICKS_PER_S))
        self.ctx = c_void_p()
        self.ok = False
        L = _lib.lib()
        if (L.jdt_xgmi_adam_size() != ctypes.sizeof(XgAdam) or L.jdt_xgmi_segs_size() != ctypes.sizeof(XgSegs)
                or L.jdt_xgmi_fsdp_size() != ctypes.sizeof(XgFsdp)):
            raise RuntimeError("XgAdam layout mismatch between Python and comm/csrc/xgmi.hip")
        h = (ctypes.c_char * (3 * HANDLE_BYTES))()
        with torch.cuda.device(device):
            rc = L.jdt_xgmi_create(rank, world, int(cap_floats), ctypes.byref(self.ctx), h)
        mine = bytes(h) if rc == 0 else None
        objs = [None] * world
        dist.all_gather_object(objs, mine, group=group)
        good = all(o is not None for o in objs)
        if good:
            allh = b"".join(objs)
            buf = ctypes.create_string_buffer(allh, len(allh))
            with torch.cuda.device(device):
                rc = L.jdt_xgmi_open(self.ctx, buf)
            good = rc == 0
            if not good:
                log.warning("xgmi: hipIpcOpenMemHandle failed on rank %d (rc %d)", rank, rc)
        else:
            log.warning("xgmi: buffer export failed on some rank (rank %d rc %d)", rank, rc)
        good = self._agree(good)
        if good and self_test:
            good = self._agree(self._self_test())
        self.ok = good
        if not good:
            self.close()

    # ------------------------------------------------------------------ plumbing
    def _agree(self, ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                         device=self.device if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))

    @property
    def capacity(self) -> int:
        return int(_lib.lib().jdt_xgmi_capacity(self.ctx)) if self.ctx else 0

    def fits(self, n: int) -> dict:
        """{"oneshot", "twoshot"}: whether each all-reduce kernel takes n floats here."""
        return allreduce_fits(int(n), self.world, self.capacity)

    def max_allreduce(self) -> int:
        """Largest n (multiple of 4) the two-shot all-reduce takes on this context."""
        lo, hi = 0, self.capacity
        while lo < hi:   # fits() is monotone in n up to padding steps: bisect, then step down
            mid = (lo + hi + 1) // 2
            if self.fits(mid)["twoshot"]:
                lo = mid
            else:
                hi = mid - 1
        while lo > 0 and not self.fits(lo)["twoshot"]:
            lo -= 1
        return lo // 4 * 4
    def error(self) -> int:
        """1 if any in-kernel barrier timed out on this rank (synchronises the device)."""
        return int(_lib.lib().jdt_xgmi_error(self.ctx)) if self.ctx else 0

    SITES = {1: "two-shot all-reduce", 2: "one-shot all-reduce", 3: "segmented RS/AG", 4: "fused FSDP step"}

    def error_info(self) -> Optional[dict]:
        """Where this rank's first barrier timeout happened (None if none): kernel,
        barrier (0: after staging, 1: after the reduce), block, awaited epoch and the
        peer that never signalled."""
        if not self.ctx or not self.error():
            return None
        out = (ctypes.c_uint * 4)()
        _lib.check(_lib.lib().jdt_xgmi_error_info(self.ctx, out), "jdt_xgmi_error_info")
        site, blk, ep, q = (int(v) for v in out)
        return {"kernel": self.SITES.get(site // 2, f"site {site}"), "barrier": site % 2, "block": blk, "epoch": ep,
                "silent_peer": q, "rank": self.rank, "world": self.world}

    def raise_if_error(self):
        """RuntimeError naming the timed-out barrier if any in-kernel wait of this rank
        timed out (a peer dead, desynchronised or not scheduled)."""
        info = self.error_info()
        if info is not None:
            raise RuntimeError(f"xgmi collective timed out on this rank (peer dead or desynchronised): {info}")

    def close(self, collective: bool = True):
        """Two-phase teardown (collective over the context's group): every rank closes its
        mappings of the peers' buffers, a barrier, then every rank releases its own -- no
        peer mapping outlives the pages it resolves to (comm/csrc/ipc_pool.hip).
        ``collective=False`` (garbage collection): one phase, this rank only."""
        if self.ctx:
            if collective:
                _lib.lib().jdt_xgmi_unmap(self.ctx)
                ipc_teardown_barrier(self.group)
            _lib.lib().jdt_xgmi_destroy(self.ctx)
            self.ctx = c_void_p()
        self.ok = False

    def __del__(self):
        try:
            self.close(collective=False)
        except Exception:
            pass

    @staticmethod
    def _check_f32(t: torch.Tensor):
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.data_ptr() % 16:
            raise ValueError("xgmi collectives take contiguous, 16-byte aligned fp32 CUDA tensors")

    # ------------------------------------------------------------------ collectives
    @staticmethod
    def set_oneshot_bytes(nbytes: int):
        """All-reduces up to ``nbytes`` (default 256 KiB, env JDT_XGMI_ONESHOT_BYTES) run
        the one-shot kernel (one barrier, every rank reads the whole vector from each
        peer); larger ones the two-shot reduce-scatter + all-gather kernel."""
        _lib.lib().jdt_xgmi_set_oneshot_bytes(int(nbytes))

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        self._check_f32(t)
        rc = _lib.lib().jdt_xgmi_allreduce(self.ctx, _ptr(t), _ptr(t), t.numel(), None, self.timeout,
                                           c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_xgmi_allreduce")
        return t

    def all_reduce_adamw_(self, grad: torch.Tensor, *, p: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                          shadow: Optional[torch.Tensor], n_params: int, running: Optional[torch.Tensor],
                          n_metrics: int, lr: float, b1: float, b2: float, eps: float, wd: float,
                          grad_scale: float, step: torch.Tensor, ticket: torch.Tensor, zero_grad: bool = True,
                          advance: bool = True):
        """SUM-all-reduce ``grad`` and, in the same kernel, AdamW on ``p[:n_params]``
        (grads scaled by ``grad_scale``: the 1/(n_mb*N) mean) and
        ``running[j] += grad_sum[n_params + j]`` for the metric slots.  ``advance=False``:
        leave the step counter to a later call of the same step (per-bucket calls; every
        call of a step reads the same step for the bias correction)."""
        self._check_f32(grad)
        a = XgAdam()
        a.wt = xg_wt()
        a.p, a.m, a.v, a.shadow = _ptr(p), _ptr(m), _ptr(v), _ptr(shadow)
        a.n_params, a.running, a.n_metrics = int(n_params), _ptr(running), int(n_metrics if running is not None else 0)
        a.lr, a.b1, a.b2, a.eps, a.wd, a.grad_scale = float(lr), float(b1), float(b2), float(eps), float(wd), float(grad_scale)
        a.step, a.ticket = _ptr(step), _ptr(ticket)
        a.zero = _ptr(grad) if zero_grad else c_void_p(0)
        a.hold = 0 if advance else 1
        rc = _lib.lib().jdt_xgmi_allreduce(self.ctx, _ptr(grad), c_void_p(0), grad.numel(), ctypes.byref(a),
                                           self.timeout, c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_xgmi_allreduce(adamw)")

    # ------------------------------------------------------------------ staged (producer-written) bucket
    def stage_plan(self, n: int) -> Optional[dict]:
        """Geometry for a producer kernel that writes an n-float bucket straight into
        this rank's staging buffer (identity layout, half = optimizer step parity):
        {"s": part length, "base": pointer of half 0, "stride": floats to half 1}, or
        None if the bucket does not fit an unpadded split."""
        s = int(_lib.lib().jdt_xgmi_stage_part(self.ctx, int(n)))
        if s <= 0:
            return None
        return {"s": s, "n": int(n), "base": int(_lib.lib().jdt_xgmi_stage_base(self.ctx)), "stride": self.capacity}

    def stage_clear(self):
        _lib.check(_lib.lib().jdt_xgmi_stage_clear(self.ctx, c_void_p(_lib.stream_ptr())), "jdt_xgmi_stage_clear")

    def stage_write(self, parity: int, src: torch.Tensor):
        self._check_f32(src)
        _lib.check(_lib.lib().jdt_xgmi_stage_write(self.ctx, int(parity), _ptr(src), src.numel(),
                                                   c_void_p(_lib.stream_ptr())), "jdt_xgmi_stage_write")

    def all_reduce_adamw_staged_(self, plan: dict, *, p: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                                 shadow: Optional[torch.Tensor], n_params: int, running: Optional[torch.Tensor],
                                 n_metrics: int, lr: float, b1: float, b2: float, eps: float, wd: float,
                                 grad_scale: float, step: torch.Tensor, ticket: torch.Tensor):
        """``all_reduce_adamw_`` of the bucket a producer staged (``stage_plan``): no
        staging copy; the producer and this kernel pick the buffer half from the
        parity of ``step`` (the optimizer counter this kernel advances)."""
        a = XgAdam()
        a.wt = xg_wt()
        a.p, a.m, a.v, a.shadow = _ptr(p), _ptr(m), _ptr(v), _ptr(shadow)
        a.n_params, a.running, a.n_metrics = int(n_params), _ptr(running), int(n_metrics if running is not None else 0)
        a.lr, a.b1, a.b2, a.eps, a.wd, a.grad_scale = float(lr), float(b1), float(b2), float(eps), float(wd), float(grad_scale)
        a.step, a.ticket = _ptr(step), _ptr(ticket)
        a.zero = c_void_p(0)
        rc = _lib.lib().jdt_xgmi_allreduce_staged(self.ctx, plan["n"], plan["s"], ctypes.byref(a), self.timeout,
                                                  c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_xgmi_allreduce_staged")

    def reduce_scatter(self, full: torch.Tensor, out: torch.Tensor, part: int) -> torch.Tensor:
        """out[0:part] = sum over ranks of full[rank*part : (rank+1)*part] (valid to full.numel())."""
        self._check_f32(full)
        self._check_f32(out)
        rc = _lib.lib().jdt_xgmi_reduce_scatter(self.ctx, _ptr(full), _ptr(out), full.numel(), int(part),
                                                self.timeout, c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_xgmi_reduce_scatter")
        return out

    def all_gather(self, part_t: torch.Tensor, out: torch.Tensor, part: int) -> torch.Tensor:
        """out[q*part : (q+1)*part] = rank q's part_t (valid to out.numel())."""
        self._check_f32(part_t)
        self._check_f32(out)
        rc = _lib.lib().jdt_xgmi_all_gather(self.ctx, _ptr(part_t), _ptr(out), out.numel(), int(part),
                                            self.timeout, c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_xgmi_all_gather")
        return out

    # ------------------------------------------------------------------ segmented (multi-tensor) RS / AG
    @staticmethod
    def segment_ok(full: torch.Tensor, part: torch.Tensor, world: int) -> bool:
        """Whether (full, part) is a shard pair the segmented kernel can move: contiguous,
        16-byte aligned, full = world parts -- along dim 0 (part a multiple of 16 bytes)
        or, 2-D, along dim 1 (each part row a multiple of 16 bytes)."""
        es = part.element_size()
        base = (full.is_cuda and part.is_cuda and full.dtype == part.dtype and full.is_contiguous()
                and part.is_contiguous() and full.data_ptr() % 16 == 0 and part.data_ptr() % 16 == 0
                and full.numel() == world * part.numel())
        if not base:
            return False
        if XgmiComm._dim1(full, part, world):
            return (part.shape[1] * es) % 16 == 0
        return (part.numel() * es) % 16 == 0

    @staticmethod
    def _dim1(full: torch.Tensor, part: torch.Tensor, world: int) -> bool:
        """A 2-D pair sharded along dim 1 (rank q's part = full[:, q*w:(q+1)*w])."""
        return (full.dim() == 2 and part.dim() == 2 and full.shape[0] == part.shape[0] > 1
                and full.shape[1] == world * part.shape[1])

    def _segs(self, pairs, allreduce=()) -> XgSegs:
        if not 0 < len(pairs) + len(allreduce) <= MAX_SEGS:
            raise ValueError(f"1..{MAX_SEGS} segments per launch")
        S = XgSegs()
        off = 0
        for k, (full, part) in enumerate(pairs):
            if not self.segment_ok(full, part, self.world):
                raise ValueError("segment is not a contiguous, 16-byte aligned dim-0 shard pair")
            es = part.element_size()
            w = part.numel() * es // 4
            nfull = full.numel() * es // 4
            if self._dim1(full, part, self.world):
                rows, pw = part.shape[0], part.shape[1] * es // 4
                S.seg[k] = XgSeg(full.data_ptr(), part.data_ptr(), w, off, nfull, 0, rows, full.shape[1] * es // 4, pw)
            else:
                S.seg[k] = XgSeg(full.data_ptr(), part.data_ptr(), w, off, nfull, 0, 0, 0, 0)
            off += w
        for k, t in enumerate(allreduce, start=len(pairs)):
            if (t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous() or t.data_ptr() % 16
                    or t.numel() % 4):
                raise ValueError("all-reduce segments are contiguous, 16-byte aligned fp32, length % 4 == 0")
            S.seg[k] = XgSeg(t.data_ptr(), t.data_ptr(), t.numel(), off, t.numel(), 1, 0, 0, 0)
            off += t.numel()
        S.n, S.S = len(pairs) + len(allreduce), off
        return S

    def all_gather_segments(self, pairs):
        """For each (full, part): full[q*len(part) : (q+1)*len(part)] = rank q's part.
        Any dtype (moved as 4-byte words); one kernel for all pairs."""
        for i in range(0, len(pairs), MAX_SEGS):
            S = self._segs(pairs[i:i + MAX_SEGS])
            rc = _lib.lib().jdt_xgmi_segments(self.ctx, ctypes.byref(S), 2, 0, self.timeout,
                                              c_void_p(_lib.stream_ptr()))
            _lib.check(rc, "jdt_xgmi_segments(all_gather)")

    def reduce_scatter_segments(self, pairs, accumulate: bool = False, allreduce=()):
        """For each fp32 (full, part): part (+)= sum over ranks of full[rank*len(part) : ...].
        ``allreduce``: fp32 tensors all-reduced in place (sum, never accumulated) in the
        same launch -- one collective instead of two."""
        for full, part in pairs:
            if full.dtype != torch.float32:
                raise ValueError("reduce-scatter sums fp32 tensors")
        allreduce = list(allreduce)
        if len(pairs) + len(allreduce) > MAX_SEGS:
            if allreduce:
                raise ValueError(f"at most {MAX_SEGS} segments with all-reduce segments")
        for i in range(0, max(len(pairs), 1), MAX_SEGS):
            S = self._segs(pairs[i:i + MAX_SEGS], allreduce if i == 0 else ())
            rc = _lib.lib().jdt_xgmi_segments(self.ctx, ctypes.byref(S), 1, int(accumulate), self.timeout,
                                              c_void_p(_lib.stream_ptr()))
            _lib.check(rc, "jdt_xgmi_segments(reduce_scatter)")

    # ------------------------------------------------------------------ fused FSDP step collective
    def fsdp_plan(self, shards, replicated, metric_slots, *, grad_base: torch.Tensor, p: torch.Tensor,
                  m: torch.Tensor, v: torch.Tensor, shadow: torch.Tensor, running: torch.Tensor, lr: float,
                  b1: float, b2: float, eps: float, wd: float, grad_scale: float, step: torch.Tensor,
                  ticket: torch.Tensor):
        """Arguments of ONE ``xg_fsdp_kernel`` launch (see comm/csrc/xgmi.hip): ``shards``
        = [(full fp32 grad, local fp32 grad view, full bf16 shadow)] of the sharded
        leaves, ``replicated`` = [(full grad, local grad view, full shadow)], and the
        local metric slots.  The local views must lie in ``grad_base`` (the local flat
        grad buffer), whose offsets index ``p`` / ``m`` / ``v`` / ``shadow``."""
        pairs = [(f, l) for f, l, _ in shards]
        n = len(pairs) + len(replicated) + 1
        if n > MAX_SEGS:
            raise ValueError(f"at most {MAX_SEGS} segments in one FSDP step launch")
        S = self._segs(pairs)   # validates the shard pairs (dim-0 / dim-1 layouts)
        off = S.S
        F = XgFsdp()
        for k, (_, _, fs) in enumerate(shards):
            F.kind[k] = FSDP_SHARD
            F.full_shadow[k] = fs.data_ptr()
        k = len(pairs)
        for full, part, fs in replicated:
            if not (full.is_contiguous() and part.is_contiguous() and full.numel() == part.numel()
                    and full.data_ptr() % 16 == 0 and part.data_ptr() % 16 == 0 and fs.data_ptr() % 8 == 0):
                raise ValueError("replicated leaf views must be contiguous and aligned")
            w = (full.numel() + 3) // 4 * 4
            S.seg[k] = XgSeg(full.data_ptr(), part.data_ptr(), w, off, full.numel(), 1, 0, 0, 0)
            F.kind[k], F.full_shadow[k] = FSDP_REPL, fs.data_ptr()
            off += w
            k += 1
        ms = metric_slots
        w = (ms.numel() + 3) // 4 * 4
        S.seg[k] = XgSeg(ms.data_ptr(), ms.data_ptr(), w, off, ms.numel(), 1, 0, 0, 0)
        F.kind[k] = FSDP_METRIC
        off += w
        S.n, S.S = k + 1, off
        a = F.A
        a.wt = xg_wt()
        a.p, a.m, a.v, a.shadow = _ptr(p), _ptr(m), _ptr(v), _ptr(shadow)
        a.n_params, a.running, a.n_metrics = 0, _ptr(running), int(ms.numel())
        a.lr, a.b1, a.b2, a.eps, a.wd, a.grad_scale = (float(lr), float(b1), float(b2), float(eps), float(wd),
                                                       float(grad_scale))
        a.step, a.ticket, a.zero = _ptr(step), _ptr(ticket), c_void_p(0)
        F.grad = _ptr(grad_base)
        return S, F

    def fsdp_stage_layout(self, plan, leaves) -> dict:
        """Where a producer kernel writes each gradient element for a STAGED fused FSDP
        step (common.h StageMap): ``leaves`` = [(name, full shape, shard dim or None)] in
        the plan's segment order (sharded leaves, then replicated ones), then the metric
        slots.  Returns {name: (packed offset, dim, per, cols)} plus "metrics", and
        "base" / "half" / "slice" of this rank's staging buffer."""
        S, _F = plan
        out = stage_layout(S, leaves, self.world)
        out["base"] = int(_lib.lib().jdt_xgmi_stage_base(self.ctx))
        out["half"] = self.capacity
        out["slice"] = int(_lib.lib().jdt_xgmi_seg_slice(int(S.S)))
        return out

    def fsdp_step(self, plan):
        S, F = plan
        rc = _lib.lib().jdt_xgmi_fsdp_step(self.ctx, ctypes.byref(S), ctypes.byref(F), self.timeout,
                                           c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_xgmi_fsdp_step")

    # ------------------------------------------------------------------ self-test
    SELF_TEST_ITERS = 32

    def _self_test(self) -> bool:
        """Exact checks of every kernel on this hardware before any trainer uses it.

        * ``SELF_TEST_ITERS`` all-reduces cycling over several sizes -- the DP bucket
          (407,054 floats: 1.63 MB of grads + 4 metric slots), a 300,001-float
          buffer, a 4,099-float one -- so both epoch parities are reused many times
          at every size (a stale peer line from an earlier same-parity call would
          show up as a wrong sum);
        * ranks arrive skewed: before every collective each rank spins for a
          rank- and iteration-dependent time (uneven load is what exposes
          visibility bugs, MI355X_MICROARCH.md);
        * reduce-scatter and all-gather at two sizes, the segmented (FSDP) kernels
          on the tutorial's shard shapes, and the fused-AdamW all-reduce against
          the same AdamW computed by torch on the summed gradient;
        * integer-valued data, so sums are exact: results must be bit-identical to
          the expected values and, when the group is nccl, to RCCL's all-reduce of
          the same data.
        Runs with a short barrier timeout (the ranks were just synchronised by the
        handle exchange) and stops at the first failure."""
        saved = self.timeout
        self.timeout = c_longlong(int(5.0 * TICKS_PER_S))
        try:
            with torch.cuda.device(self.device):
                ok = self._self_test_body()
            return ok
        except Exception as e:  # a launch error must not leave the other ranks waiting
            log.warning("xgmi self-test raised: %s", e)
            return False
        finally:
            self.timeout = saved

    def _skew(self, it: int):
        cyc = ((self.rank * 7 + it * 3) % (self.world + 1)) * 20_000
        if cyc:
            torch.cuda._sleep(cyc)

    def _fail(self, what: str) -> bool:
        torch.cuda.synchronize(self.device)
        log.warning("xgmi self-test failed on rank %d: %s%s", self.rank, what,
                    " (barrier timeout)" if self.error() else "")
        return False

    def _diff(self, x: torch.Tensor, want: torch.Tensor, base: torch.Tensor, it: int) -> str:
        """Shape of an all-reduce mismatch for the log: how many elements, where, and
        what the wrong sums decompose into (x - want in units of the per-rank terms: a
        missing rank q shows as -(base * (q + 1) + it))."""
        bad = (x != want).nonzero().flatten()
        if bad.numel() == 0:
            return ""
        i = int(bad[0])
        d = float(x[i] - want[i])
        missing = [q for q in range(self.world) if d == -(float(base[i]) * (q + 1) + it)]
        blk = int(_lib.lib().jdt_xgmi_capacity(self.ctx)) if self.ctx else 0
        return (f"; {bad.numel()} wrong, first {i} last {int(bad[-1])}, got {float(x[i])} want {float(want[i])}"
                f", missing-rank match {missing}, context #{XgmiComm._serial} in this process, cap {blk}")

    def _check(self, bad: bool, what: str) -> bool:
        """Collective verdict of one self-test check: every rank learns whether ANY
        rank failed before anyone issues the next collective (a rank that stopped
        alone would leave the others' next RCCL call paired with its own
        ``_agree`` all-reduce: mismatched collectives on one group)."""
        if bad:
            self._fail(what)
        return self._agree(not bad)

    def _self_test_body(self) -> bool:
        W, r, dev = self.world, self.rank, self.device
        cap = self.capacity
        # the largest two-shot size this context takes (the trainer's own bucket: create_for
        # sizes the context to it), the DP tutorial bucket and two odd sizes
        top = self.max_allreduce()
        sizes = sorted({n for n in (top, 407_054, 300_001, 4_099) if 0 < n <= top}, reverse=True)
        nccl = dist.get_backend(self.group) == "nccl"
        for it in range(self.SELF_TEST_ITERS):
            n = sizes[it % len(sizes)]
            base = (torch.arange(n, device=dev, dtype=torch.int64) % 97).to(torch.float32)
            x = base * (r + 1) + it
            want = base * (W * (W + 1) // 2) + W * it
            ref = x.clone() if (nccl and it % 4 == 0) else None
            self._skew(it)
            self.all_reduce_(x)
            if ref is not None:
                dist.all_reduce(ref, group=self.group)
            torch.cuda.synchronize(dev)
            if not self._check(self.error() or not torch.equal(x, want),
                               f"all-reduce mismatch (iter {it}, n {n}{self._diff(x, want, base, it)})"):
                return False
            if not self._check(ref is not None and not torch.equal(x, ref),
                               f"all-reduce differs from RCCL (iter {it}, n {n})"):
                return False
        for k, n in enumerate(sizes[:2]):
            for rep in range(2):  # both parities
                base = (torch.arange(n, device=dev, dtype=torch.int64) % 89).to(torch.float32)
                want = base * W + W * (W - 1) / 2
                part = part_len(n, W)
                out = torch.empty(part, device=dev)
                self._skew(k + rep)
                self.reduce_scatter(base + r, out, part)
                lo, hi = r * part, min(n, (r + 1) * part)
                torch.cuda.synchronize(dev)
                if not self._check(self.error() or not torch.equal(out[: hi - lo], want[lo:hi]),
                                   f"reduce-scatter mismatch (n {n})"):
                    return False
                full = torch.empty(n, device=dev)
                mine = torch.zeros(part, device=dev)
                mine[: hi - lo] = base[lo:hi] + 1000 * r + rep
                self._skew(k + rep + 1)
                self.all_gather(mine, full, part)
                exp = base.clone()
                for q in range(W):
                    exp[q * part: min(n, (q + 1) * part)] += 1000 * q + rep
                torch.cuda.synchronize(dev)
                if not self._check(self.error() or not torch.equal(full, exp), f"all-gather mismatch (n {n})"):
                    return False
        if not self._self_test_oneshot_burst():
            return False
        if not self._self_test_segments() or not self._self_test_dim1():
            return False
        return self._self_test_adamw()

    def _self_test_oneshot_burst(self) -> bool:
        """Back-to-back one-shot all-reduces (one barrier each, no host sync between
        them) alternating across a block-count boundary: 8,000 floats run on 8
        blocks, 8,200 on 9, so block 8 sits out every other call.  The buffer half
        must still alternate per CALL (xgmi.hip XgSignal::calls): with per-block
        parity, block 8 would overwrite words a slower peer's block 7 is still
        reading.  Ranks start skewed."""
        W, r, dev = self.world, self.rank, self.device
        sizes = [8_000, 8_200] * 6
        if max(sizes) * 4 > int(_lib.lib().jdt_xgmi_oneshot_bytes()) or max(sizes) * W > self.capacity // 2:
            return True
        outs, wants = [], []
        self._skew(r + 1)
        for it, n in enumerate(sizes):
            base = (torch.arange(n, device=dev, dtype=torch.int64) % 61).to(torch.float32)
            x = base * (r + 1) + it
            wants.append(base * (W * (W + 1) // 2) + W * it)
            if r == 0 and it % 3 == 0:
                torch.cuda._sleep(30_000)  # rank 0 lags inside the burst
            self.all_reduce_(x)
            outs.append(x)
        torch.cuda.synchronize(dev)
        bad = self.error() or any(not torch.equal(o, w) for o, w in zip(outs, wants))
        return self._check(bad, "one-shot burst mismatch (alternating block counts)")

    def _self_test_segments(self) -> bool:
        """Segmented AG / RS on the FSDP tutorial's per-rank shard lengths at N = 8
        (W1 rows 98 x 512, b1 64, W2 64 x 10 floats), for any world size."""
        W, r, dev = self.world, self.rank, self.device
        parts = [50_176, 64, 640]
        if sum(parts) * W > self.capacity // 2:
            return True
        for rep in range(2):
            fulls = [torch.empty(W * s, device=dev) for s in parts]
            mine = [(torch.arange(s, device=dev, dtype=torch.float32) % 31) + 100 * r + k + rep
                    for k, s in enumerate(parts)]
            self._skew(rep)
            self.all_gather_segments(list(zip(fulls, mine)))
            torch.cuda.synchronize(dev)
            for k, s in enumerate(parts):
                exp = torch.cat([(torch.arange(s, device=dev, dtype=torch.float32) % 31) + 100 * q + k + rep
                                 for q in range(W)])
                if not self._check(self.error() or not torch.equal(fulls[k], exp), "segmented all-gather mismatch"):
                    return False
            src = [(torch.arange(W * s, device=dev, dtype=torch.float32) % 53) * (r + 1) for s in parts]
            outs = [torch.full((s,), float(rep), device=dev) for s in parts]
            # + an all-reduce segment in the same launch (FSDP's replicated tail)
            tail = (torch.arange(128, device=dev, dtype=torch.float32) % 7) * (r + 1) + rep
            self._skew(rep + 1)
            self.reduce_scatter_segments(list(zip(src, outs)), accumulate=True, allreduce=[tail])
            torch.cuda.synchronize(dev)
            want_tail = (torch.arange(128, device=dev, dtype=torch.float32) % 7) * (W * (W + 1) // 2) + W * rep
            if not self._check(self.error() or not torch.equal(tail, want_tail),
                               "all-reduce segment of the segmented reduce-scatter mismatch"):
                return False
            for k, s in enumerate(parts):
                full = (torch.arange(W * s, device=dev, dtype=torch.float32) % 53) * (W * (W + 1) // 2)
                if not self._check(self.error() or not torch.equal(outs[k], full[r * s:(r + 1) * s] + rep),
                                   "segmented reduce-scatter mismatch"):
                    return False
        return True

    def _self_test_dim1(self) -> bool:
        """Segmented AG / RS of a dim-1 (column-block) shard pair: the 512 x 512 hidden
        weights of the 4-layer FSDP MLP (bf16 shadow and fp32 grads), next to a dim-0
        pair in the same launch."""
        W, r, dev = self.world, self.rank, self.device
        R, C = 64, 64 * W
        if (R * C + 4 * 512) * 2 > self.capacity // 2:
            return True
        col = torch.arange(C, device=dev)
        for rep in range(2):
            full = torch.empty(R, C, device=dev, dtype=torch.bfloat16)
            mine = ((torch.arange(R, device=dev)[:, None] * 3 + col[None, :64] + 7 * r + rep) % 61).to(torch.bfloat16)
            f0, m0 = torch.empty(512 * W, device=dev), torch.full((512,), float(r + rep), device=dev)
            self._skew(rep)
            self.all_gather_segments([(full, mine), (f0, m0)])
            torch.cuda.synchronize(dev)
            q = col // 64
            exp = ((torch.arange(R, device=dev)[:, None] * 3 + (col % 64)[None, :] + 7 * q[None, :] + rep) % 61)
            if not self._check(self.error() or not torch.equal(full, exp.to(torch.bfloat16))
                               or not torch.equal(f0, torch.arange(W, device=dev).repeat_interleave(512).float() + rep),
                               "dim-1 segmented all-gather mismatch"):
                return False
            src = ((torch.arange(R, device=dev)[:, None] + col[None, :]) % 29).float() * (r + 1)
            out = torch.empty(R, 64, device=dev)
            self._skew(rep + 1)
            self.reduce_scatter_segments([(src, out)])
            torch.cuda.synchronize(dev)
            want = ((torch.arange(R, device=dev)[:, None] + col[None, r * 64:(r + 1) * 64]) % 29).float()
            want = want * (W * (W + 1) // 2)
            if not self._check(self.error() or not torch.equal(out, want), "dim-1 segmented reduce-scatter mismatch"):
                return False
        return True

    def _self_test_adamw(self) -> bool:
        """The fused all-reduce + AdamW + metrics-fold kernel vs torch AdamW on the
        summed gradient (3 steps: both parities and the device step counter)."""
        W, r, dev = self.world, self.rank, self.device
        n_params, n_metrics = 4_096, 4
        n = n_params + n_metrics
        if part_len(n, W) * W > self.capacity // 2:
            return True
        g0 = torch.arange(n, device=dev, dtype=torch.int64)
        p = torch.linspace(-1, 1, n_params, device=dev)
        m, v = torch.zeros(n_params, device=dev), torch.zeros(n_params, device=dev)
        pr, mr, vr = p.clone(), m.clone(), v.clone()
        running = torch.zeros(n_metrics, device=dev)
        step = torch.zeros(1, dtype=torch.int32, device=dev)
        ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        # betas exactly representable in fp32, so the kernel's fp32 (1 - b) equals torch's
        lr, b1, b2, eps, wd, scale = 1e-2, 0.875, 1.0 - 2.0 ** -10, 1e-8, 1e-4, 1.0 / (4 * W)
        for t in range(1, 4):
            grad = ((g0 * (r + 1) + t) % 13 - 6).to(torch.float32)
            gsum = sum(((g0 * (q + 1) + t) % 13 - 6).to(torch.float32) for q in range(W))
            self._skew(t)
            self.all_reduce_adamw_(grad, p=p, m=m, v=v, shadow=None, n_params=n_params, running=running,
                                   n_metrics=n_metrics, lr=lr, b1=b1, b2=b2, eps=eps, wd=wd, grad_scale=scale,
                                   step=step, ticket=ticket, zero_grad=True)
            gr = gsum[:n_params] * scale
            mr.mul_(b1).add_(gr, alpha=1 - b1)
            vr.mul_(b2).addcmul_(gr, gr, value=1 - b2)
            pr.sub_(lr * ((mr / (1 - b1 ** t)) / ((vr / (1 - b2 ** t)).sqrt() + eps) + wd * pr))
            torch.cuda.synchronize(dev)
            bad = (self.error() or int(step.item()) != t or bool(grad.any())
                   or not torch.allclose(p, pr, rtol=1e-5, atol=1e-6)
                   or not torch.allclose(m, mr, rtol=1e-5, atol=1e-7)
                   or not torch.allclose(v, vr, rtol=1e-5, atol=1e-9))
            if not self._check(bad, f"fused AdamW all-reduce mismatch (step {t})"):
                return False
        want_running = sum(sum(((g0[n_params:] * (q + 1) + t) % 13 - 6).to(torch.float32) for q in range(W))
                           for t in range(1, 4))
        if not self._check(not torch.equal(running, want_running), "fused metrics fold mismatch"):
            return False
        # the staged variant (bucket pre-written into the staging half of the step's
        # parity, as mlp2_bwd / md_bwd do in DP): 3 more steps continuing the state
        plan = self.stage_plan(n)
        if not self._check(plan is None, "no unpadded staged geometry for the self-test bucket"):
            return False
        for t in range(4, 7):
            grad = ((g0 * (r + 1) + t) % 13 - 6).to(torch.float32)
            gsum = sum(((g0 * (q + 1) + t) % 13 - 6).to(torch.float32) for q in range(W))
            self.stage_write(int(step.item()) & 1, grad)
            self._skew(t)
            self.all_reduce_adamw_staged_(plan, p=p, m=m, v=v, shadow=None, n_params=n_params, running=running,
                                          n_metrics=n_metrics, lr=lr, b1=b1, b2=b2, eps=eps, wd=wd,
                                          grad_scale=scale, step=step, ticket=ticket)
            gr = gsum[:n_params] * scale
            mr.mul_(b1).add_(gr, alpha=1 - b1)
            vr.mul_(b2).addcmul_(gr, gr, value=1 - b2)
            pr.sub_(lr * ((mr / (1 - b1 ** t)) / ((vr / (1 - b2 ** t)).sqrt() + eps) + wd * pr))
            torch.cuda.synchronize(dev)
            bad = (self.error() or int(step.item()) != t
                   or not torch.allclose(p, pr, rtol=1e-5, atol=1e-6)
                   or not torch.allclose(m, mr, rtol=1e-5, atol=1e-7)
                   or not torch.allclose(v, vr, rtol=1e-5, atol=1e-9))
            if not self._check(bad, f"staged fused AdamW all-reduce mismatch (step {t})"):
                return False
        return True


# ----------------------------------------------------------------------------- transport choice per size
CALIBRATION_LADDER = (1024, 4096, 16384, 65536, 262144)   # floats: 4 KiB .. 1 MiB


def _max_over(group, v: float, device) -> float:
    t = torch.tensor([v], dtype=torch.float64, device=device if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def calibrate(comm: XgmiComm, sizes, iters: int = 20, rccl_margin_us: float = 3.0) -> dict:
    """Time this node's transports at the message sizes the trainer issues (SURVEY
    §5.8 (c)): the xGMI one-shot and two-shot all-reduce kernels and, when the group
    is nccl, RCCL's all-reduce -- each the median device time of ``iters`` calls,
    the MAX over ranks (every rank runs the same sequence).  Then
      * the one-shot threshold becomes the measured crossover (the largest ladder
        size where one-shot <= two-shot), replacing the 256 KiB default;
      * for each trainer size, ``choice`` is "xgmi" unless RCCL beats the better
        xGMI kernel by more than ``rccl_margin_us`` (the xGMI kernels also carry
        the fused AdamW / metrics fold that RCCL would need an extra launch for).
    Returns the table (bench JSON ``comm_choice``); ``rccl_us`` is None where RCCL is
    unavailable (gloo bootstrap: ranks sharing one GPU)."""
    L = _lib.lib()
    dev = comm.device
    rccl = dist.get_backend(comm.group) == "nccl"
    sizes = [int(n) for n in sizes if int(n) > 0]
    too_big = [n for n in sizes if not comm.fits(n)["twoshot"]]
    if too_big:   # the trainer sized the context: every size it issues must be timed
        raise ValueError(f"calibrate: trainer sizes {too_big} exceed this context (max {comm.max_allreduce()} floats)")
    ladder = sorted({int(n) for n in CALIBRATION_LADDER if comm.fits(n)["twoshot"]} | set(sizes))
    big = 1 << 40

    def timed(fn) -> float:
        fn()
        torch.cuda.synchronize(dev)
        dist.barrier(group=comm.group)
        ts = []
        for _ in range(iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        ts.sort()
        return _max_over(comm.group, ts[len(ts) // 2], dev)

    rows = []
    old = int(L.jdt_xgmi_oneshot_bytes())
    try:
        with torch.cuda.device(dev):
            for n in ladder:
                x = torch.ones(n, device=dev)
                one = None
                if comm.fits(n)["oneshot"]:
                    L.jdt_xgmi_set_oneshot_bytes(big)
                    one = timed(lambda: comm.all_reduce_(x))
                L.jdt_xgmi_set_oneshot_bytes(0)
                two = timed(lambda: comm.all_reduce_(x))
                rc = timed(lambda: dist.all_reduce(x, group=comm.group)) if rccl else None
                rows.append({"bytes": 4 * n, "xgmi_oneshot_us": None if one is None else round(one, 2),
                             "xgmi_twoshot_us": round(two, 2), "rccl_us": None if rc is None else round(rc, 2)})
    finally:
        L.jdt_xgmi_set_oneshot_bytes(old)
    if comm.error():
        raise RuntimeError("xgmi collective timed out during calibration")
    cross = 0
    for r in rows:   # the one-shot kernel up to the largest size where it is not slower
        if r["xgmi_oneshot_us"] is not None and r["xgmi_oneshot_us"] <= r["xgmi_twoshot_us"]:
            cross = r["bytes"]
    L.jdt_xgmi_set_oneshot_bytes(cross)
    want = {4 * n for n in sizes}
    for r in rows:
        best = min(t for t in (r["xgmi_oneshot_us"], r["xgmi_twoshot_us"]) if t is not None)
        r["xgmi_us"] = best
        r["choice"] = ("rccl" if r["rccl_us"] is not None and r["rccl_us"] + rccl_margin_us < best else "xgmi")
        r["trainer_size"] = r["bytes"] in want
    return {"oneshot_threshold_bytes": cross, "rccl": "available" if rccl else "unavailable (gloo group)",
            "rccl_margin_us": rccl_margin_us, "table": rows}


def status(comm: Optional[XgmiComm], world: int, device, mode: str = "auto") -> str:
    """What a trainer's N>1 transport ended up being, for logs and the bench JSON:
    ``passed`` (xGMI kernels, self-test passed on every rank), ``failed->rccl``
    (tried, fell back), ``off`` (RCCL requested / not a GPU job) or ``n/a`` (N=1)."""
    if world <= 1:
        return "n/a"
    if comm is not None:
        return "passed"
    return "failed->rccl" if requested(mode, world, torch.device(device)) else "off"


LAST_CALIBRATION: Optional[dict] = None   # this process's most recent calibrate() table (bench JSON)


def create_for(mesh, axis: str, cap_floats: int, device: torch.device, mode: str = "auto",
               sizes: Optional[list] = None) -> Optional[XgmiComm]:
    """An ``XgmiComm`` over ``mesh``'s ``axis`` group, or None (RCCL fallback).

    After the self-test the transports are timed at ``sizes`` (floats; default: the
    capacity requested, i.e. the trainer's bucket) -- :func:`calibrate` -- unless
    ``JDT_XGMI_CALIBRATE=0``; in "auto" mode the trainer gets RCCL (None) when RCCL
    wins at its largest size by more than the fused kernels' margin."""
    global LAST_CALIBRATION
    from ..runtime.dist import is_initialized

    n = mesh.axis_size(axis) if mesh is not None else 1
    if mesh is None or not is_initialized() or not requested(mode, n, device):
        return None
    from ..runtime.dist import spin_timeout_s

    size_grids_for_sharing(device)
    c = XgmiComm(mesh.group(axis), mesh.axis_index(axis), n, cap_floats, device, timeout_s=spin_timeout_s(30.0))
    if not c.ok:
        if mode == "xgmi":
            raise RuntimeError("xgmi collectives requested but unavailable on this node")
        log.warning("xgmi collectives unavailable; using RCCL")
        return None
    if os.environ.get("JDT_XGMI_CALIBRATE", "1") != "0":
        sizes = [int(s) for s in (sizes or [cap_floats]) if int(s) > 0]
        cal = calibrate(c, sizes)
        LAST_CALIBRATION = cal
        main = max(sizes)
        row = next(r for r in cal["table"] if r["bytes"] == 4 * main and r["trainer_size"])
        cal["trainer_bytes"] = 4 * main
        cal["transport"] = "xgmi" if row["choice"] == "xgmi" or mode == "xgmi" else "rccl"
        if mode != "xgmi" and cal["transport"] == "rccl":
            log.warning("xgmi: RCCL measured faster at %d bytes; using RCCL", 4 * main)
            c.close()
            return None
    return c
