"""Graph-capturable stage-to-stage send/recv over xGMI (comm/csrc/p2p.hip).

``XgmiP2P(group, rank, world, slot_bytes, n_slots, device)`` gives every member
of a process group an IPC-exported inbox of ``n_slots`` fixed-size slots.
``send(x, to, slot, epoch)`` pushes ``x`` into member ``to``'s slot;
``recv(out, slot, epoch)`` waits for this member's slot and copies it out.
``epoch`` is a device int32 counter (the optimizer step) that both sides read
at execution time, so the calls can be recorded once into a hipGraph and
replayed every step -- the pipeline trainer's GPipe step becomes one graph per
rank.

Construction checks the mapping with a ring exchange on the real hardware and
all members agree on the outcome; ``ok`` is False (callers fall back to RCCL
send/recv) otherwise.
"""
from __future__ import annotations

import ctypes
import logging
from ctypes import c_int, c_long, c_longlong, c_void_p
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _lib
from .xgmi import TICKS_PER_S, requested

log = logging.getLogger(__name__)

HANDLE_BYTES = 64
MAX_SLOTS = 64

_lib.declare("jdt_p2p_create", c_int, [c_int, c_int, c_long, c_int, ctypes.POINTER(c_void_p), c_void_p])
_lib.declare("jdt_p2p_open", c_int, [c_void_p, c_void_p])
_lib.declare("jdt_p2p_send", c_int, [c_void_p, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p])
_lib.declare("jdt_p2p_recv", c_int, [c_void_p, c_int, c_void_p, c_long, c_void_p, c_longlong, c_void_p])
_lib.declare("jdt_p2p_slot_bytes", c_long, [c_void_p])
_lib.declare("jdt_p2p_error", c_int, [c_void_p])
_lib.declare("jdt_p2p_reset", c_int, [c_void_p])
_lib.declare("jdt_p2p_destroy", c_int, [c_void_p])
_lib.declare("jdt_p2p_unmap", c_int, [c_void_p])


def wire_bytes(t: torch.Tensor) -> int:
    """Bytes moved for ``t`` (rounded up to the 16-byte transfer unit)."""
    return (t.numel() * t.element_size() + 15) // 16 * 16


class XgmiP2P:
    def __init__(self, group, rank: int, world: int, slot_bytes: int, n_slots: int, device: torch.device,
                 timeout_s: float = 30.0, self_test: bool = True):
        if not 0 < n_slots <= MAX_SLOTS:
            raise ValueError(f"1..{MAX_SLOTS} slots")
        self.group, self.rank, self.world, self.device = group, rank, world, device
        self.n_slots = n_slots
        self.timeout = c_longlong(int(timeout_s * TICKS_PER_S))
        self.ctx = c_void_p()
        self.ok = False
        L = _lib.lib()
        # a sender writes into the receiver's slot: every member uses the largest request
        sizes = [0] * world
        dist.all_gather_object(sizes, int(slot_bytes), group=group)
        slot_bytes = max(sizes)
        h = (ctypes.c_char * (2 * HANDLE_BYTES))()
        with torch.cuda.device(device):
            rc = L.jdt_p2p_create(rank, world, int(slot_bytes), int(n_slots), ctypes.byref(self.ctx), h)
        objs = [None] * world
        dist.all_gather_object(objs, bytes(h) if rc == 0 else None, group=group)
        good = all(o is not None for o in objs)
        if good:
            allh = b"".join(objs)
            buf = ctypes.create_string_buffer(allh, len(allh))
            with torch.cuda.device(device):
                good = L.jdt_p2p_open(self.ctx, buf) == 0
            if not good:
                log.warning("p2p: hipIpcOpenMemHandle failed on rank %d", rank)
        else:
            log.warning("p2p: inbox export failed on some rank (rank %d rc %d)", rank, rc)
        good = self._agree(good)
        if good and self_test:
            good = self._agree(self._self_test())
        self.ok = good
        if not good:
            self.close()

    def _agree(self, ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                         device=self.device if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))

    @property
    def slot_bytes(self) -> int:
        return int(_lib.lib().jdt_p2p_slot_bytes(self.ctx)) if self.ctx else 0

    def _check(self, t: torch.Tensor):
        if not t.is_cuda or not t.is_contiguous() or t.data_ptr() % 16:
            raise ValueError("p2p moves contiguous, 16-byte aligned CUDA tensors")
        if wire_bytes(t) != t.numel() * t.element_size():
            raise ValueError("p2p tensor size must be a multiple of 16 bytes")
        if wire_bytes(t) > self.slot_bytes:
            raise ValueError(f"tensor of {wire_bytes(t)} B exceeds the {self.slot_bytes} B slot")

    def send(self, x: torch.Tensor, to: int, slot: int, epoch: torch.Tensor):
        self._check(x)
        rc = _lib.lib().jdt_p2p_send(self.ctx, int(to), int(slot), c_void_p(x.data_ptr()), wire_bytes(x),
                                     c_void_p(epoch.data_ptr()), c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_p2p_send")

    def recv(self, out: torch.Tensor, slot: int, epoch: torch.Tensor) -> torch.Tensor:
        self._check(out)
        rc = _lib.lib().jdt_p2p_recv(self.ctx, int(slot), c_void_p(out.data_ptr()), wire_bytes(out),
                                     c_void_p(epoch.data_ptr()), self.timeout, c_void_p(_lib.stream_ptr()))
        _lib.check(rc, "jdt_p2p_recv")
        return out

    def error(self) -> int:
        """1 if a receive of this rank timed out (synchronises the device)."""
        return int(_lib.lib().jdt_p2p_error(self.ctx)) if self.ctx else 0

    def close(self, collective: bool = True):
        """Two-phase teardown (collective over the pipe group; comm/xgmi.py close)."""
        if self.ctx:
            if collective:
                from .xgmi import ipc_teardown_barrier

                _lib.lib().jdt_p2p_unmap(self.ctx)
                ipc_teardown_barrier(self.group)
            _lib.lib().jdt_p2p_destroy(self.ctx)
            self.ctx = c_void_p()
        self.ok = False

    def __del__(self):
        try:
            self.close(collective=False)
        except Exception:
            pass

    def _self_test(self) -> bool:
        """Ring exchange (r -> r+1) through EVERY slot at full slot size, 8 epochs
        (each slot's flag and payload reused 8 times), senders skewed by a rank-
        and epoch-dependent spin; exact values."""
        saved = self.timeout
        self.timeout = c_longlong(int(5.0 * TICKS_PER_S))
        try:
            W, r, dev = self.world, self.rank, self.device
            with torch.cuda.device(dev):
                n = min(self.slot_bytes // 4, 1 << 16) // 4 * 4
                ep = torch.zeros(1, dtype=torch.int32, device=dev)
                for it in range(8):
                    ok = True  # a failing rank keeps sending, so no peer waits on it mid-epoch
                    for slot in range(self.n_slots):
                        x = torch.arange(n, device=dev, dtype=torch.float32) + 1000 * r + 7 * it + slot
                        out = torch.empty(n, device=dev)
                        cyc = ((r * 5 + it + slot) % (W + 1)) * 10_000
                        if cyc:
                            torch.cuda._sleep(cyc)
                        self.send(x, (r + 1) % W, slot, ep)
                        self.recv(out, slot, ep)
                        want = torch.arange(n, device=dev, dtype=torch.float32) + 1000 * ((r - 1) % W) + 7 * it + slot
                        torch.cuda.synchronize(dev)
                        if ok and (self.error() or not torch.equal(out, want)):
                            log.warning("p2p self-test failed on rank %d (iter %d slot %d)", r, it, slot)
                            ok = False
                    ep += 1
                    # the next epoch's sends may only start once every member read this one;
                    # the verdict is collective, so every rank stops at the same epoch
                    torch.cuda.synchronize(dev)
                    if not self._agree(ok):
                        return False
            # training epochs restart at 1: clear the flags the test raised
            _lib.check(_lib.lib().jdt_p2p_reset(self.ctx), "jdt_p2p_reset")
            dist.barrier(group=self.group)
            return True
        except Exception as e:  # noqa: BLE001
            log.warning("p2p self-test raised: %s", e)
            return False
        finally:
            self.timeout = saved


def create_for(mesh, axis: str, slot_bytes: int, n_slots: int, device: torch.device,
               mode: str = "auto") -> Optional[XgmiP2P]:
    """An ``XgmiP2P`` over ``mesh``'s ``axis`` group, or None (RCCL send/recv fallback)."""
    from ..runtime.dist import is_initialized

    n = mesh.axis_size(axis) if mesh is not None else 1
    if mesh is None or not is_initialized() or not requested(mode, n, device):
        return None
    from ..runtime.dist import spin_timeout_s

    c = XgmiP2P(mesh.group(axis), mesh.axis_index(axis), n, slot_bytes, n_slots, device,
                timeout_s=spin_timeout_s(30.0))
    if not c.ok:
        if mode == "xgmi":
            raise RuntimeError("xgmi p2p requested but unavailable on this node")
        log.warning("xgmi p2p unavailable; using RCCL send/recv")
        return None
    return c
