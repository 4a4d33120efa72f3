"""Per-tile gradient exchange buffers for the one-launch N > 1 DP step.

The fused 2-layer DP step at N > 1 normally takes three launches per step (forward,
backward into the xGMI staging buffer, all-reduce + AdamW: comm/xgmi.py).  With a
``TileExchange`` the run-ahead backward kernel (ops/csrc/mlp_fused.hip, mlp2_bwd AHEAD
with ``Mlp2Args::tx``) all-reduces each of its 224 gradient tiles with the same tile
of the other ranks' launches -- a two-shot exchange per tile over IPC-mapped inboxes
(tile T summed by rank T % W in rank order and pushed back) -- then applies AdamW and
runs the next step's forward, as on one GPU: one launch per step.  This module owns the
inboxes (comm/csrc/tile_exchange.hip): allocation, IPC handle exchange over the
process group, and the device-resident ``TxArgs`` pointer the kernel takes.

Reference semantics: the DP step's ``pmean`` of the gradients and ``psum`` of the
metrics (/root/reference/data_paral.py:210-228) -- here a SUM whose 1/N rides in the
optimizer's gradient scale, as for the other DP collectives.
"""
from __future__ import annotations

import ctypes
import logging
from ctypes import c_int, c_longlong, c_void_p
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _lib

log = logging.getLogger(__name__)

HANDLE_BYTES = 64
TICKS_PER_S = 100_000_000   # s_memrealtime: 100 MHz
# payload per tile (floats): 7 dW1 sub-tiles of 256, then dW2 / db1 (256 each) and
# 128 for db2 + the metric slots -- ops/csrc/mlp_fused.hip tx_tile callers
TILE_PAYLOAD = 9 * 256 + 128

_lib.declare("jdt_tx_create", c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_void_p), c_void_p])
_lib.declare("jdt_tx_open", c_int, [c_void_p, c_void_p, c_longlong])
_lib.declare("jdt_tx_args", c_void_p, [c_void_p])
_lib.declare("jdt_tx_close", None, [c_void_p])
_lib.declare("jdt_tx_unmap", None, [c_void_p])
_lib.declare("jdt_mlp2_ahead_tx_ok", c_int, [c_int, c_int, c_int, c_int])
_lib.declare("jdt_tx_selftest", c_int, [c_void_p, c_int, ctypes.c_uint, c_void_p, c_void_p])
_lib.declare("jdt_tx_reset", c_int, [c_void_p])
_lib.declare("jdt_tx_error", ctypes.c_uint, [c_void_p])
_lib.declare("jdt_md_fx_ok", c_int, [c_int, c_int])
_lib.declare("jdt_md_tx_ok", c_int, [c_int, c_int])
SELFTEST_TILES = 64   # 64 workgroups per rank: 8 ranks' self-test grids fit one shared GPU


class TileExchange:
    """IPC inboxes of the per-tile exchange between the ``world`` ranks of ``group``
    (collective: every rank constructs it at the same point).  ``ok`` is False on every
    rank if any rank failed to export or map them."""

    def __init__(self, group, rank: int, world: int, tiles: int, device: torch.device,
                 pay: int = TILE_PAYLOAD, timeout_s: float = 10.0):
        self.group, self.rank, self.world, self.tiles, self.pay = group, rank, world, tiles, pay
        self.timeout_s = float(timeout_s)
        self.device = device
        self.ctx = c_void_p()
        self.ok = False
        self.selftest = None
        L = _lib.lib()
        h = (ctypes.c_char * (3 * HANDLE_BYTES))()
        with torch.cuda.device(device):
            rc = L.jdt_tx_create(rank, world, tiles, pay, ctypes.byref(self.ctx), h)
        mine = bytes(h) if rc == 0 else None
        objs = [None] * world
        dist.all_gather_object(objs, mine, group=group)
        good = all(o is not None for o in objs)
        if good:
            allh = b"".join(objs)
            buf = ctypes.create_string_buffer(allh, len(allh))
            with torch.cuda.device(device):
                good = L.jdt_tx_open(self.ctx, buf, int(timeout_s * TICKS_PER_S)) == 0
            if not good:
                log.warning("tile exchange: hipIpcOpenMemHandle failed on rank %d", rank)
        else:
            log.warning("tile exchange: buffer export failed on some rank (rank %d rc %d)", rank, rc)
        good = self._agree(good)
        if good:
            # every rank exchanges known values through the real buffers and kernel code
            # (all payload positions, W-rank sums bit-exact), then clears its flags -- the
            # step kernels' epochs start at 1 -- before any rank may use them
            good = self._self_test()
        self.ok = self._agree(good)
        if not self.ok:
            self.close()

    def _self_test(self) -> bool:
        L = _lib.lib()
        words = torch.zeros(2, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            rc = L.jdt_tx_selftest(self.args_ptr, min(self.tiles, SELFTEST_TILES), 1, words.data_ptr(),
                                   c_void_p(_lib.stream_ptr(self.device)))
            torch.cuda.synchronize(self.device)
            bad, err = (int(x) for x in words.cpu())
            rc2 = L.jdt_tx_reset(self.ctx)
        self.selftest = {"rc": int(rc), "wrong": bad, "timeouts": err, "reset": int(rc2)}
        if rc != 0 or bad or err or rc2 != 0:
            log.warning("tile exchange self-test failed on rank %d: %s", self.rank, self.selftest)
            return False
        return True

    def _agree(self, ok: bool) -> bool:
        return agree(self.group, ok, self.device)

    @property
    def args_ptr(self) -> int:
        """Device pointer of the kernel's TxArgs (Mlp2Args::tx)."""
        return int(_lib.lib().jdt_tx_args(self.ctx) or 0) if self.ctx else 0

    def error(self) -> int:
        """This rank's error word (4: an exchange wait timed out; synchronous read)."""
        return int(_lib.lib().jdt_tx_error(self.ctx)) if self.ctx else 0

    def close(self, collective: bool = True):
        """Two-phase teardown (collective over the group; comm/xgmi.py close)."""
        if self.ctx:
            if collective:
                from .xgmi import ipc_teardown_barrier

                _lib.lib().jdt_tx_unmap(self.ctx)
                ipc_teardown_barrier(self.group)
            _lib.lib().jdt_tx_close(self.ctx)
            self.ctx = c_void_p()
        self.ok = False


def agree(group, ok: bool, device: torch.device) -> bool:
    """AND of ``ok`` over ``group`` (collective)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                     device=device if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def ahead_tx_ok(rows: int, hidden: int, ranks_on_this_gpu: int, k_in: int = 784) -> bool:
    """Whether the one-launch N > 1 step can run here: the run-ahead conditions plus
    every sharing rank's grid resident at once (``ranks_on_this_gpu`` grids per GPU)."""
    return bool(_lib.lib().jdt_mlp2_ahead_tx_ok(int(rows), int(hidden), int(k_in), int(ranks_on_this_gpu)))


def deep_tx_ok(rows: int, ranks_on_this_gpu: int) -> bool:
    """The deep (>= 2 hidden layers) engine's exchanging backward launches all resident
    with ``ranks_on_this_gpu`` ranks' grids per GPU (csrc/mlp_deep.hip jdt_md_tx_ok)."""
    return bool(_lib.lib().jdt_md_tx_ok(int(rows), int(ranks_on_this_gpu)))


def deep_fx_ok(rows: int, ranks_on_this_gpu: int) -> bool:
    """The deep engine's FSDP form (md_bwd FX) resident as deep_tx_ok."""
    return bool(_lib.lib().jdt_md_fx_ok(int(rows), int(ranks_on_this_gpu)))


def fx_owner_span(world: int, rows: int = 784, chunk: int = 112) -> int:
    """Most shard owners any ``chunk``-row W1 input chunk of the FSDP one-launch exchange
    touches (dim-0 shards of ``rows / world`` rows; chunks start at multiples of ``chunk``).
    mlp2_bwd's FX partial stores go to the chunk's first and last owner only, so the step
    is valid only when this is <= 2 (and ``world`` divides ``rows``)."""
    if world < 1 or rows % world:
        return 1 << 30
    rpq = rows // world
    return max((c0 + chunk - 1) // rpq - c0 // rpq + 1 for c0 in range(0, rows, chunk))


def create_for(mesh, axis: str, device: torch.device, tiles: int) -> Optional[TileExchange]:
    """The exchange for ``axis`` of ``mesh`` on GPUs (None off the GPU, at N = 1, or if
    any rank could not build it)."""
    from ..comm import collectives as C

    W = C.axis_size(mesh, axis)
    if W < 2 or device.type != "cuda" or W > 8:
        return None
    from ..runtime.dist import spin_timeout_s

    tx = TileExchange(mesh.group(axis), C.axis_index(mesh, axis), W, tiles, device, timeout_s=spin_timeout_s(10.0))
    return tx if tx.ok else None
