"""Process-per-device runtime: bootstrap, device mesh, sub-groups.

The reference runs all "devices" inside ONE process as XLA host devices
(util.py:31-38) and names a 1-D mesh ``Mesh(devices, ('data',))``
(data_paral.py:150-152).  On MI355X each GPU is its own process: bootstrap is
``torchrun`` (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR from the env), the
backend is ``nccl`` (= RCCL over xGMI on ROCm), and a :class:`Mesh` names the
axes of an N-D process grid (``("data",)``, ``("data", "pipe")``...) by building
one process group per axis line.  The CPU simulation mode is the same code
with the gloo backend and one process per simulated device.
"""
from __future__ import annotations

import datetime
import math
import os
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

_STATE: Dict[str, object] = {"device": None, "backend": None, "mesh": None}


def current_mesh() -> Optional["Mesh"]:
    """The most recently constructed :class:`Mesh` of this process (or None)."""
    return _STATE.get("mesh")  # type: ignore[return-value]


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def device() -> torch.device:
    d = _STATE.get("device")
    if d is None:
        d = torch.device("cpu")
    return d  # type: ignore[return-value]


def sim_cpu_requested() -> bool:
    return os.environ.get("JDT_SIM_CPU") is not None


def init(backend: Optional[str] = None, timeout_s: float = 600.0) -> torch.device:
    """Initialise the process group from torchrun-style env vars (idempotent).

    backend None -> ``$JDT_BACKEND`` if set (``gloo`` rehearses several ranks
    sharing one GPU -- RCCL refuses that -- while the xGMI P2P kernels still
    run), else ``nccl`` (RCCL) when a GPU is usable and simulation is not
    requested, else ``gloo`` on CPU.  Sets the current HIP device to LOCAL_RANK.
    """
    use_gpu = (not sim_cpu_requested()) and torch.cuda.is_available()
    if use_gpu:
        dev = torch.device("cuda", local_rank() % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
        _host_sync_mode()
    else:
        dev = torch.device("cpu")
    _STATE["device"] = dev
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1 and not is_initialized():
        be = backend or os.environ.get("JDT_BACKEND") or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
        _STATE["backend"] = be
    return dev


def _host_sync_mode():
    """JDT_SYNC_SPIN=1: host waits on this device (torch.cuda.synchronize, event
    waits) spin instead of sleeping until an interrupt (hipDeviceScheduleSpin on the
    current device), so a short timed region's closing synchronize returns as soon as
    the last kernel completes.  Recorded in _STATE["host_sync"]."""
    _STATE["host_sync"] = "auto"
    if os.environ.get("JDT_SYNC_SPIN", "0") != "1":
        return
    import ctypes

    try:
        hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch already loaded (same soname)
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))   # hipDeviceScheduleSpin
    except OSError:
        rc = -1
    _STATE["host_sync"] = "spin" if rc == 0 else f"auto (hipSetDeviceFlags rc {rc})"


def host_sync_mode() -> str:
    return str(_STATE.get("host_sync", "auto"))


def backend() -> Optional[str]:
    return dist.get_backend() if is_initialized() else None


def shutdown():
    if is_initialized():
        try:
            dist.barrier()
        except Exception:  # noqa: BLE001
            pass
        dist.destroy_process_group()


def collectives_capturable() -> bool:
    """Whether this job's collectives can be recorded into a hipGraph: RCCL (the nccl
    backend) enqueues every collective on the caller's stream, so torch.cuda.graph
    captures it; gloo runs on the host and cannot be captured."""
    return backend() == "nccl"


def ranks_per_gpu() -> int:
    """The most ranks of the job that drive one physical GPU (same PCI domain / bus /
    device): > 1 in the rehearsal setup of several processes on one card, where
    concurrent spinning streams time-share the GPU's queues (profiles/r4_pp_streams_ab.txt,
    r4_overlap_sync_ab.txt) and co-resident grids must share its CUs; 1 on a node with one
    rank per GPU, with one rank, or off the GPU.  Collective over the world group (every
    rank must call it); cached."""
    if "gpu_share" in _STATE:
        return int(_STATE["gpu_share"])
    dev = device()
    n = 1
    if is_initialized() and world_size() > 1 and dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        mine = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
        ids = [None] * world_size()
        dist.all_gather_object(ids, mine)
        ids = [tuple(x) for x in ids]
        n = max(ids.count(x) for x in ids)
    _STATE["gpu_share"] = n
    return n


def spin_timeout_s(base_s: float) -> float:
    """Wall-clock bound of an in-kernel wait (xGMI barriers, inbox receives, tile
    exchange) for this job: ``base_s`` with a GPU per rank; with k ranks time-sharing
    one GPU (rehearsals) a peer's grid may wait for its queue to be scheduled, so the
    bound grows with k (x k / 2).  Collective on first use (ranks_per_gpu)."""
    k = ranks_per_gpu()
    return float(base_s) * max(1.0, k / 2.0)


def ranks_share_gpu() -> bool:
    """Two ranks of the job drive the same GPU (ranks_per_gpu() > 1)."""
    return ranks_per_gpu() > 1


def quiesce(dev):
    """Before a trainer frees IPC buffers its peers write into (collective when a process
    group is up): this rank's queue drained, then every rank's, so no peer kernel still
    writes into a context being torn down.  The exported buffers themselves go back to a
    per-process pool, never to the driver (comm/csrc/ipc_pool.hip): with them freed, a
    new context's start-up self-test saw its own tensors change under it even after this
    barrier (profiles/r5_ipc_pool.txt, 4 ranks sharing the GPU)."""
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize(dev)
    barrier()


def barrier():
    if is_initialized():
        if backend() == "nccl":
            dist.barrier(device_ids=[device().index])
        else:
            dist.barrier()


class Mesh:
    """N-D process mesh.  ``Mesh({"data": 2, "pipe": 4})``: rank = row-major index
    over the axes in the given order (the last axis varies fastest), so with
    ("data", "pipe") the pipe stages of one data replica are consecutive ranks --
    on an 8-GPU MI355X node every pair is one xGMI hop regardless.

    ``unit_groups=True`` gives axes of size 1 a real process group too (the world
    group of a 1-rank job, else a 1-member group), and the collectives of
    comm/collectives.py then run on them instead of short-circuiting: a one-GPU job
    issues exactly the RCCL calls (and graph captures) an N-GPU job does."""

    def __init__(self, axes: Dict[str, int] | Sequence[Tuple[str, int]], unit_groups: bool = False):
        items = list(axes.items()) if isinstance(axes, dict) else list(axes)
        self.axis_names: Tuple[str, ...] = tuple(a for a, _ in items)
        self.shape: Tuple[int, ...] = tuple(int(s) for _, s in items)
        ws = world_size()
        if math.prod(self.shape) != ws:
            raise ValueError(f"mesh {dict(items)} needs {math.prod(self.shape)} ranks, world has {ws}")
        self.rank = rank()
        self.unit_groups = bool(unit_groups) and is_initialized()
        self.coords = self._coords(self.rank)
        self._groups: Dict[str, Optional[dist.ProcessGroup]] = {}
        self._group_ranks: Dict[str, Tuple[int, ...]] = {}
        for ai, a in enumerate(self.axis_names):
            mine = None
            # every rank must create every group, in the same order
            for line in self._lines(ai):
                g = dist.new_group(list(line)) if (is_initialized() and self.shape[ai] != ws and
                                                    (self.shape[ai] > 1 or self.unit_groups)) else None
                if self.rank in line:
                    mine = (g, line)
            g, line = mine
            if is_initialized() and self.shape[ai] == ws and (ws > 1 or self.unit_groups):
                g = dist.group.WORLD
            self._groups[a] = g
            self._group_ranks[a] = tuple(line)
        _STATE["mesh"] = self

    def _coords(self, r: int) -> Tuple[int, ...]:
        c = []
        for s in reversed(self.shape):
            c.append(r % s)
            r //= s
        return tuple(reversed(c))

    def _rank_of(self, coords: Sequence[int]) -> int:
        r = 0
        for c, s in zip(coords, self.shape):
            r = r * s + c
        return r

    def _lines(self, ai: int):
        others = [range(s) for i, s in enumerate(self.shape) if i != ai]
        import itertools

        for combo in itertools.product(*others):
            line = []
            for k in range(self.shape[ai]):
                coords = list(combo)
                coords.insert(ai, k)
                line.append(self._rank_of(coords))
            yield tuple(line)

    # ---------------------------------------------------------------- queries
    def group(self, axis: str) -> Optional[dist.ProcessGroup]:
        return self._groups[axis]

    def group_ranks(self, axis: str) -> Tuple[int, ...]:
        return self._group_ranks[axis]

    def axis_index(self, axis: str) -> int:
        return self.coords[self.axis_names.index(axis)]

    def axis_size(self, axis: str) -> int:
        return self.shape[self.axis_names.index(axis)]

    def global_rank(self, axis: str, index: int) -> int:
        """Global rank of the member at ``index`` along ``axis`` in this rank's line."""
        return self._group_ranks[axis][index]

    def __repr__(self):
        return f"Mesh({dict(zip(self.axis_names, self.shape))}, rank={self.rank}, coords={self.coords})"
