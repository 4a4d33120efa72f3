"""Debug aids: replication checker, failure reporting, serialized-kernel mode.

The reference disables shard_map's replication check everywhere
(``check_rep=False``, data_paral.py:161,247; param_sharding.py:258,273,376) and
has no race/failure tooling.  Here:

* :func:`check_replicated` -- T7: hash the tensors that must be identical on
  every member of a mesh axis (DP params after a step, replicated FSDP leaves)
  and all-gather the hashes; raises with the diverging ranks.
* :func:`debug_mode` -- HIP_LAUNCH_BLOCKING / AMD_SERIALIZE_KERNEL style
  serialisation so a faulting kernel is reported at its launch.
* :func:`guarded` -- run a step function; on an exception print it on the
  failing rank (``print_exception``, util.py:12-14), tear the process group
  down so peers fail fast instead of hanging in a collective, and re-raise.
"""
from __future__ import annotations

import contextlib
import hashlib
import os
from typing import Dict, Iterable, Optional

import torch
import torch.distributed as dist

from ..comm import collectives as C
from ..runtime.dist import Mesh, is_initialized
from .metrics import print_exception


def tensor_digest(t: torch.Tensor) -> int:
    b = t.detach().contiguous().cpu().view(torch.uint8).numpy().tobytes()
    return int.from_bytes(hashlib.blake2b(b, digest_size=8).digest(), "little", signed=True)


class ReplicationError(RuntimeError):
    pass


def check_replicated(tensors: Dict[str, torch.Tensor], mesh: Optional[Mesh], axis: str) -> None:
    """All members of ``axis`` must hold bit-identical ``tensors``."""
    n = C.axis_size(mesh, axis)
    if n == 1 or not is_initialized():
        return
    names = sorted(tensors)
    h = torch.tensor([tensor_digest(tensors[k]) for k in names], dtype=torch.int64)
    dev = tensors[names[0]].device if dist.get_backend(mesh.group(axis)) == "nccl" else torch.device("cpu")
    h = h.to(dev)
    allh = C.all_gather(h[None], mesh, axis, dim=0).cpu()
    bad = [(names[j], [int(r) for r in range(n) if allh[r, j] != allh[0, j]]) for j in range(len(names))
           if not bool((allh[:, j] == allh[0, j]).all())]
    if bad:
        raise ReplicationError(f"replicated tensors diverged on axis {axis!r}: {bad}")


SERIALIZE_ENV = {"HIP_LAUNCH_BLOCKING": "1", "AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3"}


@contextlib.contextmanager
def debug_mode(serialize: bool = True):
    """Serialise kernel launches (faults surface at the offending launch).

    The HIP runtime reads these variables when it initialises, so the context
    only takes effect for a process (or child) that has not touched the GPU yet;
    entry scripts expose it as ``--serialize-kernels``, applied before any GPU call."""
    import warnings

    old = {k: os.environ.get(k) for k in SERIALIZE_ENV}
    if serialize:
        if torch.cuda.is_initialized():
            warnings.warn("debug_mode(): the HIP runtime is already initialised in this process; the "
                          "serialisation variables only reach child processes (use --serialize-kernels)")
        os.environ.update(SERIALIZE_ENV)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def guarded(fn, *args, **kw):
    try:
        return fn(*args, **kw)
    except Exception as e:  # noqa: BLE001
        print_exception(e)
        if is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001
                pass
        raise


def replicated_state(trainer):
    """(tensors that must be bit-identical across the trainer's data axis, axis name).

    DP: every parameter and both AdamW moments (replicated by construction:
    same init + the same all-reduced gradient).  FSDP: only the leaves the
    sharding rule kept whole (param_sharding.py:89-92) and the running metrics.
    GPipe: this stage's parameters across the data replicas of the stage."""
    from ..parallel.dp import DataParallelTrainer
    from ..parallel.fsdp import FSDPTrainer
    from ..parallel.pipeline import GPipeTrainer

    if isinstance(trainer, FSDPTrainer):
        sp = trainer.sp
        out = {f"param/{n}": sp.local.p(n) for n in sp.repl_names}
        out["metrics"] = trainer.metrics
        return out, trainer.cfg.axis
    if isinstance(trainer, (DataParallelTrainer, GPipeTrainer)):
        P = trainer.state.params
        out = {f"param/{n}": P.p(n) for n in P.names()}
        for k in ("m", "v", "buf"):
            if k in trainer.state.opt_state:
                out[f"opt/{k}"] = trainer.state.opt_state[k]
        axis = trainer.cfg.axis if isinstance(trainer, DataParallelTrainer) else trainer.cfg.data_axis
        return out, axis
    raise TypeError(f"no replication contract for {type(trainer).__name__}")


def check_trainer_replication(trainer) -> None:
    """``--check-replication`` of the entry scripts: raise
    :class:`ReplicationError` naming the diverged tensors and ranks."""
    if hasattr(trainer, "finalize"):
        trainer.finalize()
    tensors, axis = replicated_state(trainer)
    if trainer.mesh is None or not tensors:
        return
    if tensors and next(iter(tensors.values())).is_cuda:
        torch.cuda.synchronize()
    check_replicated(tensors, trainer.mesh, axis)
    from ..runtime.dist import rank

    if rank() == 0:
        print(f"[check-replication] {len(tensors)} replicated tensors bit-identical across axis {axis!r}",
              flush=True)
