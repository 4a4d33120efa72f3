"""JAX-named collectives over a :class:`~..runtime.dist.Mesh` axis.

================  =======================================  ==========================
reference (jax)   here                                      RCCL call
================  =======================================  ==========================
axis_index        ``axis_index(mesh, axis)``                none (mesh coordinate)
psum(1, axis)     ``axis_size(mesh, axis)``                 none
psum / pmean      ``psum_(x, mesh, axis)`` (in place)      ncclAllReduce
all_gather tiled  ``all_gather(x, mesh, axis, dim)``        ncclAllGather
psum_scatter      ``psum_scatter(x, mesh, axis, dim)``      ncclReduceScatter
ppermute          ``ppermute(x, mesh, axis, perm)``         ncclSend/ncclRecv group
================  =======================================  ==========================

Mean variants return the SUM and let the caller fold ``1/N`` into the next
kernel (the optimizer's grad_scale), except where a standalone mean is asked
for.  On the gloo backend (CPU simulation) the tensor-native collectives that
gloo lacks are emulated with the list forms; semantics are identical.

Every call takes the current stream implicitly (RCCL enqueues on torch's
current stream when ``async_op=False``), so they are hipGraph-capturable.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..runtime.dist import Mesh, is_initialized


def axis_index(mesh: Optional[Mesh], axis: str) -> int:
    return 0 if mesh is None else mesh.axis_index(axis)


def axis_size(mesh: Optional[Mesh], axis: str) -> int:
    return 1 if mesh is None else mesh.axis_size(axis)


def _active(mesh: Optional[Mesh], axis: str) -> bool:
    """Whether a collective along ``axis`` is a real call (a 1-member axis only on a
    ``Mesh(unit_groups=True)``)."""
    if mesh is None or not is_initialized():
        return False
    return mesh.axis_size(axis) > 1 or (getattr(mesh, "unit_groups", False) and mesh.group(axis) is not None)


def active(mesh: Optional[Mesh], axis: str) -> bool:
    """Public form of the check above: the trainers issue their collectives iff this holds."""
    return _active(mesh, axis)


def _is_gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


def _host(x: torch.Tensor, g) -> torch.Tensor:
    """gloo works on host memory: GPU tensors (several ranks sharing one GPU in the
    multi-process GPU tests) are staged through a CPU copy."""
    return x.cpu() if (x.is_cuda and _is_gloo(g)) else x


def psum_(x: torch.Tensor, mesh: Optional[Mesh], axis: str) -> torch.Tensor:
    """In-place SUM all-reduce along ``axis``."""
    if _active(mesh, axis):
        g = mesh.group(axis)
        h = _host(x, g)
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=g)
        if h is not x:
            x.copy_(h)
    return x


def pmean_(x: torch.Tensor, mesh: Optional[Mesh], axis: str) -> torch.Tensor:
    psum_(x, mesh, axis)
    n = axis_size(mesh, axis)
    if n > 1:
        x.mul_(1.0 / n)
    return x


def psum_multi_(x: torch.Tensor, mesh: Optional[Mesh], axes: Sequence[str]) -> torch.Tensor:
    for a in axes:
        psum_(x, mesh, a)
    return x


def all_gather(x: torch.Tensor, mesh: Optional[Mesh], axis: str, dim: int = 0,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Tiled all-gather: concatenate the shards of every member along ``dim``."""
    n = axis_size(mesh, axis)
    if not _active(mesh, axis):
        if out is not None:
            out.copy_(x)
            return out
        return x
    g = mesh.group(axis)
    x = x.contiguous()
    if dim != 0:
        return torch.cat(_gather_list(x, g, n), dim=dim) if out is None else out.copy_(
            torch.cat(_gather_list(x, g, n), dim=dim))
    if out is None:
        out = torch.empty((x.shape[0] * n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if _is_gloo(g):
        out.copy_(torch.cat(_gather_list(x, g, n), dim=0))
    else:
        dist.all_gather_into_tensor(out, x, group=g)
    return out


def _gather_list(x, g, n) -> List[torch.Tensor]:
    h = _host(x, g)
    parts = [torch.empty_like(h) for _ in range(n)]
    dist.all_gather(parts, h, group=g)
    return [p.to(x.device) for p in parts] if h is not x else parts


def psum_scatter(x: torch.Tensor, mesh: Optional[Mesh], axis: str, dim: int = 0,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Tiled reduce-scatter (SUM): member i receives the i-th ``dim``-slice of the sum."""
    n = axis_size(mesh, axis)
    if not _active(mesh, axis):
        if out is not None:
            out.copy_(x)
            return out
        return x
    g = mesh.group(axis)
    idx = mesh.axis_index(axis)
    if dim != 0 and not _is_gloo(g):
        # RCCL: scatter along dim 0 of the dim-first layout (the i-th dim-slice of
        # the sum is the i-th dim-0 slice after movedim), then move the dim back
        xt = x.movedim(dim, 0).contiguous()
        res = torch.empty((xt.shape[0] // n,) + tuple(xt.shape[1:]), dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(res, xt, op=dist.ReduceOp.SUM, group=g)
        res = res.movedim(0, dim)
        if out is None:
            return res.contiguous()
        out.copy_(res)
        return out
    if _is_gloo(g):
        red = _host(x, g).clone()
        dist.all_reduce(red, group=g)
        red = red.to(x.device)
        res = red.chunk(n, dim=dim)[idx]
        if out is None:
            return res.contiguous()
        out.copy_(res)
        return out
    x = x.contiguous()
    if out is None:
        out = torch.empty((x.shape[0] // n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, op=dist.ReduceOp.SUM, group=g)
    return out


def ppermute(x: torch.Tensor, mesh: Optional[Mesh], axis: str, perm: Sequence[Tuple[int, int]],
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """jax.lax.ppermute along ``axis``: for each (src, dst) pair (axis indices),
    member src sends ``x`` to member dst.  Members that receive nothing get zeros."""
    if out is None:
        out = torch.zeros_like(x)
    else:
        out.zero_()
    if not _active(mesh, axis):
        for s, d in perm:
            if s == d == 0:
                out.copy_(x)
        return out
    me = mesh.axis_index(axis)
    ops = []
    for s, d in perm:
        if s == me and d == me:
            out.copy_(x)
        elif s == me:
            ops.append(dist.P2POp(dist.isend, x.contiguous(), mesh.global_rank(axis, d), mesh.group(axis)))
        elif d == me:
            ops.append(dist.P2POp(dist.irecv, out, mesh.global_rank(axis, s), mesh.group(axis)))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    return out


def send(x: torch.Tensor, mesh: Mesh, axis: str, dst_index: int):
    dist.send(x.contiguous(), mesh.global_rank(axis, dst_index), group=mesh.group(axis))


def recv(x: torch.Tensor, mesh: Mesh, axis: str, src_index: int) -> torch.Tensor:
    dist.recv(x, mesh.global_rank(axis, src_index), group=mesh.group(axis))
    return x


def broadcast_(x: torch.Tensor, mesh: Optional[Mesh], axis: str, src_index: int = 0) -> torch.Tensor:
    if _active(mesh, axis):
        g = mesh.group(axis)
        h = _host(x, g)
        dist.broadcast(h, mesh.global_rank(axis, src_index), group=g)
        if h is not x:
            x.copy_(h)
    return x
