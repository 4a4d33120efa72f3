"""RNG folding (data_paral.py:28-34 ``fold_rng_over_axis``; util.py:51, 91 ``split``).

JAX threads explicit PRNG keys; on MI355X dropout is a counter-based Philox
stream addressed by (seed, offset) and regenerated in the backward epilogue, so
a "key" here is a 64-bit integer.  ``split``/``fold_in`` are deterministic
integer mixes (splitmix64), which gives the same statistical contract as
threefry: independent streams per (step, minibatch, device).  Bit parity with
JAX's threefry is out of scope.
"""
from __future__ import annotations

from typing import List, Sequence

_MASK = (1 << 64) - 1
_U64 = 1 << 64


def _mix(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK
    return z ^ (z >> 31)


def PRNGKey(seed: int) -> int:
    return _mix(int(seed) & _MASK)


def _s64(v: int) -> int:
    """u64 bit pattern as the int64 torch stores."""
    v &= _MASK
    return v - _U64 if v >> 63 else v


def _mix_t(z):
    """``_mix`` over an int64 tensor (wrapping arithmetic; logical shifts emulated)."""
    z = z + _s64(0x9E3779B97F4A7C15)
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _s64(0x94D049BB133111EB)
    return z ^ ((z >> 31) & ((1 << 33) - 1))


class ScanKey(int):
    """The rng a rolled (graph-replayed) minibatch step receives in
    ``util.accum_grads_scan`` -- the analogue of the reference's ``keys[batch_idx]``
    gather inside ``jax.lax.scan`` (util.py:91, 107-108).

    It carries every minibatch's key twice: on the host (``keys``) and on the device
    (``dev``, int64), plus the device int32 ``index`` of the minibatch being replayed.
    ``fold_in`` / ``split`` / ``fold_rng_over_axis`` map over all keys on both sides
    (device side: torch ops, captured into the graph), and a model's ``apply`` reads
    the replayed minibatch's key with :meth:`device_seed` -- so a captured step draws
    exactly the dropout masks the eager loop draws with ``split(key, n)[i]``.  As a
    plain int it is minibatch 0's key: host code that consumes the int itself (e.g. to
    seed a CPU generator) sees the same value on every replay."""

    def __new__(cls, keys: Sequence[int], dev, index):
        o = int.__new__(cls, int(keys[0]) & _MASK)
        o.keys, o.dev, o.index = [int(k) & _MASK for k in keys], dev, index
        return o

    @classmethod
    def from_keys(cls, keys: Sequence[int], index):
        import torch

        return cls(keys, torch.tensor([_s64(k) for k in keys], dtype=torch.int64, device=index.device), index)

    def fold_in(self, data: int) -> "ScanKey":
        d = _s64(_mix(int(data) & _MASK))
        return ScanKey([fold_in(k, data) for k in self.keys], _mix_t(self.dev ^ d), self.index)

    def device_seed(self, mask: int = 0xFFFFFFFF):
        """int64[1] device tensor: the replayed minibatch's key ``& mask`` (a fresh
        select per call, so a call inside a capture records its own kernels)."""
        return self.dev.index_select(0, self.index.long()) & mask


def fold_in(key: int, data: int) -> int:
    if isinstance(key, ScanKey):
        return key.fold_in(data)
    return _mix((int(key) ^ _mix(int(data) & _MASK)) & _MASK)


def split(key: int, num: int = 2) -> List[int]:
    return [fold_in(key, 0x5EED0000 + i) for i in range(num)]


def fold_rng_over_axis(rng: int, mesh, axis_name: str | None = None) -> int:
    """Give each member of ``axis_name`` its own stream (data_paral.py:28-34).

    Also callable with the reference's signature ``fold_rng_over_axis(rng,
    axis_name)``: the axis is then looked up on the most recently built
    :class:`~jax_distributed_tuts_amd.runtime.dist.Mesh` of this process (the
    analogue of the enclosing ``shard_map``'s mesh); no mesh -> index 0."""
    if isinstance(mesh, str) and axis_name is None:
        from ..runtime.dist import current_mesh

        mesh, axis_name = current_mesh(), mesh
        if mesh is not None and axis_name not in mesh.axis_names:
            mesh = None
    idx = 0 if mesh is None else mesh.axis_index(axis_name)
    return fold_in(rng, idx)
