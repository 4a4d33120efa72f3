"""RNG folding (data_paral.py:28-34 ``fold_rng_over_axis``; util.py:51, 91 ``split``).

JAX threads explicit PRNG keys; on MI355X dropout is a counter-based Philox
stream addressed by (seed, offset) and regenerated in the backward epilogue, so
a "key" here is a 64-bit integer.  ``split``/``fold_in`` are deterministic
integer mixes (splitmix64), which gives the same statistical contract as
threefry: independent streams per (step, minibatch, device).  Bit parity with
JAX's threefry is out of scope.
"""
from __future__ import annotations

from typing import List

_MASK = (1 << 64) - 1


def _mix(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK
    return z ^ (z >> 31)


def PRNGKey(seed: int) -> int:
    return _mix(int(seed) & _MASK)


def fold_in(key: int, data: int) -> int:
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
