"""Gradient buckets whose all-reduce overlaps the rest of the backward pass.

The reference all-reduces after the whole step's gradient is known
(``pmean`` at data_paral.py:210-212; XLA decides the scheduling).  Here the
explicit-backward models report parameters as soon as their gradients are
final (``backward(on_ready=...)``, output layer first); a bucket -- a
contiguous range of the flat gradient buffer, sized for the xGMI ring
(default 25 MiB: large enough to stay bandwidth-bound on one link, small
enough that the first buckets leave while the lower layers still compute) --
is all-reduced asynchronously on RCCL's stream the moment its last member is
ready.  The 4 metric scalars ride in the output-side bucket.  ``finish()``
makes the compute stream wait for every bucket before the optimizer.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import math

import torch
import torch.distributed as dist

from ..runtime.dist import Mesh
from ..utils.flat import FlatParams


class GradBuckets:
    def __init__(self, P: FlatParams, mesh: Optional[Mesh], axis: str, bucket_bytes: int = 25 << 20):
        self.P, self.mesh, self.axis = P, mesh, axis
        from .collectives import active

        self.active = active(mesh, axis)
        specs = list(P.specs)
        groups: List[List[str]] = []
        cur: List[str] = []
        size = 0
        for s in reversed(specs):  # output side first = the order backward finishes them
            cur.append(s.name)
            size += 4 * int(math.prod(s.shape))
            if size >= bucket_bytes:
                groups.append(cur)
                cur, size = [], 0
        if cur:
            groups.append(cur)
        self.ranges: List[Tuple[int, int]] = []
        hi = P.grad.numel()  # first (output-side) bucket also carries the metric slots
        for gi, names in enumerate(groups):
            lo = 0 if gi == len(groups) - 1 else min(P.offsets[n][0] for n in names)
            self.ranges.append((lo, hi))
            hi = lo
        self.bucket_of: Dict[str, int] = {n: gi for gi, names in enumerate(groups) for n in names}
        self.sizes = [len(g) for g in groups]
        self.pending: List[int] = []
        self.works = []
        self.launched: List[bool] = []

    def begin(self):
        self.pending = list(self.sizes)
        self.launched = [False] * len(self.sizes)
        self.works = []

    def _launch(self, b: int):
        if self.launched[b]:
            return
        self.launched[b] = True
        lo, hi = self.ranges[b]
        self.works.append(dist.all_reduce(self.P.grad[lo:hi], op=dist.ReduceOp.SUM,
                                          group=self.mesh.group(self.axis), async_op=True))

    def ready(self, names):
        if not self.active or not self.pending:
            return
        for n in names:
            b = self.bucket_of.get(n)
            if b is None:
                continue
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._launch(b)

    def finish(self):
        if not self.active:
            return
        if not self.pending:
            self.begin()
        for b in range(len(self.sizes)):
            self._launch(b)  # anything never reported (or no overlap this step)
        for w in self.works:
            w.wait()
        self.pending = []
