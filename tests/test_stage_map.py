"""The FSDP staged bucket (ops/csrc/common.h StageMap / stage_store): a producer that
writes each full-layout gradient element through the map must leave, in every peer
slot q of the staging buffer, exactly the words the fused FSDP collective reads for
part q of each segment (comm/csrc/xgmi.hip ``seg_full_index`` layout).  Pure host
mirror of both index maps over the 2- and 4-layer classifiers' FSDP segments."""
import math

import pytest
import torch

from jax_distributed_tuts_amd.comm.xgmi import XgSeg, XgSegs, geometry, stage_layout
from jax_distributed_tuts_amd.models.mlp import Classifier
from jax_distributed_tuts_amd.parallel.fsdp import shard_rule


def stage_store(layout, slice_, W, name, row, col, v, buf):
    """Python mirror of common.h stage_store (one half), vectorised over index tensors."""
    off, dim, per, cols = layout[name]
    if dim == 2:
        for q in range(W):
            buf[q * slice_ + off + row * cols + col] = v
        return
    q = torch.div(row if dim == 0 else col, per, rounding_mode="floor")
    jj = (row - q * per) * cols + col if dim == 0 else row * per + (col - q * per)
    buf[q * slice_ + off + jj] = v


def seg_full_index(seg, q, jj):
    """Python mirror of xgmi.hip seg_full_index."""
    if seg["rows"] <= 1:
        return (0 if seg["bcast"] else q * seg["s"]) + jj
    w = seg["s"] // seg["rows"]
    r = torch.div(jj, w, rounding_mode="floor")
    return r * seg["ld"] + q * seg["qoff"] + (jj - r * w)


def build(num_layers, W):
    model = Classifier(num_layers=num_layers)
    sharded, repl = [], []
    for s in model.param_specs():
        d, _ = shard_rule(s.shape, (None,) * len(s.shape), "data", W, 16, s.name)
        (repl if d is None else sharded).append((s.name, tuple(s.shape), d))
    segs, off = [], 0
    for name, shape, d in sharded:   # XgmiComm._segs
        n = math.prod(shape)
        if d == 1:
            rows, pw = shape[0], shape[1] // W
            segs.append(dict(name=name, s=n // W, off=off, nfull=n, bcast=0, rows=rows, ld=shape[1], qoff=pw))
        else:
            segs.append(dict(name=name, s=n // W, off=off, nfull=n, bcast=0, rows=0, ld=0, qoff=0))
        off += n // W
    for name, shape, _ in repl:      # XgmiComm.fsdp_plan replicated tail
        n = math.prod(shape)
        w = (n + 3) // 4 * 4
        segs.append(dict(name=name, s=w, off=off, nfull=n, bcast=1, rows=0, ld=0, qoff=0))
        off += w
    segs.append(dict(name="metrics", s=4, off=off, nfull=4, bcast=1, rows=0, ld=0, qoff=0))
    off += 4
    return model, sharded, repl, segs, off


@pytest.mark.parametrize("num_layers", [2, 4])
@pytest.mark.parametrize("W", [2, 4, 8])
def test_producer_map_matches_collective_layout(num_layers, W):
    model, sharded, repl, segs, S_total = build(num_layers, W)
    # the layout fsdp_stage_layout derives from the plan's segment table
    S = XgSegs()
    for k, sg in enumerate(segs):
        S.seg[k] = XgSeg(0, 0, sg["s"], sg["off"], sg["nfull"], sg["bcast"], sg["rows"], sg["ld"], sg["qoff"])
    S.n, S.S = len(segs), S_total
    lay = stage_layout(S, sharded + [(n, s, None) for n, s, _ in repl], W)
    g_, chunk = geometry(S_total)
    slice_ = g_ * chunk
    buf = torch.full((W * slice_,), float("nan"), dtype=torch.float64)
    fulls = {}
    gen = torch.Generator().manual_seed(num_layers * 10 + W)
    for name, shape, _ in sharded + [(n, s, None) for n, s, _ in repl]:
        t = torch.randn(shape, generator=gen, dtype=torch.float64)
        fulls[name] = t
        t2 = t.reshape(shape[0], -1) if len(shape) == 2 else t.reshape(-1, 1)
        r, c = torch.meshgrid(torch.arange(t2.shape[0]), torch.arange(t2.shape[1]), indexing="ij")
        stage_store(lay, slice_, W, name, r.reshape(-1), c.reshape(-1), t2.reshape(-1), buf)
    metrics = torch.tensor([3.0, 32.0, 7.0, 32.0], dtype=torch.float64)
    stage_store(lay, slice_, W, "metrics", torch.arange(4), torch.zeros(4, dtype=torch.int64), metrics, buf)
    fulls["metrics"] = metrics
    # what the collective reads for part q of each segment
    for q in range(W):
        for sg in segs:
            full = fulls[sg["name"]].reshape(-1)
            lim = sg["nfull"] if sg["bcast"] else min(sg["s"], sg["nfull"] - q * sg["s"])
            got = buf[q * slice_ + sg["off"]: q * slice_ + sg["off"] + lim]
            want = full[seg_full_index(sg, q, torch.arange(lim))]
            assert torch.equal(got, want), (sg["name"], q)
