"""Diagnostic: phase stamps of the one-launch N > 1 DP step (csrc/mlp_fused.hip mlp2_bwd
AHEAD with the per-tile gradient exchange, comm/tile_exchange.py), rank 0 of W ranks.

    JDT_BACKEND=gloo python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29513 tools/stamp_dp_tx.py

Prints, over workgroups (median / max, us from each workgroup's start), the end of the
backward's dW1 MFMAs, the exchange's start and end (slots 12 / 13), AdamW, the next
step's forward phases, and the launch span.
"""
from __future__ import annotations

import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.models.mlp import Classifier  # noqa: E402
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp  # noqa: E402
from jax_distributed_tuts_amd.runtime import dist as D  # noqa: E402
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw  # noqa: E402


def main():
    dev = D.init()
    W, r = D.world_size(), D.rank()
    rows = 128 // W
    g = torch.Generator().manual_seed(r)
    b = Batch(torch.randn(rows, 784, generator=g).to(dev),
              torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(dev))
    mesh = D.Mesh({"data": W})
    st = init_dp(Classifier(), adamw(1e-3), 69, dev)
    tr = DataParallelTrainer(st, mesh, DPConfig(4, "kernel"))
    for _ in range(3):
        tr.step(b)
    torch.cuda.synchronize()
    eng = tr.fused
    if not tr.one_launch:
        print(f"[rank {r}] one-launch step not available here (JDT_DP_AHEAD / co-residency)", flush=True)
        D.shutdown()
        return
    L = _lib.lib()
    s = _lib.stream_ptr()
    T = type(eng._ahead_args)
    ah = T()
    ctypes.memmove(ctypes.byref(ah), ctypes.byref(eng._ahead_args), ctypes.sizeof(T))
    sc = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
    ah.stamps = sc.data_ptr()
    spans = []
    n = (512 // 16) * 7
    for _ in range(20):
        D.barrier()
        _lib.check(L.jdt_mlp2(ctypes.byref(ah), 2, 784, 10, s), "bwd_ahead_tx")
        torch.cuda.synchronize()
        x = sc.cpu()[: n * 16].view(n, 16).double() * 10e-3
        spans.append(x)
    D.barrier()
    if r == 0:
        allx = torch.stack(spans)   # [iters, n, 16]
        rel = allx - allx[:, :, :1]
        print(f"ranks {W}, {rows} rows per rank, {n} workgroups, {len(spans)} launches (medians over both)")
        for i, nm in ((1, "CE+X/LDS staged"), (2, "dZ1"), (12, "exchange start (dW1 MFMA done)"),
                      (13, "exchange end (sums in)"), (3, "AdamW done"), (8, "Z1 partial stored"),
                      (9, "column barrier passed"), (11, "epilogue share"), (4, "logit atomics, end")):
            d = rel[:, :, i].reshape(-1)
            print(f"  {nm:32s} end @ median {float(d.median()):6.2f} us  max {float(d.max()):6.2f}")
        sp = (allx[:, :, 4].max(dim=1).values - allx[:, :, 0].min(dim=1).values)
        print(f"  launch span first start -> last end: median {float(sp.median()):.2f} us")
        ex = (allx[:, :, 13] - allx[:, :, 12]).reshape(-1)
        print(f"  exchange (slot 13 - 12) per workgroup: median {float(ex.median()):.2f} us, "
              f"p90 {float(ex.quantile(0.9)):.2f}")
    eng.finalize()
    D.shutdown()


if __name__ == "__main__":
    main()
