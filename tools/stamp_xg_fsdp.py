"""Diagnostic: phase stamps of the fused FSDP step collective (comm/csrc/xgmi.hip
``xg_fsdp_kernel``) -- stage, barrier A, reduce + sharded AdamW + publish, barrier B,
bf16 gather -- on N ranks sharing the box's GPU (gloo bootstrap, xGMI IPC kernels).
Prints rank 0's per-phase medians over blocks (us from each block's start) and the
eager step's per-launch device times.

    python tools/stamp_xg_fsdp.py [--ranks 2] [--layers 2]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

PH = ["stage stored", "barrier A", "reduce+AdamW+publish", "barrier B", "gather bf16"]


def body(layers: int, reps: int):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.utils.config import fsdp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    dev = D.device()
    mesh = D.Mesh({"data": D.world_size()})
    cfg = fsdp_config()
    st = init_fsdp(Classifier(num_layers=layers), adamw(1e-4), 6969, dev, mesh, "data", 16)
    b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=True,
                                          comm="xgmi"))
    for _ in range(5):
        tr.step(b)
    torch.cuda.synchronize()
    plan = tr._fsdp_plan()
    assert plan is not None, "fused FSDP collective not in use"
    S, F = plan
    G = 96
    stamps = torch.zeros(G * 8, dtype=torch.int64, device=dev)
    F.stamps = ctypes.c_void_p(stamps.data_ptr())
    rows = []
    for _ in range(reps):
        stamps.zero_()
        D.barrier()
        tr.step(b)
        torch.cuda.synchronize()
        s = stamps.view(G, 8).cpu().double()
        s = s[s[:, 0] > 0]
        rows.append(s)
    F.stamps = ctypes.c_void_p(0)
    tr.finalize()
    if D.rank() == 0:
        s = torch.cat(rows)
        t0 = s[:, 0:1]
        d = (s[:, 1:6] - t0) * 1e-2   # 100 MHz ticks -> us
        print(f"ranks {D.world_size()}, {layers}-layer classifier, {s.shape[0] // reps} blocks, {reps} steps")
        for i, n in enumerate(PH):
            print(f"  {n:22s} end @ median {float(d[:, i].median()):6.2f} us   max {float(d[:, i].max()):6.2f}")
        print(f"  start skew within a launch (median over steps): "
              f"{float(torch.stack([(r[:, 0].max() - r[:, 0].min()) * 1e-2 for r in rows]).median()):.2f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from jax_distributed_tuts_amd.runtime.launch import spawn

    spawn(body, a.ranks, a.layers, a.reps, gpu=True)


if __name__ == "__main__":
    main()
