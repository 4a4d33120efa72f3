"""Diagnostic: phase-edge stamps (s_memrealtime, 100 MHz) of the persistent
n-step classifier kernel (csrc/mlp_fused.hip, mlp2_loop_kernel LSTAMP points).
Per step it prints the median / max over workgroups of: forward body, wait in
the first grid barrier, backward body, wait in the second barrier, and the
per-step period.

    python tools/stamp_loop.py [--rows 128] [--steps 10]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.models.mlp import Classifier  # noqa: E402
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp  # noqa: E402
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw  # noqa: E402


def main():
    os.environ.setdefault("JDT_MLP2_LOOP", "1")
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(args.rows, 784, generator=g).to(dev),
              torch.randint(0, 10, (args.rows,), generator=g).to(torch.int32).to(dev))
    st = init_dp(Classifier(), adamw(1e-3), 69, dev)
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    tr.step(b)
    eng = tr.fused
    assert eng.loop_ok, "loop kernel unavailable"
    n = args.steps
    G = max((args.rows + 15) // 16 * 32, 32 * 7)
    stamps = torch.zeros(G * n * 5, dtype=torch.int64, device=dev)
    for _ in range(20):   # warm
        eng.run_loop(b, n)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(50):
        eng.run_loop(b, n)
    ev1.record()
    torch.cuda.synchronize()
    print(f"unstamped: {ev0.elapsed_time(ev1) * 1e3 / (50 * n):.2f} us/step ({n} steps per launch)")
    eng.run_loop(b, n, stamps=stamps)
    torch.cuda.synchronize()
    s = stamps.view(G, n, 5).double().cpu() * 0.01   # ticks -> us
    s = s - s[:, 0:1, 0:1].min()
    names = ["fwd body", "barrier 1 wait", "bwd body", "barrier 2 wait"]
    for it in range(n):
        row = []
        for k in range(4):
            if it == n - 1 and k == 3:
                continue
            d = s[:, it, k + 1] - s[:, it, k]
            row.append(f"{names[k]} med {float(d.median()):5.2f} max {float(d.max()):5.2f}")
        end = s[:, it, 4 if it < n - 1 else 3]
        print(f"step {it}: " + " | ".join(row) + f" | phase-end spread {float(end.max() - end.min()):.2f}")
    per = (s[:, n - 1, 3].max() - s[:, 0, 0].min()) / n
    print(f"stamped: {float(per):.2f} us/step")


if __name__ == "__main__":
    main()
