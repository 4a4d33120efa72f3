"""Where does the driver form's fixed cost go with the persistent headline kernel?  For
20 steps: host wall of (replay + synchronize) for the captured 20-step graph (one kernel
node) vs a direct launch of the same persistent kernel, vs GPU time between events.

    python tools/probe_pst_launch.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from jax_distributed_tuts_amd.runtime import dist as D  # noqa: E402


def main():
    dev = D.init()
    import argparse
    ns = argparse.Namespace(num_layers=2, optimizer="adamw", accum="kernel", comm="auto")
    tr, batch, _ = bench.build_dp(ns, dev)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    S = 20
    tr.capture(batch, steps_per_graph=S)
    tr.run_steps(batch, S)
    eng = tr.fused
    torch.cuda.synchronize()
    for label, fn in (("graph replay", lambda: tr.run_steps(batch, S)),
                      ("direct launch", lambda: eng.run_ahead(batch, S, prologue=False))):
        walls, gpus = [], []
        for _ in range(30):
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            gpus.append(a.elapsed_time(b) * 1e3)
        walls.sort(); gpus.sort()
        print(f"{label:14s}: wall median {walls[15]:7.1f} us (min {walls[0]:7.1f}) | events median {gpus[15]:7.1f} us"
              f" -> {S / walls[15] * 1e6:,.0f} steps/s by wall")
    tr.finalize()


if __name__ == "__main__":
    main()
