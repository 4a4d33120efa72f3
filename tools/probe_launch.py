"""Where does a short timed region's fixed cost go?  Headline DP step captured
as one S-step hipGraph (bench.py's schedule): host wall time of replay+sync vs
the GPU time between events recorded around the replay, for S = 1 .. 200, plus an
empty-kernel graph of the same node count.

    python tools/probe_launch.py
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from jax_distributed_tuts_amd.runtime import dist as D  # noqa: E402


def main():
    dev = D.init()
    ap = argparse.Namespace(num_layers=2, optimizer="adamw", accum="kernel", comm="auto")
    tr, batch, _ = bench.build_dp(ap, dev)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    for S in (1, 5, 20, 100, 200):
        tr.capture(batch, steps_per_graph=S)
        gm = tr.multi[1] if tr.multi else tr.graph[1]
        walls, gpus, firsts = [], [], []
        for it in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record()
            gm.replay()
            b.record()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            (firsts if it == 0 else walls).append((t2 - t0) * 1e6)
            gpus.append(a.elapsed_time(b) * 1e3)
            if it == 0:
                launch_us = (t1 - t0) * 1e6
        walls.sort()
        gpus.sort()
        print(f"S={S:4d}: wall {walls[len(walls) // 2]:8.1f} us (first {firsts[0]:8.1f}) | gpu events "
              f"{gpus[len(gpus) // 2]:8.1f} us | per step wall {walls[len(walls) // 2] / S:6.2f} gpu "
              f"{gpus[len(gpus) // 2] / S:6.2f} | host launch call {launch_us:7.1f} us", flush=True)
    # empty kernels, same count per graph
    x = torch.zeros(1, device=dev)
    for n in (2, 40, 200, 400):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n):
                x.add_(1)
        ws = []
        for _ in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            ws.append((time.perf_counter() - t0) * 1e6)
        ws.sort()
        print(f"empty graph {n:4d} kernels: wall {ws[3]:8.1f} us ({ws[3] / n:5.2f} us per kernel)", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        torch.cuda.synchronize()
    print(f"bare synchronize: {(time.perf_counter() - t0) * 1e4:.1f} us", flush=True)


if __name__ == "__main__":
    main()
