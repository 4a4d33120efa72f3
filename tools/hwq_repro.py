"""Minimal reproducer (no jdt kernels): a hipGraph with k fork/join branches captured
from k streams, replayed in a process with fewer hardware queues.

    GPU_MAX_HW_QUEUES=2 python tools/hwq_repro.py --streams 4

Round 4 found the 4-stream LM step (parallel/pipeline.py) segfaulting inside the
first hipGraphLaunch with GPU_MAX_HW_QUEUES=2 while the same streams run correctly
eagerly (profiles/r4_hwq2_diagnosis.txt).  This script captures the same graph
SHAPE with plain torch ops only -- main stream forks to k - 1 side streams, each
runs a chain of elementwise kernels, main joins them -- to tell a HIP-runtime
defect from a fault of ours.  Prints one line per stage, so a crash names it."""
from __future__ import annotations

import argparse
import faulthandler
import os
import sys

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--chain", type=int, default=8)
    ap.add_argument("--replays", type=int, default=5)
    a = ap.parse_args()
    faulthandler.enable(all_threads=True)
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', '(default)')} streams={a.streams}", flush=True)
    dev = torch.device("cuda", 0)
    k = a.streams
    xs = [torch.randn(1 << 16, device=dev) for _ in range(k)]
    side = [torch.cuda.Stream(dev) for _ in range(k - 1)]

    def body():
        main_s = torch.cuda.current_stream(dev)   # the capture stream while capturing
        for s in side:
            s.wait_stream(main_s)
        for i in range(k):
            ctx = torch.cuda.stream(side[i - 1]) if i else torch.cuda.stream(main_s)
            with ctx:
                for _ in range(a.chain):
                    xs[i].mul_(1.0001).add_(0.5)
        for s in side:
            main_s.wait_stream(s)

    body()
    torch.cuda.synchronize()
    print("eager ok", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    print("captured", flush=True)
    for r in range(a.replays):
        g.replay()
        torch.cuda.synchronize()
        print(f"replay {r} ok", flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    sys.exit(main())
