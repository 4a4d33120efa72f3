"""Per-kernel cost floor inside a hipGraph on this GPU: 100 back-to-back copies of a
trivial kernel captured once and replayed; prints microseconds per kernel.  Tells how
much of a launch-heavy step (the transformer LM: ~67 kernels per step) is launch
boundaries rather than work.

    python tools/launch_floor.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_kernel_us(fn, n=100, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (n * reps)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rows = []
    for numel, label in ((1, "fill 1 float (1 workgroup)"), (1 << 16, "fill 256 KB"), (1 << 20, "fill 4 MB"),
                         (1 << 22, "fill 16 MB")):
        t = torch.empty(numel, device=dev)
        rows.append((label, per_kernel_us(lambda t=t: t.fill_(1.0))))
    from jax_distributed_tuts_amd.ops import kernels as K

    x = torch.randn(2048, 512, device=dev).to(torch.bfloat16)
    gm, bt = torch.ones(512, device=dev), torch.zeros(512, device=dev)
    rows.append(("ln_fwd 2048 x 512", per_kernel_us(lambda: K.layernorm_fwd(x, gm, bt, 1e-6))))
    for label, us in rows:
        print(f"{label:32s} {us:7.2f} us per kernel")


if __name__ == "__main__":
    main()
