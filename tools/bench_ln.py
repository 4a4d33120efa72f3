"""LayerNorm backward sweep: waves per workgroup W x rows per wave R (workgroups = T / (W R)) on the
transformer's [T, d] shapes; each timing = 50 launches in one hipGraph, median of 5.

    python tools/bench_ln.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return sorted(ts)[2]


def main():
    dev = torch.device("cuda", 0)
    for T, d in ((2048, 512), (512, 512), (256, 512)):
        x = torch.randn(T, d, device=dev).to(torch.bfloat16)
        dy = torch.randn(T, d, device=dev).to(torch.bfloat16)
        dres = torch.randn(T, d, device=dev).to(torch.bfloat16)
        gamma = torch.rand(d, device=dev) + 0.5
        _, mean, rstd = K.layernorm_fwd(x, gamma, torch.zeros(d, device=dev))
        dg, db, ds = (torch.zeros(d, device=dev) for _ in range(3))
        row = []
        for W, R in ((0, 0), (4, 2), (4, 4), (4, 8), (8, 1), (8, 2), (8, 4), (16, 1), (16, 2)):
            _lib.lib().jdt_ln_set_waves(W)
            _lib.lib().jdt_ln_set_rows(R)
            t = timed(lambda: K.layernorm_bwd(dy, x, mean, rstd, gamma, dg, db, dres=dres, dsum=ds))
            row.append(f"W{W}R{R}: {t:5.2f}" if W else f"auto: {t:5.2f}")
        _lib.lib().jdt_ln_set_waves(0)
        _lib.lib().jdt_ln_set_rows(0)
        # floors: the same kernel without the column-sum outputs (no atomics), a
        # forward, and a bf16 add of two [T, d] tensors (3 tensor passes)
        t_na = timed(lambda: K.layernorm_bwd(dy, x, mean, rstd, gamma, None, None, dres=dres, dsum=None))
        t_f = timed(lambda: K.layernorm_fwd(x, gamma, torch.zeros(d, device=dev)))
        t_add = timed(lambda: torch.add(dy, dres))
        print(f"ln_bwd T={T} d={d}: " + " | ".join(row) +
              f" | no colsums {t_na:6.2f} | ln_fwd {t_f:6.2f} | torch add {t_add:6.2f} us")


if __name__ == "__main__":
    main()
