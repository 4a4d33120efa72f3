"""The transformer LM step's input-gradient-chain GEMMs at the bench configuration
(2048 tokens, d 512, d_ff 2048, V 2048), each with exactly the epilogue the model gives
it (bias, GELU + pre-activation store, residual, GELU' + bias-grad), against the same
GEMM without the epilogue: 50 copies captured in one hipGraph, operands rotated over 8
buffer sets so most reads miss the L2 as in the model.  Tells how much of an in-model
GEMM is the epilogue and how much is the main loop on cold operands.

    python tools/bench_lm_gemms.py [--sweep 10,11,15,...]

--sweep: every case again with each forced tile config (ops.kernels.gemm cfg=).
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import argparse  # noqa: E402

from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402

T, D, F, V = 2048, 512, 2048, 2048
SETS = 8


def bf(*shape):
    return (torch.randn(*shape, device="cuda") * 0.05).to(torch.bfloat16)


def timed(fn, n=50, reps=10):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for i in range(SETS):
            fn(i)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(n):
                fn(i % SETS)
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", default="")
    ap.add_argument("--gm", type=int, default=-1,
                    help="force the tile row-group size of every GEMM (csrc/gemm.hip group_m; -1 = table)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    if a.gm >= 0:
        from jax_distributed_tuts_amd.ops import _lib
        _lib.lib().jdt_gemm_set_group_m(a.gm)
    W = {n: [bf(k, m) for _ in range(SETS)] for n, (k, m) in
         {"qkv": (D, 3 * D), "out": (D, D), "fc1": (D, F), "fc2": (F, D), "head": (D, V)}.items()}
    bias = {n: torch.zeros(W[n][0].shape[1], device="cuda") for n in W}
    X = {n: [bf(T, k) for _ in range(SETS)] for n, k in (("d", D), ("f", F), ("q", 3 * D), ("v", V))}
    Z = [bf(T, F) for _ in range(SETS)]
    outs = {n: [torch.empty(T, k, device="cuda", dtype=torch.bfloat16) for _ in range(SETS)]
            for n, k in (("d", D), ("f", F), ("q", 3 * D), ("v", V))}
    g1 = torch.zeros(F, device="cuda")
    cases = [
        ("qkv fwd", lambda i: K.gemm(X["d"][i], W["qkv"][i], bias=bias["qkv"], out=outs["q"][i]),
         lambda i: K.gemm(X["d"][i], W["qkv"][i], out=outs["q"][i])),
        ("out fwd +resid", lambda i: K.gemm(X["d"][i], W["out"][i], bias=bias["out"], resid=X["d"][(i + 1) % SETS],
                                            out=outs["d"][i]),
         lambda i: K.gemm(X["d"][i], W["out"][i], out=outs["d"][i])),
        ("fc1 fwd gelu+z", lambda i: K.gemm(X["d"][i], W["fc1"][i], bias=bias["fc1"], act="gelu", z_out=Z[i],
                                            out=outs["f"][i]),
         lambda i: K.gemm(X["d"][i], W["fc1"][i], out=outs["f"][i])),
        ("fc2 fwd +resid", lambda i: K.gemm(X["f"][i], W["fc2"][i], bias=bias["fc2"], resid=X["d"][i],
                                            out=outs["d"][i]),
         lambda i: K.gemm(X["f"][i], W["fc2"][i], out=outs["d"][i])),
        ("head fwd", lambda i: K.gemm(X["d"][i], W["head"][i], bias=bias["head"], out=outs["v"][i]),
         lambda i: K.gemm(X["d"][i], W["head"][i], out=outs["v"][i])),
        ("head dX", lambda i: K.gemm(X["v"][i], W["head"][i], b_layout="nk", out=outs["d"][i]), None),
        ("fc2 dX gelu'+db", lambda i: K.gemm(X["d"][i], W["fc2"][i], b_layout="nk", z_in=Z[i], act_bwd="gelu",
                                             dbias=g1, out=outs["f"][i]),
         lambda i: K.gemm(X["d"][i], W["fc2"][i], b_layout="nk", out=outs["f"][i])),
        ("fc2 dX gelu' no db", lambda i: K.gemm(X["d"][i], W["fc2"][i], b_layout="nk", z_in=Z[i], act_bwd="gelu",
                                                out=outs["f"][i]), None),
        ("fc1 dX", lambda i: K.gemm(X["f"][i], W["fc1"][i], b_layout="nk", out=outs["d"][i]), None),
        ("out dX", lambda i: K.gemm(X["d"][i], W["out"][i], b_layout="nk", out=outs["d"][i]), None),
        ("qkv dX", lambda i: K.gemm(X["q"][i], W["qkv"][i], b_layout="nk", out=outs["d"][i]), None),
    ]
    tot = 0.0
    for name, fn, plain in cases:
        t = timed(fn)
        tp = timed(plain) if plain is not None else float("nan")
        tot += t
        print(f"{name:18s} {t:7.2f} us  (no epilogue {tp:7.2f})")
    print(f"sum {tot:.1f} us (x4 layers for the per-layer ones in the step)")
    if not a.sweep:
        return
    cfgs = [int(c) for c in a.sweep.split(",")]
    orig = K.gemm
    for name, fn, _ in cases:
        row = []
        for c in cfgs:
            K.gemm = lambda *args, _c=c, **kw: orig(*args, cfg=_c, **kw)
            try:
                row.append(f"{c}:{timed(fn):6.2f}")
            except Exception as e:  # noqa: BLE001 -- a tile outside the shape's envelope
                row.append(f"{c}:  n/a ")
                print(f"  ({name} cfg {c}: {str(e)[:60]})", file=sys.stderr)
            finally:
                K.gemm = orig
        print(f"{name:18s} " + "  ".join(row))


if __name__ == "__main__":
    main()
