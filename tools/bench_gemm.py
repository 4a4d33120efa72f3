"""GEMM micro-benchmark on the transformer / MLP shapes: our gfx950 kernel (each
layout the models use) vs torch.matmul (hipBLASLt) on the same operands.
Each timing is 50 back-to-back launches captured in one hipGraph (no host
launch cost), median of 5 replays.

    python tools/bench_gemm.py [--cfg N] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402

REPS = 50

# (name, M, N, K, a_layout, b_layout, fp32-accumulate output)
SHAPES = [
    ("qkv fwd", 512, 1536, 512, "mk", "kn", False),
    ("out fwd", 512, 512, 512, "mk", "kn", False),
    ("fc1 fwd", 512, 2048, 512, "mk", "kn", False),
    ("fc2 fwd", 512, 512, 2048, "mk", "kn", False),
    ("head fwd", 512, 2048, 512, "mk", "kn", False),
    ("fc1 dX", 512, 512, 2048, "mk", "nk", False),
    ("fc2 dX", 512, 2048, 512, "mk", "nk", False),
    ("fc1 dW", 512, 2048, 512, "km", "kn", True),
    ("fc2 dW", 2048, 512, 512, "km", "kn", True),
    ("qkv fwd 2k", 2048, 1536, 512, "mk", "kn", False),
    ("fc2 fwd 2k", 2048, 512, 2048, "mk", "kn", False),
    ("fc1 dW 2k", 512, 2048, 2048, "km", "kn", True),
    ("fc1 fwd 2k", 2048, 2048, 512, "mk", "kn", False),
    ("fc2 dX 2k", 2048, 2048, 512, "mk", "nk", False),
    ("fc1 dX 2k", 2048, 512, 2048, "mk", "nk", False),
    ("fc2 dW 2k", 2048, 512, 2048, "km", "kn", True),
    ("qkv dW 2k", 512, 1536, 2048, "km", "kn", True),
    ("out fwd 2k", 2048, 512, 512, "mk", "kn", False),
    ("out dX 2k", 2048, 512, 512, "mk", "nk", False),
    ("qkv dX 2k", 2048, 512, 1536, "mk", "nk", False),
    ("out dW 2k", 512, 512, 2048, "km", "kn", True),
    ("hyb qkv fwd", 256, 1536, 512, "mk", "kn", False),
    ("hyb fc2 fwd", 256, 512, 2048, "mk", "kn", False),
    ("mlp fwd", 32, 512, 512, "mk", "kn", False),
    ("mlp dW", 512, 512, 32, "km", "kn", True),
]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            fn()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / REPS)
    ts.sort()
    return ts[2]


# the transformer backward's grouped launches (2048 tokens, d 512, ff 2048, V 2048):
# a layer's weight gradient h^T dz and input gradient dz W^T in ONE gemm_group
GROUPS = [
    ("fc2 bwd", [(2048, 512, 2048, "km", "kn", True), (2048, 2048, 512, "mk", "nk", False)]),
    ("fc1 bwd", [(512, 2048, 2048, "km", "kn", True), (2048, 512, 2048, "mk", "nk", False)]),
    ("qkv bwd", [(512, 1536, 2048, "km", "kn", True), (2048, 512, 1536, "mk", "nk", False)]),
    ("out bwd", [(512, 512, 2048, "km", "kn", True), (2048, 512, 512, "mk", "nk", False)]),
]


def bench_groups(dev, tile: int):
    from jax_distributed_tuts_amd.ops import _lib
    _lib.lib().jdt_gemm_set_group_tile(tile)
    res = []
    for name, probs in GROUPS:
        ops = []
        fl = 0.0
        for M, N, Kd, al, bl, f32 in probs:
            a = torch.randn(*((M, Kd) if al == "mk" else (Kd, M)), device=dev).to(torch.bfloat16)
            b = torch.randn(*((Kd, N) if bl == "kn" else (N, Kd)), device=dev).to(torch.bfloat16)
            c = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
            ops.append((a, b, c, al, bl, f32))
            fl += 2.0 * M * N * Kd

        def run():
            with K.gemm_group():
                for a, b, c, al, bl, f32 in ops:
                    K.gemm(a, b, a_layout=al, b_layout=bl, out=c, accumulate=f32)

        t = timed(run)
        tref = timed(lambda: [torch.matmul(a if al == "mk" else a.t(), b if bl == "kn" else b.t())
                              for a, b, c, al, bl, f32 in ops])
        # numerics
        for a, b, c, al, bl, f32 in ops:
            c.zero_()
        run()
        err = 0.0
        for a, b, c, al, bl, f32 in ops:
            want = (a if al == "mk" else a.t()).float() @ (b if bl == "kn" else b.t()).float()
            err = max(err, float((c.float() - want).abs().max() / (want.abs().max() + 1e-6)))
        print(f"group {name:10s} tile {tile:3d}: {t:8.2f} us {fl / t / 1e6:7.1f} TF/s | torch {tref:8.2f} us "
              f"{fl / tref / 1e6:7.1f} TF/s | rel err {err:.2e}")
        res.append({"group": name, "tile": tile, "ours_us": t, "torch_us": tref, "rel_err": err})
    _lib.lib().jdt_gemm_set_group_tile(0)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--json", default=None)
    ap.add_argument("--exact", type=int, default=0, help="force the exact-slice depth (0 = heuristic)")
    ap.add_argument("--splits", type=int, default=-1)
    ap.add_argument("--only", default=None, help="comma-separated shape names to run (e.g. 'qkv fwd,fc1 dW')")
    ap.add_argument("--groups", default=None, help="comma-separated group tiles to sweep (e.g. '32,64,128'; 0 = auto)")
    ap.add_argument("--r", type=int, default=-1, help="64-deep K sub-tiles per LDS ring slot (-1 auto)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    from jax_distributed_tuts_amd.ops import _lib
    _lib.lib().jdt_gemm_set_exact(args.exact)
    _lib.lib().jdt_gemm_set_r(args.r)
    out = []
    print(f"{'shape':14s} {'M':>5s} {'N':>5s} {'K':>5s} {'ours us':>9s} {'TF/s':>7s} {'torch us':>9s} {'TF/s':>7s}")
    only = set(x.strip() for x in args.only.split(",")) if args.only else None
    for name, M, N, Kd, al, bl, f32 in SHAPES:
        if only and name not in only:
            continue
        a = torch.randn(*((M, Kd) if al == "mk" else (Kd, M)), device=dev).to(torch.bfloat16)
        b = torch.randn(*((Kd, N) if bl == "kn" else (N, Kd)), device=dev).to(torch.bfloat16)
        c = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        try:
            ours = timed(lambda: K.gemm(a, b, a_layout=al, b_layout=bl, out=c, accumulate=f32, cfg=args.cfg,
                                         splits=args.splits))
        except RuntimeError:
            print(f"{name:14s} {M:5d} {N:5d} {Kd:5d}   (config not applicable)")
            continue
        am = a if al == "mk" else a.t()
        bm = b if bl == "kn" else b.t()
        ref = timed(lambda: torch.matmul(am, bm))
        fl = 2.0 * M * N * Kd
        print(f"{name:14s} {M:5d} {N:5d} {Kd:5d} {ours:9.2f} {fl / ours / 1e6:7.1f} {ref:9.2f} {fl / ref / 1e6:7.1f}")
        # numerics spot check
        c.zero_()
        K.gemm(a, b, a_layout=al, b_layout=bl, out=c, accumulate=f32, cfg=args.cfg, splits=args.splits)
        want = (am.float() @ bm.float())
        err = float((c.float() - want).abs().max() / (want.abs().max() + 1e-6))
        out.append({"shape": name, "M": M, "N": N, "K": Kd, "ours_us": ours, "torch_us": ref, "rel_err": err})
        if err > 2e-2:
            print(f"   !! rel err {err:.3e}")
    if args.groups:
        for t in args.groups.split(","):
            out.extend(bench_groups(dev, int(t)))
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
