"""GEMM fixed-cost vs per-K-tile cost: M = N = 2048 (bf16 out, mk x kn) over
K = 64 .. 2048, no split, for a list of tile configs; also a store-only probe
(K = 64) and torch.matmul.  Each timing: 50 launches in one hipGraph, median of 5.

    python tools/gemm_ksweep.py [--cfgs 11,12,14] [--mn 2048]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402
from tools.bench_gemm import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="11,12,14")
    ap.add_argument("--mn", type=int, default=2048)
    ap.add_argument("--layouts", default="mk/kn,mk/nk,km/kn")
    ap.add_argument("--epi", default="1", help="comma list of vectorised-epilogue settings to compare (0,1)")
    ap.add_argument("--group-m", default="0", help="comma list of tile row-group sizes to compare (0 = row-major)")
    ap.add_argument("--ks", default="64,128,256,512,1024,2048")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    M = N = args.mn
    for lay in args.layouts.split(","):
        al, bl = lay.split("/")
        for Kd in (int(k) for k in args.ks.split(",")):
            a = torch.randn(*((M, Kd) if al == "mk" else (Kd, M)), device=dev).to(torch.bfloat16)
            b = torch.randn(*((Kd, N) if bl == "kn" else (N, Kd)), device=dev).to(torch.bfloat16)
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            row = []
            for ev in (int(x) for x in args.epi.split(",")):
                _lib.lib().jdt_gemm_set_epi_vec(ev)
                for cfg in (int(x) for x in args.cfgs.split(",")):
                    for gm in (int(x) for x in args.group_m.split(",")):
                        _lib.lib().jdt_gemm_set_group_m(gm)
                        t = timed(lambda: K.gemm(a, b, a_layout=al, b_layout=bl, out=c, cfg=cfg, splits=1))
                        row.append(f"c{cfg}g{gm} {t:6.2f}")
                    _lib.lib().jdt_gemm_set_group_m(-1)
            _lib.lib().jdt_gemm_set_epi_vec(1)
            tr = timed(lambda: torch.matmul(a if al == "mk" else a.t(), b if bl == "kn" else b.t()))
            fl = 2.0 * M * N * Kd
            print(f"{al}/{bl} M=N={M} K={Kd:5d}: " + " | ".join(row) + f" | torch {tr:6.2f} us ({fl / tr / 1e6:.0f} TF/s)",
                  flush=True)


if __name__ == "__main__":
    main()
