"""One LM-chain GEMM shape launched back to back, for rocprofv3 --pmc (L2 hit rate of
the LDS-DMA main loop): fc1's forward (2048 x 2048 x 512, bias + GELU + z store) or any
(M, N, K) given, either on one operand set (warm) or rotating over 8 (operands mostly
beyond the L2, as in the model).

    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -- python3 tools/pmc_lm_gemm.py --cold
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mnk", default="2048,2048,512")
    ap.add_argument("--cold", action="store_true")
    ap.add_argument("--epilogue", action="store_true")
    ap.add_argument("--n", type=int, default=40)
    ap.add_argument("--cfg", type=int, default=-1)
    a = ap.parse_args()
    M, N, Kd = (int(x) for x in a.mnk.split(","))
    sets = 8 if a.cold else 1
    bf = lambda *s: (torch.randn(*s, device="cuda") * 0.05).to(torch.bfloat16)  # noqa: E731
    X = [bf(M, Kd) for _ in range(sets)]
    W = [bf(Kd, N) for _ in range(sets)]
    O = [torch.empty(M, N, device="cuda", dtype=torch.bfloat16) for _ in range(sets)]
    Z = [torch.empty(M, N, device="cuda", dtype=torch.bfloat16) for _ in range(sets)]
    bias = torch.zeros(N, device="cuda")
    kw = {} if a.cfg < 0 else {"cfg": a.cfg}
    for i in range(a.n):
        j = i % sets
        if a.epilogue:
            K.gemm(X[j], W[j], bias=bias, act="gelu", z_out=Z[j], out=O[j], **kw)
        else:
            K.gemm(X[j], W[j], out=O[j], **kw)
    torch.cuda.synchronize()
    print("done", M, N, Kd, "cold" if a.cold else "warm")


if __name__ == "__main__":
    main()
