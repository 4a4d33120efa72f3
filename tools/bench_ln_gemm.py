"""LayerNorm-fused GEMM (csrc/gemm.hip gemm_ln_kernel) against ln_fwd + gemm on the
transformer's LN -> projection shapes, per tile config.  50 launches per hipGraph,
median of 5 (tools/bench_gemm.timed).

    python tools/bench_ln_gemm.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402
from tools.bench_gemm import timed  # noqa: E402

SHAPES = [("qkv 2k", 2048, 512, 1536, "none"), ("fc1 2k", 2048, 512, 2048, "gelu"), ("head 2k", 2048, 512, 2048, "none"),
          ("qkv 512", 512, 512, 1536, "none"), ("fc1 512", 512, 512, 2048, "gelu"), ("qkv 256", 256, 512, 1536, "none")]


def main():
    dev = torch.device("cuda", 0)
    for name, M, Kd, N, act in SHAPES:
        x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        g, b = torch.ones(Kd, device=dev), torch.zeros(Kd, device=dev)
        w = (torch.randn(Kd, N, device=dev) / Kd ** 0.5).to(torch.bfloat16)
        bias = torch.zeros(N, device=dev).to(torch.bfloat16)
        z = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if act != "none" else None

        def two():
            y, _, _ = K.layernorm_fwd(x, g, b)
            K.gemm(y, w, bias=bias, act=act, z_out=z)

        line = f"{name:8s} {M}x{N}x{Kd}: ln+gemm {timed(two):6.2f}"
        for cfg in (0, 1, 2, 3, 4):
            _lib.lib().jdt_gemm_ln_set_cfg(cfg)
            line += f" | c{cfg} {timed(lambda: K.ln_gemm(x, g, b, w, bias=bias, act=act, z_out=z)):6.2f}"
        _lib.lib().jdt_gemm_ln_set_cfg(0)
        print(line + " us", flush=True)


if __name__ == "__main__":
    main()
