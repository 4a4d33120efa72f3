"""Attention timings on the transformer LM's shapes (S 128, H 8, Dh 64, causal):
the S <= 128 kernels (csrc/attn128.hip) against the tile-streaming flash kernels
(csrc/flash_attn.hip), forward and backward (A/B).  Each timing: 50 launches in one hipGraph, median of 5.

    python tools/bench_attn.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402
from tools.bench_gemm import timed  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for B, S, H in ((16, 128, 8), (4, 128, 8), (2, 128, 8), (4, 256, 8)):
        d = H * 64
        qkv = torch.randn(B * S, 3 * d, device=dev).to(torch.bfloat16)
        do = torch.randn(B * S, d, device=dev).to(torch.bfloat16)
        o, lse = K.attention_fwd(qkv, B, S, H)
        dq = torch.empty_like(qkv)
        db = torch.zeros(3 * d, device=dev)
        line = f"B={B} S={S} H={H}:"
        for a128 in ((1, 0) if S <= 128 else (0,)):
            _lib.lib().jdt_flash_set_attn128(a128)
            o, lse = K.attention_fwd(qkv, B, S, H)
            tf = timed(lambda: K.attention_fwd(qkv, B, S, H))
            tb = timed(lambda: K.attention_bwd(do, qkv, lse, B, S, H, dqkv=dq, o=o, dbias=db))
            line += f" | {'attn128' if a128 else 'flash'} fwd {tf:6.2f} bwd {tb:6.2f} us"
        _lib.lib().jdt_flash_set_attn128(1)
        print(line, flush=True)


if __name__ == "__main__":
    main()
