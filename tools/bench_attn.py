"""Flash attention timings on the transformer LM's shape (B 16, S 128, H 8, Dh 64,
causal): forward, backward with the whole-head kernel and with the key-block
kernel (A/B).  Each timing: 50 launches in one hipGraph, median of 5.

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
    for B, S, H in ((16, 128, 8), (8, 128, 8), (4, 256, 8)):
        d = H * 64
        qkv = torch.randn(B * S, 3 * d, device=dev).to(torch.bfloat16)
        do = torch.randn(B * S, d, device=dev).to(torch.bfloat16)
        o, lse = K.attention_fwd(qkv, B, S, H)
        dq = torch.empty_like(qkv)
        db = torch.zeros(3 * d, device=dev)
        tf = timed(lambda: K.attention_fwd(qkv, B, S, H))
        res = []
        for head in (1, 0):
            _lib.lib().jdt_flash_set_head(head)
            res.append(timed(lambda: K.attention_bwd(do, qkv, lse, B, S, H, dqkv=dq, o=o, dbias=db)))
        _lib.lib().jdt_flash_set_head(1)
        print(f"B={B} S={S} H={H}: fwd {tf:6.2f} us | bwd whole-head {res[0]:6.2f} us | bwd key-block {res[1]:6.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
