"""Diagnostic: in-kernel phase stamps (s_memrealtime, 100 MHz) of the S <= 128 attention
backward (csrc/attn128.hip attn128_bwd_kernel A_STAMP points, thread 0 = wave 0, which owns
key tile 0: the most dK / dV pairs): per phase the median over workgroups of its end
relative to the workgroup's start, and the launch span.

    python tools/stamp_attn.py [--batch 16]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402

PH = ["staged (Q, K, dO, O loads + delta)", "wave 0 dK/dV loop done", "all waves (barrier)", "wave 0 dQ done",
      "end (dK/dV stores)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--no-dbias", action="store_true", help="without the fused QKV bias gradient")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, S, H = a.batch, 128, 8
    d = H * 64
    qkv = torch.randn(B * S, 3 * d, device=dev).to(torch.bfloat16)
    do = torch.randn(B * S, d, device=dev).to(torch.bfloat16)
    o, lse = K.attention_fwd(qkv, B, S, H)
    dq = torch.empty_like(qkv)
    db = None if a.no_dbias else torch.zeros(3 * d, device=dev)
    st = torch.zeros(B * H * 8, dtype=torch.int64, device=dev)
    L = _lib.lib()
    for _ in range(3):
        K.attention_bwd(do, qkv, lse, B, S, H, dqkv=dq, o=o, dbias=db)
    L.jdt_attn128_set_stamps(ctypes.c_void_p(st.data_ptr()))
    try:
        K.attention_bwd(do, qkv, lse, B, S, H, dqkv=dq, o=o, dbias=db)
        torch.cuda.synchronize()
    finally:
        L.jdt_attn128_set_stamps(None)
    t = st.view(B * H, 8).cpu().double()
    t0 = t[:, 0]
    print(f"attn128_bwd B={B} S={S} H={H}: span {(t[:, 5].max() - t0.min()) / 100:.2f} us, "
          f"start skew {(t0.max() - t0.min()) / 100:.2f} us")
    for k, name in enumerate(PH, start=1):
        rel = (t[:, k] - t0) / 100.0
        print(f"    {name:36s} end @ median {rel.median():6.2f}  max {rel.max():6.2f} us")


if __name__ == "__main__":
    main()
