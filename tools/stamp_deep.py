"""Diagnostic: in-kernel phase stamps (s_memrealtime, 100 MHz) of the deep fused
MLP backward launches (csrc/mlp_deep.hip MD_STAMP points): per layer, the median
over workgroups of each phase end relative to the workgroup's start, and the
launch span.

    python tools/stamp_deep.py [--layers 4] [--rows 128]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.models.mlp import Classifier  # noqa: E402
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp  # noqa: E402
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw  # noqa: E402

PH = ["issue loads", "dZ (+CE) -> LDS", "dW MFMA + AdamW", "end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--rows", type=int, default=128)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(args.rows, 784, generator=g).to(dev),
              torch.randint(0, 10, (args.rows,), generator=g).to(torch.int32).to(dev))
    st = init_dp(Classifier(num_layers=args.layers), adamw(1e-3), 69, dev)
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    for _ in range(30):
        tr.step(b)
    eng = tr.fused
    fwd, bwd = eng._args
    bufs = []
    for a in bwd:
        t = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
        a.stamps = t.data_ptr()
        bufs.append(t)
    for _ in range(5):
        tr.step(b)
    torch.cuda.synchronize()
    L = _lib.lib()
    s = _lib.stream_ptr()
    for j, a in enumerate(bwd):
        bufs[j].zero_()
    for i, a in enumerate(fwd):
        L.jdt_md_layer(ctypes.byref(a), 0, int(i == eng.nh - 1), s)
    for j, a in enumerate(bwd):
        L.jdt_md_layer(ctypes.byref(a), 1, int(j == 0), s)
    torch.cuda.synchronize()
    for j, a in enumerate(bwd):
        layer = eng.nh - 1 - j
        kc = 112 if a.K == 784 else 64
        nwg = (a.N // 16) * (a.K // kc)
        st_ = bufs[j][: nwg * 8].view(nwg, 8).double().cpu() * 0.01
        t0 = st_[:, 0]
        print(f"--- md_bwd layer {layer} (K={a.K}, {nwg} WGs) span {float(st_[:, 3].max() - t0.min()):.2f} us, "
              f"start skew {float(t0.max() - t0.min()):.2f}")
        for k in range(1, 4):
            d = st_[:, k] - t0
            print(f"    {PH[k - 1]:20s} end @ median {float(d.median()):5.2f}  max {float(d.max()):5.2f}")


if __name__ == "__main__":
    main()
