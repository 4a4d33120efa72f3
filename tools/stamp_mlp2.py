"""Diagnostic: in-kernel phase stamps (s_memrealtime, 100 MHz) of the fused
classifier step kernels (csrc/mlp_fused.hip STAMP points).  Prints, per kernel,
the median over workgroups of each phase's end relative to that workgroup's
start, plus the span from the first workgroup start to the last end.

    python tools/stamp_mlp2.py [--rows 128]
"""
from __future__ import annotations

import argparse
import copy
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.models.mlp import Classifier  # noqa: E402
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp  # noqa: E402
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw  # noqa: E402

NAMES = {0: ["start", "loads+LDS staged", "MFMA+reduce", "epilogue(Z1,H1)", "logit atomics"],
         1: ["start", "CE+X/LDS staged", "dZ1", "dW1 MFMA+AdamW", "db1/dW2/db2"]}


def report(kind, st, nwg):
    raw = st[: nwg * 16].view(nwg, 16).double()
    clk = (raw[:, 6] - raw[:, 5]) / (raw[:, 4] - raw[:, 0]) * 100.0  # MHz
    print(f"    shader clock during the kernel: median {float(clk.median()):.0f} MHz "
          f"(min {float(clk.min()):.0f}, max {float(clk.max()):.0f})")
    st = raw * 10e-3  # ticks -> us
    t0 = st[:, 0]
    print(f"--- {['mlp2_fwd', 'mlp2_bwd'][kind]}  ({nwg} WGs)  span first-start->last-end: "
          f"{float(st[:, 4].max() - t0.min()):.2f} us; start skew {float(t0.max() - t0.min()):.2f} us")
    prev = torch.zeros(nwg, dtype=torch.float64)
    for i in range(1, 5):
        d = st[:, i] - t0
        print(f"  {NAMES[kind][i]:22s} end @ median {float(d.median()):7.2f} us  max {float(d.max()):7.2f}"
              f"   (phase median {float((d - prev).median()):6.2f})")
        prev = d
    if kind == 1:
        # per input chunk (blockIdx.y; chunk 0 also runs the dW2/db1/db2 wave)
        ny = nwg // 32
        for y in range(ny):
            sl = st[y * 32:(y + 1) * 32]
            ends = [float((sl[:, i] - sl[:, 0]).median()) for i in range(1, 5)]
            mx = float((sl[:, 4] - t0.min()).max())
            print(f"    chunk {y}: phase ends (median) " + " ".join(f"{e:5.2f}" for e in ends) + f"  last end {mx:5.2f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(a.rows, 784, generator=g).to(dev),
              torch.randint(0, 10, (a.rows,), generator=g).to(torch.int32).to(dev))
    st = init_dp(Classifier(), adamw(1e-3), 69, dev)
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    for _ in range(3):
        tr.step(b)
    eng = tr.fused
    L = _lib.lib()
    sa = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
    sb = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
    T = type(eng._args)
    args0, args1 = T(), T()
    ctypes.memmove(ctypes.byref(args0), ctypes.byref(eng._args), ctypes.sizeof(T))
    ctypes.memmove(ctypes.byref(args1), ctypes.byref(eng._args), ctypes.sizeof(T))
    args0.stamps, args1.stamps = sa.data_ptr(), sb.data_ptr()
    s = _lib.stream_ptr()
    for _ in range(a.iters):
        _lib.check(L.jdt_mlp2(ctypes.byref(args0), 0, 784, 10, s), "fwd")
        _lib.check(L.jdt_mlp2(ctypes.byref(args1), 1, 784, 10, s), "bwd")
    torch.cuda.synchronize()
    H = 512
    rb = int(os.environ.get("JDT_MLP2_RB", "16"))
    nf = ((a.rows + rb - 1) // rb) * (H // 16)
    report(0, sa.cpu(), nf)
    report(1, sb.cpu(), (H // 16) * 7)
    # inter-kernel gap: last fwd end -> first bwd start
    fa = sa.cpu()[: nf * 16].view(-1, 16)
    fb = sb.cpu()[: (H // 16) * 7 * 16].view(-1, 16)
    print(f"fwd last end -> bwd first start: {float(fb[:, 0].min() - fa[:, 4].max()) * 10e-3:.2f} us")
    if getattr(eng, "ahead_ok", False):
        # run-ahead backward: same phases plus the next step's forward (slots 8-11)
        eng.run_ahead(b, 1)
        ah = type(eng._ahead_args)()
        ctypes.memmove(ctypes.byref(ah), ctypes.byref(eng._ahead_args), ctypes.sizeof(T))
        sc = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
        ah.stamps = sc.data_ptr()
        for _ in range(a.iters):
            _lib.check(L.jdt_mlp2(ctypes.byref(ah), 2, 784, 10, s), "bwd_ahead")
        torch.cuda.synchronize()
        n = (H // 16) * 7
        report(1, sc.cpu(), n)
        st_ = sc.cpu()[: n * 16].view(n, 16).double() * 10e-3
        t0 = st_[:, 0]
        print("--- run-ahead phases (us from each workgroup's start: median / max over workgroups)")
        for i, nm in ((3, "dW1+AdamW done"), (8, "Z1 partial stored (vmcnt 0)"), (9, "column barrier passed"),
                      (10, "partials + hand-offs loaded"), (11, "epilogue share (G1/H1, H tile)"),
                      (4, "logit atomics issued, end")):
            d = st_[:, i] - t0
            print(f"  {nm:32s} {float(d.median()):6.2f}  max {float(d.max()):6.2f}")
        print(f"  span first start -> last end: {float(st_[:, 4].max() - t0.min()):.2f} us")
        # boundary between two consecutive run-ahead launches (the per-step gap of the graph)
        sd = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
        ah2 = type(eng._ahead_args)()
        ctypes.memmove(ctypes.byref(ah2), ctypes.byref(ah), ctypes.sizeof(T))
        ah2.stamps = sd.data_ptr()
        gaps = []
        for _ in range(a.iters):
            _lib.check(L.jdt_mlp2(ctypes.byref(ah), 2, 784, 10, s), "bwd_ahead")
            _lib.check(L.jdt_mlp2(ctypes.byref(ah2), 2, 784, 10, s), "bwd_ahead")
            torch.cuda.synchronize()
            x = sc.cpu()[: n * 16].view(n, 16).double() * 10e-3
            y = sd.cpu()[: n * 16].view(n, 16).double() * 10e-3
            gaps.append(float(y[:, 0].min() - x[:, 4].max()))
        gaps.sort()
        print(f"  run-ahead launch k last end -> launch k+1 first start: median {gaps[len(gaps) // 2]:.2f} us "
              f"(min {gaps[0]:.2f}, max {gaps[-1]:.2f})")


if __name__ == "__main__":
    main()
