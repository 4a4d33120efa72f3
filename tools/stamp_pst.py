"""Diagnostic: phase stamps (s_memrealtime, 100 MHz) of the persistent run-ahead launch
(csrc/mlp_fused.hip mlp2_pst_kernel).  One n-step launch with stamps on; per workgroup the
phase ends of step n-2 (the body's STAMP points; the last step also stores the optimizer
state), the step time (start of n-2 -> start of n-1) and the grid barrier between them
(slots 12 -> 13).  Medians over the 224
workgroups, microseconds.

    python tools/stamp_pst.py [--steps 20] [--rows 128]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.models.mlp import Classifier  # noqa: E402
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp  # noqa: E402
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw  # noqa: E402

PHASES = [(1, "CE -> dlogits (loads landed)"), (2, "dZ1"), (15, "  wave 0: dW1 tile MFMA"),
          (14, "  wave 0: AdamW + W1' tile"), (3, "dW1 MFMA + AdamW + hand-offs"),
          (8, "next Z1 partials stored"), (9, "column barrier passed"), (10, "partials loaded"),
          (11, "forward epilogue (G1 / H1)"), (4, "logit atomics issued")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rows", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(args.rows, 784, generator=g).to(dev),
              torch.randint(0, 10, (args.rows,), generator=g).to(torch.int32).to(dev))
    st = init_dp(Classifier(), adamw(1e-3), 69, dev)
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    tr.step(b)
    eng = tr.fused
    assert eng.pst_ok, "persistent run-ahead unavailable here"
    eng.run_ahead(b, args.steps)                         # warm
    stamps = torch.zeros(224 * 16, dtype=torch.int64, device=dev)
    eng._ahead_args.stamps = stamps.data_ptr()
    for rep in range(args.reps):
        stamps.zero_()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        eng.run_ahead(b, args.steps, prologue=False)
        ev1.record()
        torch.cuda.synchronize()
        s = stamps.view(224, 16).double() * 1e-2       # us
        t0 = s[:, 0]
        step = float((s[:, 7] - s[:, 0]).median())
        bar = float((s[:, 13] - s[:, 12]).median())
        print(f"rep {rep}: launch {ev0.elapsed_time(ev1) * 1e3 / args.steps:.2f} us/step (events) | "
              f"step n-2 start -> n-1 start: median {step:.2f} us | last grid barrier (n-2 -> n-1): median {bar:.2f} us, "
              f"max {float((s[:, 13] - s[:, 12]).max()):.2f}")
        if rep == args.reps - 1:
            prev = torch.zeros_like(t0)
            for k, name in PHASES:
                d = s[:, k] - t0
                print(f"    {name:32s} end @ median {float(d.median()):6.2f} us  max {float(d.max()):6.2f}"
                      f"   (phase median {float((d - prev).median()):5.2f})")
                prev = d
            print(f"    start skew of step n-2 {float(t0.max() - t0.min()):.2f} us; "
                  f"first start -> last end {float(s[:, 4].max() - t0.min()):.2f} us")
            tile = stamps.view(224, 16)[:, 6].cpu()
            by = (tile // 256).double()
            print("    per input chunk (chunk 0 runs the dW2 / db1 / db2 wave; block (0,0) the CE metrics):")
            for y in range(int(by.max()) + 1):
                sel = (by == y).to(s.device)
                ends = [float((s[sel, k] - t0[sel]).median()) for k, _ in PHASES]
                extra = ""
                if y == 0:
                    extra = f"   aux wave done {float((s[sel, 5] - t0[sel]).median()):5.2f}"
                print(f"      chunk {y}: " + " ".join(f"{e:5.2f}" for e in ends) + extra)
            ends = (s[:, 4] - s[:, 0].min()).cpu()
            order = torch.argsort(ends, descending=True)[:12]
            print("    slowest workgroups (end of step n-2 rel. earliest start): " + ", ".join(
                f"wg {int(i)} tile (bx {int(tile[i]) % 256}, by {int(tile[i]) // 256}) {float(ends[i]):.2f}" for i in order))
            bxv = (tile % 256).to(s.device)
            for label, sel in (("column block 0", bxv == 0), ("lead (0,0)", (tile == 0).to(s.device)),
                               ("other blocks", bxv != 0)):
                e = [float((s[sel, k] - t0[sel]).median()) for k, _ in PHASES]
                print(f"    {label:15s}: " + " ".join(f"{x:5.2f}" for x in e) +
                      f"   start rel. earliest {float((t0[sel] - t0.min()).median()):5.2f}")
            stt = (s[:, 0] - s[:, 0].min()).cpu()
            late = torch.argsort(stt, descending=True)[:6]
            print("    latest starters: " + ", ".join(f"wg {int(i)} +{float(stt[i]):.2f}" for i in late))
            xcd = torch.arange(224) % 8
            for x in range(8):
                sel = (xcd == x).to(s.device)
                print(f"      dispatch XCD {x}: phase-3 end median {float((s[sel, 3] - t0[sel]).median()):5.2f}, "
                      f"last-step start (rel. earliest) median {float((t0[sel] - t0.min()).median()):5.2f}")
    eng._ahead_args.stamps = None
    tr.finalize()


if __name__ == "__main__":
    main()
