"""Diagnostic: per-tick stamps of the in-kernel GPipe step (ops/csrc/pp_stage.hip).

Runs an MLP pipeline of one 512-wide layer per stage (784 -> 512 x S -> 10 over S
stages, the head on the last) with S ranks, captures the step like bench.py, and has
every rank's stage launch record s_memrealtime (100 MHz) per workgroup: kernel start,
weights staged, the end of each forward tick and of each backward tick, AdamW done.
Every rank prints the median over its 32 workgroups, relative to the FIRST stage's
kernel start (all ranks read the same device clock when they share one GPU), so the
output is the pipeline's fill / drain timeline: tick cost = spacing of consecutive
ticks on the critical path.

    python tools/stamp_pp.py --gpus 4 [--microbatches 4]    (JDT_BACKEND=gloo on one GPU)
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.runtime import dist as D  # noqa: E402
from jax_distributed_tuts_amd.runtime import launch as LCH  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=4)
    ap.add_argument("--microbatches", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    LCH.maybe_launch(args.gpus, __file__, sys.argv[1:])
    dev = D.init()
    LCH.check_world(args.gpus)
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    S = D.world_size()
    cfg = dp_config()
    mesh = D.Mesh({"data": 1, "pipe": S})
    tr = build_mlp_pipeline(cfg, mesh, dev, S, num_microbatches=args.microbatches)
    b = synthetic_batch(cfg, cfg.seed + 1)
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr.step(b)
    eng = tr.pp_kernel
    if eng is None:
        if D.rank() == 0:
            print("stage kernel not engaged (see parallel/pp_kernel.local_ok)")
        D.shutdown()
        return
    stamps = torch.zeros(32 * 32, dtype=torch.int64, device=dev)
    eng.set_stamps(stamps)
    tr.capture(b, steps_per_graph=1)
    # steps, then one stamped step whose timeline is printed
    tr.run_steps(b, args.steps)
    torch.cuda.synchronize()
    D.barrier()
    tr.step(b)
    torch.cuda.synchronize()
    tr.finalize()
    st = stamps.view(32, 32).double()
    n = args.microbatches
    med = lambda k: float(st[:, k].median())   # noqa: E731
    t = torch.tensor([med(0)], dtype=torch.float64)
    allt = [torch.zeros(1, dtype=torch.float64) for _ in range(S)]
    torch.distributed.all_gather(allt, t)
    t0 = min(float(x) for x in allt)
    us = lambda k: (med(k) - t0) / 100.0   # noqa: E731   ticks -> us
    row = {"stage": D.rank(), "start": us(0), "staged": us(1),
           "fwd": [round(us(2 + i), 2) for i in range(min(n, 8))],
           "bwd": [round(us(10 + i), 2) for i in reversed(range(min(n, 8)))], "adam": us(18),   # stage launch end
           # microbatch 1's sub-tick marks: forward inputs there / MFMAs done / epilogue done,
           # backward dZ formed / dW MFMAs done
           "sub": [round(us(k), 2) for k in range(19, 24)],
           # end of the stage launch: partial gradients being stored / stored (the AdamW
           # launch follows)
           "end": [round(us(k), 2) for k in (24, 18)]}
    rows = [None] * S
    torch.distributed.all_gather_object(rows, row)
    if D.rank() == 0:
        print(f"in-kernel GPipe step, {S} stages x 1 layer, {n} microbatches of {128 // n} rows "
              f"(us from the first stage's kernel start; medians over 32 workgroups)")
        for r in rows:
            print(f"  stage {r['stage']}: start {r['start']:7.2f} staged {r['staged']:7.2f} fwd ticks end "
                  + " ".join(f"{x:7.2f}" for x in r["fwd"]) + "  bwd ticks end "
                  + " ".join(f"{x:7.2f}" for x in r["bwd"]) + f"  adam {r['adam']:7.2f}")
            print("    end: partial gradients stored {:7.2f} -> {:7.2f}".format(*r["end"]))
            print(f"    mb1 fwd: inputs {r['sub'][0]:7.2f} mfma {r['sub'][1]:7.2f} epilogue {r['sub'][2]:7.2f} sent "
                  f"{r['fwd'][1] if len(r['fwd']) > 1 else 0:7.2f} | bwd: dZ {r['sub'][3]:7.2f} dW {r['sub'][4]:7.2f}")
        f_last = rows[-1]["fwd"][-1] - rows[0]["fwd"][0]
        ticks_f = n + S - 2
        b_first = rows[0]["bwd"][-1] - rows[-1]["bwd"][0]
        print(f"  forward fill+drain: {f_last:.2f} us over {ticks_f} tick hops -> {f_last / max(1, ticks_f):.2f} us/tick;"
              f" backward: {b_first:.2f} us over {ticks_f} hops -> {b_first / max(1, ticks_f):.2f} us/tick;"
              f" step (first start -> last adam): {max(r['adam'] for r in rows):.2f} us")
    D.shutdown()


if __name__ == "__main__":
    main()
