"""Short timed regions: S steps as one hipGraph replay vs S steps launched back to
back from native code (FusedMLP2.run_native -> jdt_mlp2_run) vs a hybrid (a few
native steps first, so the GPU is busy while the graph launch is set up, then an
(S - lead)-step graph).  Headline DP step; wall time of launch + synchronize,
first call and median of the following alternating calls.

    python tools/probe_native_run.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import argparse  # noqa: E402

import bench  # noqa: E402
from jax_distributed_tuts_amd.runtime import dist as D  # noqa: E402


def main():
    dev = D.init()
    ap = argparse.Namespace(num_layers=2, optimizer="adamw", accum="kernel", comm="auto")
    tr, batch, _ = bench.build_dp(ap, dev)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    eng = tr.fused
    for S in (20, 100, 300):
        for lead in (1, 2, 4):
            tr.capture(batch, steps_per_graph=S)
            g_full = tr.multi[1]
            tr.capture(batch, steps_per_graph=S - lead)
            g_part = tr.multi[1]
            runs = {"graph": lambda: g_full.replay(), "native": lambda: eng.run_native(batch, S),
                    "hybrid": lambda: (eng.run_native(batch, lead), g_part.replay())}
            ws = {k: [] for k in runs}
            for it in range(9):
                for k, fn in runs.items():
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    fn()
                    torch.cuda.synchronize()
                    ws[k].append((time.perf_counter() - t0) * 1e6)
            line = f"S={S:4d} lead={lead}:"
            for k, v in ws.items():
                med = sorted(v[1:])[4]
                line += f" | {k} first {v[0]:7.1f} med {med:7.1f} us ({S / med * 1e6:7.0f}/s)"
            print(line, flush=True)


if __name__ == "__main__":
    main()
