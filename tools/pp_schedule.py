"""GPipe schedule table: per-stage compute time against microbatch count on one
MI355X, and the S-stage fill/drain step time it implies.

For every stage of the two BASELINE pipeline layouts -- the 8-stage tutorial MLP
(config #4, 784-512x8-10, global batch 128) and the 4-stage transformer LM
(config #5's pipe axis, 16 sequences / 2 data replicas = 8 per pipe) -- this
builds the stage model exactly as the trainer does (pipeline.mlp_stage /
transformer.lm_stage), captures one step's stage compute (n forwards, then n
backwards with the input gradient when the stage has a predecessor) as a
hipGraph and times its replay, for n = 1, 2, 4, 8, 16 microbatches.  The
forward-only graph is timed too, so each stage gets a forward and a backward
tick cost ``t_f(n)``, ``t_b(n)`` (per microbatch).

GPipe with S stages runs n + S - 1 forward ticks and n + S - 1 backward ticks;
a tick lasts as long as its slowest stage, so the modeled step is

    T(n) = (n + S - 1) * (max_s t_f,s(n) + max_s t_b,s(n) + 2 * hop)

``hop`` is the stage hand-off per tick (xGMI inbox send + receive kernels),
given on the command line (default 0: compute only).  The optimizer, which runs
once per step whatever n is, is left out.  The bubble fraction (S-1)/(n+S-1)
only says how much of the pipe is idle; whether more microbatches shorten the
step depends on how fast t(n) falls with the microbatch's rows -- which is what
this measures.  Reference: /root/reference/pipeline_parallel.py:37-38 (the
GPipe microbatch schedule the tutorial describes).

    python tools/pp_schedule.py [--reps 200] [--hop-us 0] [--out profiles/pp_schedule.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.models.mlp import MLP  # noqa: E402
from jax_distributed_tuts_amd.models.transformer import TransformerConfig, TransformerLM, lm_stage  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402
from jax_distributed_tuts_amd.parallel.fused_stage import FusedMLPStage, stage_supported  # noqa: E402
from jax_distributed_tuts_amd.parallel.pipeline import init_stage_params, mlp_stage  # noqa: E402


def _time_graph(fn, reps: int) -> float:
    """Median-free mean device time (us) of one replay of ``fn`` captured as a graph."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()   # warm: kernel args built, workspaces allocated
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def mlp_stage_costs(S: int, s: int, rows: int, n: int, reps: int, dev):
    dims = [784] + [512] * 8 + [10]
    model = mlp_stage(dims, S, s)
    full = MLP(dims)
    mb = rows // n
    if not stage_supported(model, mb, dev):
        return None
    P = init_stage_params(model, full.param_specs(), 0, dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    eng = FusedMLPStage(model, P, n, mb, step, seed=7)
    first, last = s == 0, s == S - 1
    g = torch.Generator().manual_seed(s)
    xs = [(torch.randn(mb, 784, generator=g) if first else torch.randn(mb, 512, generator=g).bfloat16()).to(dev)
          for _ in range(n)]
    labels = [torch.randint(0, 10, (mb,), generator=g, dtype=torch.int32).to(dev) for _ in range(n)]
    dh = [(torch.randn(mb, 512, generator=g) * 1e-3).bfloat16().to(dev) for _ in range(n)]

    def fwd():
        for i in range(n):
            eng.forward(i, xs[i])

    def both():
        fwd()
        for i in reversed(range(n)):
            if last:
                eng.backward(i, labels=labels[i], need_dx=not first)
            else:
                eng.backward(i, dh=dh[i], need_dx=not first)

    tf = _time_graph(fwd, reps)
    tt = _time_graph(both, reps)
    return tf / n, max(tt - tf, 0.0) / n


def lm_stage_costs(S: int, s: int, seqs: int, n: int, reps: int, dev):
    cfg = TransformerConfig()
    if seqs % n:
        return None
    nseq = seqs // n
    model = lm_stage(cfg, S, s)
    P = init_stage_params(model, TransformerLM(cfg).param_specs(), 0, dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    first, last = s == 0, s == S - 1
    g = torch.Generator().manual_seed(s)
    if first:
        xs = [torch.randint(0, cfg.vocab_size, model.input_shape(nseq), generator=g, dtype=torch.int32).to(dev)
              for _ in range(n)]
    else:
        xs = [torch.randn(model.input_shape(nseq), generator=g).bfloat16().to(dev) for _ in range(n)]
    labels = [torch.randint(0, cfg.vocab_size, (nseq * cfg.seq_len,), generator=g, dtype=torch.int32).to(dev)
              for _ in range(n)]
    dh = [(torch.randn(model.output_shape(nseq), generator=g) * 1e-3).bfloat16().to(dev) for _ in range(n)]
    caches, douts = [None] * n, [None] * n

    def fwd():
        for i in range(n):
            out, caches[i] = model.forward(P, xs[i], train=True, seed=7, offset=i << 16, step=step)
            if last:
                d = torch.empty_like(out)
                K.softmax_xent(out, labels[i], grad_scale=1.0 / labels[i].numel(), dlogits=d,
                               dbias=P.g("head/bias"), metrics=P.metrics_slot)
                douts[i] = d

    def both():
        fwd()
        for i in reversed(range(n)):
            model.backward(P, caches[i], douts[i] if last else dh[i], dout_is_dz=last, need_dx=not first)

    tf = _time_graph(fwd, reps)
    tt = _time_graph(both, reps)
    return tf / n, max(tt - tf, 0.0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--hop-us", type=float, default=0.0, help="stage hand-off cost per tick per direction (us)")
    ap.add_argument("--counts", default="1,2,4,8,16")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    counts = [int(c) for c in args.counts.split(",")]
    layouts = [("mlp_pp8", 8, 128, mlp_stage_costs), ("lm_pp4", 4, 8, lm_stage_costs)]
    report = {"hop_us": args.hop_us, "layouts": {}}
    for name, S, rows, fn in layouts:
        rows_out = []
        for n in counts:
            if rows % n:
                continue
            per = [fn(S, s, rows, n, args.reps, dev) for s in range(S)]
            if any(p is None for p in per):
                continue
            tf = max(p[0] for p in per)
            tb = max(p[1] for p in per)
            ticks = n + S - 1
            step = ticks * (tf + tb + 2 * args.hop_us)
            r = {"n_mb": n, "rows_per_mb": rows // n, "tick_fwd_us": round(tf, 2), "tick_bwd_us": round(tb, 2),
                 "per_stage_fwd_us": [round(p[0], 2) for p in per], "per_stage_bwd_us": [round(p[1], 2) for p in per],
                 "ticks": ticks, "bubble": round((S - 1) / ticks, 3), "modeled_step_us": round(step, 1),
                 "one_gpu_stage_compute_us": [round(n * (p[0] + p[1]), 1) for p in per]}
            rows_out.append(r)
            print(json.dumps({"layout": name, **{k: v for k, v in r.items() if not k.startswith("per_stage")}}),
                  flush=True)
        best = min(rows_out, key=lambda r: r["modeled_step_us"]) if rows_out else None
        report["layouts"][name] = {"stages": S, "rows": rows, "table": rows_out,
                                   "best_n_mb": best["n_mb"] if best else None}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(report, f, indent=1)
    print(json.dumps({k: v["best_n_mb"] for k, v in report["layouts"].items()}))


if __name__ == "__main__":
    main()
