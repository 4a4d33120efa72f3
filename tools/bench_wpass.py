"""The transformer W pass (every deferred weight-gradient GEMM of a step, models/
transformer.py weight_grads) on the bench LM (4 layers, d 512, d_ff 2048, V 2048, 2048
tokens): per-GEMM launches in order on one stream, round-robin over 4 streams, and ONE
launch (ops.kernels.gemm_wpass) per tile config -- each captured 20x in one hipGraph,
median of 5 replays, random arena data; plus the one-launch result checked against the
per-GEMM one (fp32 gradients, same inputs).

    python tools/bench_wpass.py [--adamw]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.models.transformer import TransformerConfig, TransformerLM, WGradArena  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402
from jax_distributed_tuts_amd.utils.flat import FlatParams  # noqa: E402

REPS = 20


def timed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            fn()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / REPS)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0,1,2,3,4,5")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = TransformerConfig()
    m = TransformerLM(cfg)
    P = FlatParams(m.param_specs(), device=dev).init_(0)
    ar = WGradArena(m, 16, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    for d in list(ar.blocks.values()) + [ar.head]:
        for t in d.values():
            t.copy_(torch.randn(t.shape, generator=g, device=dev).to(torch.bfloat16))
    streams = [torch.cuda.Stream(dev) for _ in range(3)]

    def per_gemm():
        m.weight_grads(P, ar)

    def rr4():
        main_s = torch.cuda.current_stream(dev)
        for s_ in streams:
            s_.wait_stream(main_s)
        allst = [main_s] + streams
        m.weight_grads(P, ar, on=lambda j: torch.cuda.stream(allst[j % 4]))
        for s_ in streams:
            main_s.wait_stream(s_)

    def one(c):
        def f():
            with K.gemm_wpass(cfg=c):
                m.weight_grads(P, ar)
        return f

    P.grad.zero_()
    per_gemm()
    torch.cuda.synchronize()
    ref = P.grad.clone()
    res = {"per-GEMM (1 stream)": timed(per_gemm), "round-robin 4 streams": timed(rr4)}
    flops = sum(2 * h.shape[0] * h.shape[1] * dz.shape[1] for _, h, dz in
                [it for part in ["head"] + list(range(cfg.n_layers)) for it in m.weight_grad_items(ar, part)])
    for c in [int(x) for x in a.cfgs.split(",")]:
        P.grad.zero_()
        one(c)()
        torch.cuda.synchronize()
        err = float((P.grad - ref).norm() / ref.norm())
        res[f"one launch cfg {c} (rel err {err:.1e})"] = timed(one(c))
    for k, v in res.items():
        print(f"{k:45s} {v:8.1f} us  {flops / v / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
