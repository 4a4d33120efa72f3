"""T5: collective latency / bandwidth sweep over RCCL (xGMI) or gloo.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_comm.py
    python tools/bench_comm.py --sim-cpu 4        # gloo plumbing check

Reports, per op and message size (4 KiB .. 64 MiB), the median latency and the
algorithm bandwidth (bytes / time) plus the ring-equivalent bus bandwidth
(2(N-1)/N for all-reduce, (N-1)/N for all-gather / reduce-scatter) -- the
numbers to hold against the 7 x ~153 GB/s xGMI links of an MI355X node when
choosing bucket sizes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jax_distributed_tuts_amd.runtime import dist as D  # noqa: E402
from jax_distributed_tuts_amd.runtime.launch import run  # noqa: E402


def _time(fn, iters, sync):
    for _ in range(3):
        fn()
    sync()
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        sync()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2]


def main(args):
    dev = D.device()
    n = D.world_size()
    gpu = dev.type == "cuda"
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    out = []
    size = 4096
    while size <= args.max_bytes:
        numel = size // 4
        numel -= numel % n
        x = torch.ones(numel, device=dev)
        y = torch.empty(numel * n, device=dev)
        z = torch.empty(numel // n, device=dev)
        res = {"bytes": numel * 4}
        if n > 1:
            res["all_reduce_us"] = _time(lambda: dist.all_reduce(x), args.iters, sync) * 1e6
            if gpu:
                res["all_gather_us"] = _time(lambda: dist.all_gather_into_tensor(y, x), args.iters, sync) * 1e6
                res["reduce_scatter_us"] = _time(lambda: dist.reduce_scatter_tensor(z, x), args.iters, sync) * 1e6
            b = numel * 4
            res["all_reduce_busbw_GBs"] = b * 2 * (n - 1) / n / (res["all_reduce_us"] * 1e-6) / 1e9
        out.append(res)
        size *= 4
    if D.rank() == 0:
        for r in out:
            print(json.dumps({"n": n, "backend": D.backend(), **{k: round(v, 2) for k, v in r.items()}}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--sim-cpu", type=int, default=None)
    ap.add_argument("--max-bytes", type=int, default=64 << 20)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    run(main, a, sim_cpu=a.sim_cpu)
