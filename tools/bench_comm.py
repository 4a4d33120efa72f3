"""T5: collective latency / bandwidth sweep over RCCL (xGMI) or gloo.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_comm.py
    python tools/bench_comm.py --sim-cpu 4        # gloo plumbing check

Reports, per op and message size (4 KiB .. 64 MiB), the median latency and the
algorithm bandwidth (bytes / time) plus the ring-equivalent bus bandwidth
(2(N-1)/N for all-reduce, (N-1)/N for all-gather / reduce-scatter) -- the
numbers to hold against the 7 x ~153 GB/s xGMI links of an MI355X node when
choosing bucket sizes.

On GPUs it also times this framework's own xGMI kernels on the same sizes
(comm/xgmi.py two-shot all-reduce, reduce-scatter, all-gather; comm/p2p.py
inbox send+recv between neighbours), each as 20 back-to-back launches captured
in one hipGraph -- the "xgmi_*" columns, to compare against RCCL's.  RCCL
columns need the nccl backend (one GPU per rank); with ``JDT_BACKEND=gloo``
(several ranks sharing one GPU, a plumbing rehearsal) only the xGMI kernels run.
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


def _graph_time(fn, reps: int = 20) -> float:
    """Median per-call time (s) of ``fn`` captured ``reps`` times in one hipGraph."""
    fn()
    torch.cuda.synchronize()
    D.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    ts = []
    for _ in range(5):
        D.barrier()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3 / reps)
    ts.sort()
    return ts[2]


def main(args):
    dev = D.device()
    n = D.world_size()
    gpu = dev.type == "cuda"
    rccl = D.backend() == "nccl" or not gpu
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    xg = p2p = None
    if gpu and n > 1:
        from jax_distributed_tuts_amd.comm.p2p import XgmiP2P
        from jax_distributed_tuts_amd.comm.xgmi import XgmiComm

        mesh = D.Mesh({"data": n})
        xg = XgmiComm(mesh.group("data"), D.rank(), n, args.max_bytes // 4 + 4096, dev)
        p2p = XgmiP2P(mesh.group("data"), D.rank(), n, min(args.max_bytes, 8 << 20), 2, dev)
        if not (xg.ok and p2p.ok):
            xg = p2p = None
    out = []
    size = 4096
    while size <= args.max_bytes:
        numel = size // 4
        numel -= numel % (4 * n)
        x = torch.ones(numel, device=dev)
        y = torch.empty(numel * n, device=dev)
        z = torch.empty(numel // n, device=dev)
        res = {"bytes": numel * 4}
        b = numel * 4
        if n > 1 and rccl:
            res["all_reduce_us"] = _time(lambda: dist.all_reduce(x), args.iters, sync) * 1e6
            if gpu:
                res["all_gather_us"] = _time(lambda: dist.all_gather_into_tensor(y, x), args.iters, sync) * 1e6
                res["reduce_scatter_us"] = _time(lambda: dist.reduce_scatter_tensor(z, x), args.iters, sync) * 1e6
            res["all_reduce_busbw_GBs"] = b * 2 * (n - 1) / n / (res["all_reduce_us"] * 1e-6) / 1e9
        if xg is not None:
            part = numel // n
            res["xgmi_all_reduce_us"] = _graph_time(lambda: xg.all_reduce_(x)) * 1e6
            if b <= 256 * 1024:   # one-shot by default at this size: time the two-shot kernel too
                xg.set_oneshot_bytes(0)
                res["xgmi_all_reduce_2shot_us"] = _graph_time(lambda: xg.all_reduce_(x)) * 1e6
                xg.set_oneshot_bytes(256 * 1024)
            res["xgmi_reduce_scatter_us"] = _graph_time(lambda: xg.reduce_scatter(x, z, part)) * 1e6
            res["xgmi_all_gather_us"] = _graph_time(lambda: xg.all_gather(z, x, part)) * 1e6
            res["xgmi_all_reduce_busbw_GBs"] = b * 2 * (n - 1) / n / (res["xgmi_all_reduce_us"] * 1e-6) / 1e9
            if b <= p2p.slot_bytes:
                ep = torch.zeros(1, dtype=torch.int32, device=dev)
                r, to = D.rank(), (D.rank() + 1) % n

                def ring():  # every rank sends to its right neighbour and receives from its left
                    p2p.send(x, to, 0, ep)
                    p2p.recv(y[:numel], 0, ep)
                    ep.add_(1)
                res["xgmi_p2p_sendrecv_us"] = _graph_time(ring) * 1e6
        out.append(res)
        size *= 4
    if xg is not None:
        xg.close()
        p2p.close()
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
