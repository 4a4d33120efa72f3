"""Grid barrier vs kernel boundary on this GPU (tools/barrier_lab/barrier_lab.hip, a lab
kernel built into its own library here, not into the production kernel library).

The headline step is one run-ahead launch per step; a persistent n-step launch would
replace each launch boundary with a grid barrier.  This times, at the headline grid
(224 workgroups of 512 threads, all resident):
  * a flat counter barrier (mlp2_loop_kernel's) and an XCD-hierarchical one, per barrier,
    from one launch of 1024 barriers minus the same loop without barriers;
  * the dependent-kernel boundary: 1024 trivial 224-workgroup kernels back to back in one
    hipGraph, per kernel.

    python tools/barrier_lab.py [--grid 224] [--iters 1024]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
from ctypes import c_int, c_longlong, c_void_p

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402

LAB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "barrier_lab")


def lab_lib():
    """Build (hipcc, gfx950) and load tools/barrier_lab/libbarrier_lab.so."""
    import subprocess

    src, so = os.path.join(LAB, "barrier_lab.hip"), os.path.join(LAB, "libbarrier_lab.so")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        inc = os.path.join(os.path.dirname(LAB), "..", "jax_distributed_tuts_amd", "ops", "csrc")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        f"-I{inc}", src, "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.jdt_barrier_lab.restype, L.jdt_barrier_lab.argtypes = c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                                                    c_void_p, c_longlong, c_void_p]
    L.jdt_boundary_lab.restype, L.jdt_boundary_lab.argtypes = c_int, [c_int, c_void_p, c_void_p]
    return L


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=224)
    ap.add_argument("--iters", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    _lib.lib()
    L = lab_lib()
    ctr = torch.zeros(16 * 32, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    sink = torch.zeros(1024, device=dev)
    stamps = torch.zeros(a.iters // 64 + 2, dtype=torch.int64, device=dev)
    res = {}
    for kind, name in ((2, "loop only"), (0, "flat counter"), (1, "XCD-hierarchical")):
        def run():
            ctr.zero_()
            _lib.check(L.jdt_barrier_lab(kind, a.grid, a.iters, c_void_p(ctr.data_ptr()), c_void_p(err.data_ptr()),
                                         c_void_p(sink.data_ptr()), c_void_p(stamps.data_ptr()), 200_000_000,
                                         c_void_p(_lib.stream_ptr())), "barrier_lab")
        run()
        torch.cuda.synchronize()
        res[name] = timed(run)
        if int(err.item()):
            print(f"{name}: a barrier timed out (not every workgroup resident?)")
            return
        st = stamps.cpu().double()
        per = (st[1:a.iters // 64 + 1] - st[0:a.iters // 64]) / 64 / 100.0   # us per barrier, in-kernel
        print(f"{name:18s}: launch {res[name]:9.1f} us for {a.iters} iterations; in-kernel (wg 0) per 64 "
              f"barriers median {float(per.median()) if kind != 2 else 0.0:.3f} us/barrier")
    loop = res["loop only"]
    for name in ("flat counter", "XCD-hierarchical"):
        print(f"  {name:18s} per barrier: {(res[name] - loop) / a.iters:.3f} us")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        _lib.check(L.jdt_boundary_lab(a.grid, c_void_p(sink.data_ptr()), c_void_p(_lib.stream_ptr())), "warm")
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(a.iters):
            _lib.check(L.jdt_boundary_lab(a.grid, c_void_p(sink.data_ptr()), c_void_p(_lib.stream_ptr())), "boundary")
    g.replay()
    torch.cuda.synchronize()
    tb = timed(g.replay)
    print(f"  kernel boundary (graph of {a.iters} trivial {a.grid}-workgroup kernels): {tb / a.iters:.3f} us per kernel")


if __name__ == "__main__":
    main()
