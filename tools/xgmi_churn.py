"""Context churn on the xGMI collectives: build an XgmiComm (start-up self-test), run a
trainer-like burst of collectives, tear it down, repeat -- the life cycle bench.py's
autotune puts a context through a dozen times per process.  Counts self-test failures
per teardown mode:

  quiesce  every rank's queue drained, then a barrier, then free (runtime.dist.quiesce)
  local    this rank's queue drained, then free (no barrier)
  none     free right after the last launch (hipFree's own implicit synchronisation only)

Run under torchrun with JDT_BACKEND=gloo to rehearse several ranks on one GPU:

  torchrun --nproc-per-node 4 --master-addr 127.0.0.1 tools/xgmi_churn.py --iters 12
"""
import argparse
import json
import time

import torch
import torch.distributed as dist

from jax_distributed_tuts_amd.comm import xgmi as X
from jax_distributed_tuts_amd.runtime import dist as D


def burst(c: X.XgmiComm, dev, n_calls: int, rank: int):
    """Back-to-back all-reduces of the trainer bucket size and small ones (no host sync)."""
    big = torch.ones(407_054, device=dev) * (rank + 1)
    small = torch.ones(4_100, device=dev) * (rank + 1)
    for i in range(n_calls):
        c.all_reduce_(big if i % 3 else small)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--modes", default="quiesce,local,none")
    ap.add_argument("--calls", type=int, default=40)
    args = ap.parse_args()
    dev = D.init()
    rank, world = D.rank(), D.world_size()
    X.size_grids_for_sharing(dev)
    timeout = D.spin_timeout_s(30.0)
    out = {}
    for mode in args.modes.split(","):
        fails, t0 = 0, time.perf_counter()
        for it in range(args.iters):
            c = X.XgmiComm(dist.group.WORLD, rank, world, 408_576, dev, timeout_s=timeout)
            fails += int(not c.ok)
            if c.ok:
                burst(c, dev, args.calls, rank)
            if mode == "quiesce":
                D.quiesce(dev)
            elif mode == "local":
                torch.cuda.synchronize(dev)
            c.close()
            if rank == 0:
                print(f"[churn] mode {mode} iter {it}: {'ok' if c.ok else 'FAILED'} (rank 0 failures so far {fails})",
                      flush=True)
            D.barrier()
        out[mode] = {"contexts": args.iters, "selftest_failures": fails,
                     "s": round(time.perf_counter() - t0, 1)}
    t = torch.tensor([v["selftest_failures"] for v in out.values()], dtype=torch.int64)
    dist.all_reduce(t)
    for k, v in zip(out, t.tolist()):
        out[k]["selftest_failures_all_ranks"] = v
    if rank == 0:
        print(json.dumps({"world": world, "results": out}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
