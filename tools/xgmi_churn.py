"""Context churn on the xGMI collectives: build an XgmiComm (start-up self-test), run a
trainer-like burst of collectives, tear it down, repeat -- the life cycle bench.py's
autotune puts a context through a dozen times per process.  Between contexts every rank
allocates torch tensors (so freed exported pages can be recycled into them) filled with a
canary pattern that is checked after the next context's self-test and burst: a write
through a stale peer mapping shows as a changed canary.  Teardown modes:

  two-phase  every rank closes its peer mappings, a barrier, then every rank releases
             its own buffers (comm/xgmi.py close, the production path)
  quiesce    every rank's queue drained, a barrier, then ONE call that closes this rank's
             mappings and releases its buffers (the round-5 teardown)
  none       the one-call teardown right after the last launch

Run with the exported-buffer pool off to see the teardown alone (JDT_IPC_POOL=0), under
torchrun with JDT_BACKEND=gloo to rehearse several ranks on one GPU:

  JDT_IPC_POOL=0 torchrun --nproc-per-node 4 --master-addr 127.0.0.1 tools/xgmi_churn.py --iters 12
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.comm import xgmi as X  # noqa: E402
from jax_distributed_tuts_amd.runtime import dist as D  # noqa: E402


def burst(c: X.XgmiComm, dev, n_calls: int, rank: int):
    """Back-to-back all-reduces of the trainer bucket size and small ones (no host sync)."""
    big = torch.ones(407_054, device=dev) * (rank + 1)
    small = torch.ones(4_100, device=dev) * (rank + 1)
    for i in range(n_calls):
        c.all_reduce_(big if i % 3 else small)


def canaries(dev, it: int, rank: int):
    """A few tensors of 0.5 .. 8 MB, each filled with its own pattern."""
    out = []
    for k, mb in enumerate((0.5, 1.6, 4.0, 8.0)):
        n = int(mb * (1 << 20)) // 4
        v = float(1000 * it + 10 * k + rank + 1)
        out.append((torch.full((n,), v, device=dev), v))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--modes", default="two-phase,quiesce")
    ap.add_argument("--calls", type=int, default=40)
    args = ap.parse_args()
    dev = D.init()
    rank, world = D.rank(), D.world_size()
    X.size_grids_for_sharing(dev)
    timeout = D.spin_timeout_s(30.0)
    out = {}
    for mode in args.modes.split(","):
        fails = bad_canary = 0
        t0 = time.perf_counter()
        held = []
        for it in range(args.iters):
            c = X.XgmiComm(dist.group.WORLD, rank, world, 408_576, dev, timeout_s=timeout)
            fails += int(not c.ok)
            if c.ok:
                burst(c, dev, args.calls, rank)
            torch.cuda.synchronize(dev)
            for t, v in held:   # allocated before this context: must be untouched
                bad_canary += int(not bool((t == v).all()))
            if mode == "two-phase":
                D.quiesce(dev)
                c.close()
            else:
                if mode == "quiesce":
                    D.quiesce(dev)
                c.close(collective=False)
            # tensors allocated right after the teardown (recycled pages), checked after the
            # next context's self-test and burst
            held = canaries(dev, it, rank)
            if rank == 0:
                print(f"[churn] mode {mode} iter {it}: {'ok' if c.ok else 'FAILED'} (rank 0 self-test failures "
                      f"{fails}, canary failures {bad_canary})", flush=True)
            D.barrier()
        out[mode] = {"contexts": args.iters, "selftest_failures": fails, "canary_failures": bad_canary,
                     "s": round(time.perf_counter() - t0, 1)}
    t = torch.tensor([[v["selftest_failures"], v["canary_failures"]] for v in out.values()], dtype=torch.int64)
    dist.all_reduce(t)
    for k, v in zip(out, t.tolist()):
        out[k]["selftest_failures_all_ranks"], out[k]["canary_failures_all_ranks"] = v
    if rank == 0:
        print(json.dumps({"world": world, "ipc_pool": os.environ.get("JDT_IPC_POOL", "1"), "results": out}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
