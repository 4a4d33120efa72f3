"""Launchers: a built-in single-node ``torchrun``, or an in-process spawn of N
gloo CPU ranks.

The reference trains on every device with ONE command: it builds
``Mesh(np.array(jax.devices()), ('data',))`` inside a single process
(data_paral.py:150-152, param_sharding.py:249-251).  On MI355X a device is a
process, so the same one-command behaviour is :func:`local_launch`: when an
entry script or ``bench.py`` is asked for N > 1 GPUs and is not already a rank
of a job (no ``WORLD_SIZE`` in the env), it starts N fresh child interpreters
of itself -- BEFORE anything touches the GPU -- with torchrun-style env
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), one GPU
per ``LOCAL_RANK`` and the nccl (= RCCL over xGMI) backend, waits for them and
exits with the first failing child's status.  Children are started with
``subprocess`` (never ``exec``) and stopped by their exact PIDs.

``sim_multiCPU_dev(N)`` (util.py:31-38 in the reference) forced XLA to expose N
host devices and hid the GPUs.  Here the equivalent is N local processes on
the gloo backend: :func:`run` notices ``JDT_SIM_CPU=N`` (or ``--sim-cpu N``)
and spawns them with ``torch.multiprocessing`` (fresh interpreters, so no
GPU state is ever forked), each with RANK/WORLD_SIZE/MASTER_* set and
rendezvous on 127.0.0.1.  Under ``torchrun`` it simply initialises and runs.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
import traceback
from typing import Any, Callable, List, Optional, Sequence

import torch.multiprocessing as mp

from . import dist as D


def free_port() -> int:
    """A free rendezvous port BELOW the kernel's ephemeral range: a port handed out
    by ``bind(0)`` is ephemeral, so between our probe and rank 0's TCPStore bind a
    peer's outgoing (store / gloo pair) socket can be given the same number and the
    bind fails with EADDRINUSE -- an intermittent launch failure."""
    import random

    lo = 20000
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo = min(lo, int(f.read().split()[0]) - 2000)
    except (OSError, ValueError, IndexError):
        pass
    rnd = random.Random(os.getpid() ^ time.time_ns())
    # an ephemeral range starting near 1024 leaves no room below it: plain bind(0)
    for _ in range(64 if lo - 64 > 1024 else 0):
        port = rnd.randrange(max(1024, lo - 10000), lo)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ----------------------------------------------------------------------------- one command, N GPU ranks
def is_launched_rank() -> bool:
    """True inside a process that is already one rank of a job (torchrun, our
    own :func:`local_launch`, or a gloo simulation child)."""
    return "WORLD_SIZE" in os.environ or "RANK" in os.environ


def visible_gpus() -> int:
    """Number of visible GPUs without initialising HIP in this process
    (``torch.cuda.device_count`` only queries the driver)."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 0


def child_env(rank: int, world: int, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port), "JDT_LAUNCHED": "1"})
    return env


def local_launch(nproc: int, argv: Sequence[str], *, env: Optional[dict] = None, poll_s: float = 0.2,
                 grace_s: float = 10.0) -> int:
    """Start ``nproc`` ranks of ``python argv...`` on this node and wait for them.

    Returns 0 when every rank exits 0, else the first failing rank's exit status
    (the other ranks are then stopped: SIGTERM to their exact PIDs, SIGKILL after
    ``grace_s``).  rank r gets LOCAL_RANK=r, i.e. ``cuda:r`` (runtime/dist.py)."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(nproc):
        procs.append(subprocess.Popen([sys.executable, *argv], env=child_env(r, nproc, port, env)))
    status = 0
    try:
        live = list(range(nproc))
        while live:
            for r in list(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.remove(r)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"[launch] rank {r} exited with status {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    _stop(procs, grace_s)
            if live:
                time.sleep(poll_s)
    except KeyboardInterrupt:
        _stop(procs, grace_s)
        raise
    return status


def _stop(procs: List[subprocess.Popen], grace_s: float):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t0 = time.time()
    for p in procs:
        left = max(0.0, grace_s - (time.time() - t0))
        try:
            p.wait(timeout=left)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def maybe_launch(nproc: Optional[int], script: str, argv: Sequence[str]):
    """Entry-script hook: if ``nproc`` > 1 ranks are wanted and this process is not
    already a rank, run :func:`local_launch` of ``script argv`` and exit with its
    status.  Call it before anything initialises the GPU."""
    if nproc is None or nproc <= 1 or is_launched_rank():
        return
    sys.exit(local_launch(int(nproc), [os.path.abspath(script), *argv]))


def check_world(expected: Optional[int]):
    """Fail loudly (exit 3) if this job does not have ``expected`` ranks -- a
    multi-GPU request must never silently measure or train on fewer devices."""
    if expected is None:
        return
    ws = D.world_size()
    if ws != int(expected):
        print(f"[launch] error: {expected} ranks requested but the job has WORLD_SIZE={ws}", file=sys.stderr,
              flush=True)
        D.shutdown()
        sys.exit(3)


def resolve_gpus(requested: Optional[int]) -> int:
    """``--gpus`` of the entry scripts: None = every visible GPU (the reference's
    ``jax.devices()``), at least 1 (CPU-only machines run one rank)."""
    if requested is not None:
        return int(requested)
    if "WORLD_SIZE" in os.environ:
        return int(os.environ["WORLD_SIZE"])
    return max(1, visible_gpus())


# ----------------------------------------------------------------------------- gloo simulation
def _child(local_rank: int, world: int, port: int, fn: Callable, args: tuple, env: dict, gpu: bool = False):
    os.environ.update(env)
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if not gpu:
        os.environ["JDT_SIM_CPU"] = str(world)
        os.environ["HIP_VISIBLE_DEVICES"] = ""
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
    try:
        D.init(backend="gloo")
        fn(*args)
    except Exception as e:  # noqa: BLE001
        from ..utils.metrics import print_exception

        print_exception(e)
        traceback.print_exc()
        raise
    finally:
        D.shutdown()


def spawn(fn: Callable, world: int, *args: Any, env: dict | None = None, gpu: bool = False):
    """Run ``fn(*args)`` on ``world`` gloo ranks (blocking).  With ``gpu=True`` the
    ranks keep the GPUs (rank r on device r % device_count -- on a one-GPU box all
    ranks share cuda:0, which rehearses the multi-process GPU paths such as the
    xGMI IPC collectives; the process group stays gloo since RCCL refuses two
    ranks on one device).  For N RCCL ranks on N GPUs use :func:`local_launch`."""
    for attempt in range(1 if gpu else 2):
        port = free_port()
        try:
            mp.start_processes(_child, args=(world, port, fn, args, dict(env or {}), gpu), nprocs=world,
                               join=True, start_method="spawn")
            return
        except mp.ProcessExitedException as e:
            # CPU simulation only: a rank killed by a signal (not a Python error --
            # those raise ProcessRaisedException) is gloo's rare teardown abort
            # ("terminate called without an active exception"); run the job once more
            if gpu or attempt or e.signal_name is None:
                raise
            print(f"[spawn] rank {e.error_index} died with {e.signal_name}; re-running the {world}-rank job once",
                  file=sys.stderr, flush=True)


def run(fn: Callable, *args: Any, sim_cpu: int | None = None, expect_world: Optional[int] = None):
    """Entry-point runner used by data_paral.py / param_sharding.py / pipeline_parallel.py.
    ``expect_world``: exit non-zero unless the job has exactly that many ranks."""
    if sim_cpu is None and os.environ.get("JDT_SIM_CPU") and "RANK" not in os.environ:
        sim_cpu = int(os.environ["JDT_SIM_CPU"])
    if sim_cpu and "RANK" not in os.environ:
        spawn(fn, int(sim_cpu), *args)
        return
    D.init()
    check_world(expect_world)
    try:
        fn(*args)
    except Exception as e:  # report on the failing rank, then tear down so peers fail fast
        from ..utils.metrics import print_exception

        print_exception(e)
        raise
    finally:
        D.shutdown()
