"""Launchers: torchrun-style env, or an in-process spawn of N gloo CPU ranks.

``sim_multiCPU_dev(N)`` (util.py:31-38 in the reference) forced XLA to expose N
host devices and hid the GPUs.  Here the equivalent is N local processes on
the gloo backend: :func:`run` notices ``JDT_SIM_CPU=N`` (or ``--sim-cpu N``)
and spawns them with ``torch.multiprocessing`` (fresh interpreters, so no
GPU state is ever forked), each with RANK/WORLD_SIZE/MASTER_* set and
rendezvous on 127.0.0.1.  Under ``torchrun`` it simply initialises and runs.
"""
from __future__ import annotations

import os
import socket
import traceback
from typing import Any, Callable

import torch.multiprocessing as mp

from . import dist as D


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
    ranks on one device)."""
    port = free_port()
    mp.start_processes(_child, args=(world, port, fn, args, dict(env or {}), gpu), nprocs=world, join=True,
                       start_method="spawn")


def run(fn: Callable, *args: Any, sim_cpu: int | None = None):
    """Entry-point runner used by data_paral.py / param_sharding.py / pipeline_parallel.py."""
    if sim_cpu is None and os.environ.get("JDT_SIM_CPU") and "RANK" not in os.environ:
        sim_cpu = int(os.environ["JDT_SIM_CPU"])
    if sim_cpu and "RANK" not in os.environ:
        spawn(fn, int(sim_cpu), *args)
        return
    D.init()
    try:
        fn(*args)
    except Exception as e:  # report on the failing rank, then tear down so peers fail fast
        from ..utils.metrics import print_exception

        print_exception(e)
        raise
    finally:
        D.shutdown()
