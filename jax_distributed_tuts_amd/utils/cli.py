"""Command-line plumbing shared by the entry scripts.

``entry_main(main, args, script)`` is the common ``__main__`` of the three entry
scripts: N-rank launch (``--gpus``), optional profiling, then the run.

``--profile [COUNTERS]`` re-runs the same command as a *child* of
``rocprofv3 --pmc COUNTERS --kernel-trace --stats`` (counters only with the
kernel trace; never combined with the runtime/HIP/HSA/marker trace domains) and
exits with its status.  It happens before anything touches the GPU: the
profiler's preloaded library initialises the device itself, so the parent must
not have.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

DEFAULT_COUNTERS = "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"


def add_common_args(ap: argparse.ArgumentParser, steps: int, accum_default: str = "loop",
                    accum_choices=("loop", "scan", "fused", "kernel")):
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPU ranks to train on (default: every visible GPU, like the reference's jax.devices()); "
                         "N > 1 without torchrun starts N local RCCL ranks (runtime/launch.py)")
    ap.add_argument("--sim-cpu", type=int, default=None, help="simulate N devices as gloo CPU ranks")
    ap.add_argument("--check-replication", action="store_true",
                    help="after training, verify that every replicated parameter is bitwise equal on all ranks "
                         "(the debug replacement of the reference's disabled shard_map check_rep)")
    ap.add_argument("--deterministic", action="store_true",
                    help="fixed-order reductions only (no fp32 atomics): bitwise-reproducible runs")
    ap.add_argument("--serialize-kernels", action="store_true",
                    help="debug: HIP_LAUNCH_BLOCKING=1 AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3, set before any GPU "
                         "call (a fault then surfaces at the launch that caused it); slow")
    ap.add_argument("--optimizer", choices=["adamw", "sgd"], default="adamw",
                    help="adamw: the reference's optax.adamw (fused AdamW kernels); sgd: the fused SGD kernel")
    ap.add_argument("--steps", type=int, default=steps)
    ap.add_argument("--num-layers", type=int, default=2)
    ap.add_argument("--accum", choices=list(accum_choices), default=accum_default,
                    help="loop: per-minibatch kernels (reference semantics, util.accum_grads_loop); scan: one "
                         "captured minibatch step replayed per minibatch (util.accum_grads_scan); fused: all rows "
                         "in one pass; kernel: whole-step fused HIP kernels")
    ap.add_argument("--use-scan", action="store_true", help="alias of --accum scan (util.accum_grads use_scan)")
    ap.add_argument("--profile", nargs="?", const=DEFAULT_COUNTERS, default=None, metavar="COUNTERS",
                    help="run under rocprofv3 --pmc (PMC counters + kernel stats)")
    ap.add_argument("--profile-dir", default="gpurun_out/profile")
    return ap


def _strip_profile(argv):
    """argv without --profile [COUNTERS] / --profile-dir DIR (and their = forms)."""
    out, i = [], 0
    while i < len(argv):
        a = argv[i]
        if a == "--profile":
            i += 2 if i + 1 < len(argv) and not argv[i + 1].startswith("-") else 1
        elif a == "--profile-dir":
            i += 2
        elif a.startswith("--profile=") or a.startswith("--profile-dir="):
            i += 1
        else:
            out.append(a)
            i += 1
    return out


def profile_cmd(script: str, argv, counters: str, outdir: str):
    return (["rocprofv3", "--pmc", *counters.split(), "--kernel-trace", "--stats", "--output-format", "csv",
             "-d", os.path.abspath(outdir), "-o", "run", "--", sys.executable, os.path.abspath(script)]
            + _strip_profile(list(argv)))


def maybe_profile(args, script: str):
    """If ``--profile`` was given (and we are not already the profiled child), run
    this script under rocprofv3 as a child process and exit with its code."""
    if not getattr(args, "profile", None) or os.environ.get("JDT_PROFILED") == "1":
        return
    # multi-rank jobs: runtime/launch.py started the ranks first (the launcher never
    # runs under the profiler), and each rank profiles itself into its own directory
    outdir = args.profile_dir if "RANK" not in os.environ else os.path.join(args.profile_dir,
                                                                            f"rank{os.environ['RANK']}")
    cmd = profile_cmd(script, sys.argv[1:], args.profile, outdir)
    os.makedirs(outdir, exist_ok=True)
    env = dict(os.environ, JDT_PROFILED="1", TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    print("[profile] " + " ".join(cmd), file=sys.stderr, flush=True)
    sys.exit(subprocess.call(cmd, env=env))


def make_tx(args, lr: float):
    """The optimizer named by ``--optimizer`` at the config's learning rate."""
    from .train_state import adamw, sgd

    return sgd(lr) if getattr(args, "optimizer", "adamw") == "sgd" else adamw(lr)


def entry_main(main, args, script: str):
    """``__main__`` of an entry script, in the only safe order:

    1. ``--gpus N`` (> 1, not already a rank): start N local ranks of this script
       and exit with their status -- the launcher process never touches the GPU;
    2. ``--profile``: this rank re-runs itself under rocprofv3 as a child;
    3. run ``main(args)`` on the job's process group, failing (exit 3) unless it
       has exactly the requested number of ranks."""
    import faulthandler

    from ..runtime.launch import maybe_launch, resolve_gpus, run

    # a native crash (HIP runtime segfault, abort) prints every thread's Python stack
    faulthandler.enable(all_threads=True)
    if getattr(args, "serialize_kernels", False):
        # read by the HIP runtime at initialisation: set here, before any GPU call,
        # so this process and every rank the launcher starts inherit them
        from .debug import SERIALIZE_ENV

        os.environ.update(SERIALIZE_ENV)
    if args.sim_cpu:
        maybe_profile(args, script)
        run(main, args, sim_cpu=args.sim_cpu)
        return
    n = resolve_gpus(args.gpus)
    maybe_launch(n, script, sys.argv[1:])
    maybe_profile(args, script)
    if args.deterministic:
        # fixed-order reductions: the fused engines' ordered logit sums (no fp32
        # atomics), fixed-order split-K / xGMI reductions.  The generic per-minibatch
        # kernels still reduce bias gradients with fp32 atomics, so the step runs on
        # the fused kernels.
        os.environ["JDT_DETERMINISTIC"] = "1"
        if getattr(args, "accum", None) in ("loop", "scan", "fused"):
            print(f"[deterministic] --accum {args.accum} -> kernel (fused, fixed-order reductions)", file=sys.stderr)
            args.accum = "kernel"
    run(main, args, expect_world=n)
