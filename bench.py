"""Headline benchmark: steps/sec (whole node) of the tutorial MLP training step.

Metric and config come from BASELINE.json / BASELINE.md: the reference's
data-parallel tutorial step (data_paral.py) -- Classifier 784 -> 512 (SiLU,
dropout 0.1) -> 10, bf16 compute / fp32 params, global batch 128 split over the
GPUs (P('data')), 4 gradient-accumulation minibatches per step, AdamW(1e-3),
one gradient+metrics all-reduce per step.  Global batch is fixed as N grows
(the reference's config), so scaling is "strong".  Synthetic data (N(0,1)
inputs, uniform integer labels), random init -- no datasets are available.

Every timed step is a complete training step: all 4 minibatch fwd/bwd passes,
the RCCL all-reduce (N > 1), the fused AdamW update and the metrics fold.

    python bench.py                                # N=1
    python bench.py --gpus 8                       # 8 local ranks, one per GPU (built-in launcher)
    torchrun --nproc-per-node 8 bench.py --gpus 8  # the same job under torchrun
    python bench.py --strategy fsdp|pp             # the other two tutorials

``--gpus N`` is enforced: without torchrun the script starts N ranks itself
(runtime/launch.py, before any GPU call); under a launcher it exits non-zero
unless WORLD_SIZE == N.  ``JDT_BACKEND=gloo`` makes the ranks' process group
gloo (several ranks sharing one GPU -- RCCL refuses that -- while the xGMI
kernels still run between them).
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import time

import torch

from jax_distributed_tuts_amd.runtime import dist as D
from jax_distributed_tuts_amd.runtime import launch as LCH
from jax_distributed_tuts_amd.runtime.dist import Mesh

METRIC = "steps/sec (whole node) for tutorial MLP at 1/2/4/8 MI355X, DP vs shard vs PP"


def build_dp(args, dev):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw, sgd

    cfg = dp_config()
    cfg.model.num_layers = args.num_layers
    mesh = Mesh({"data": D.world_size()})
    model = Classifier.from_config(cfg.model)
    eps = getattr(args, "adam_eps", None)   # autotune's validation probes: AdamW(eps = 10)
    tx = (adamw(cfg.optimizer.learning_rate, **({"eps": eps} if eps else {})) if args.optimizer == "adamw"
          else sgd(cfg.optimizer.learning_rate))
    state = init_dp(model, tx, cfg.seed, dev, mesh)
    batch = shard_batch(synthetic_batch(cfg, cfg.seed + 1), mesh, "data")
    batch = Batch(batch.inputs.to(dev), batch.labels.to(dev))
    tr = DataParallelTrainer(state, mesh, DPConfig(cfg.optimizer.num_minibatches, args.accum, comm=args.comm))
    desc = {"model": f"tutorial MLP {'-'.join(map(str, model.dims))} (SiLU, dropout 0.1)",
            "global_batch": cfg.data.batch_size, "seq_len": None, "num_minibatches": cfg.optimizer.num_minibatches,
            "parallelism": f"dp{D.world_size()}", "accum": args.accum, "optimizer": args.optimizer}
    return tr, batch, desc


def build_fsdp(args, dev):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.config import fsdp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    cfg = fsdp_config()
    cfg.model.num_layers = args.num_layers
    mesh = Mesh({"data": D.world_size()})
    model = Classifier.from_config(cfg.model)
    eps = getattr(args, "adam_eps", None)   # autotune's validation probes: AdamW(eps = 10)
    st = init_fsdp(model, adamw(cfg.model.lr, **({"eps": eps} if eps else {})), cfg.seed, dev, mesh, "data",
                   cfg.model.min_weight_size)
    batch = shard_batch(synthetic_batch(cfg, cfg.seed + 1), mesh, "data")
    batch = Batch(batch.inputs.to(dev), batch.labels.to(dev))
    once = args.accum != "loop"
    tr = FSDPTrainer(st, mesh, FSDPConfig(cfg.num_minibatches, cfg.model.min_weight_size, "data", gather_once=once,
                                          scatter_once=once, fused_kernels=args.accum == "kernel"))
    desc = {"model": f"tutorial MLP {'-'.join(map(str, model.dims))} (SiLU, dropout 0.1)",
            "global_batch": cfg.data.batch_size, "seq_len": None, "num_minibatches": cfg.num_minibatches,
            "parallelism": f"fsdp{D.world_size()}", "gather_once": once}
    return tr, batch, desc


def build_pp(args, dev):
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    cfg = dp_config()
    ws = D.world_size()
    dp = args.dp
    # autotune's validation probes: AdamW(eps = 10), and no dropout -- a different
    # microbatch count draws a different dropout stream, so only the probe without it
    # compares schedules value for value (utils/autotune.py)
    eps = getattr(args, "adam_eps", None)
    probe = eps is not None
    mesh = Mesh({"data": dp, "pipe": ws // dp})
    if args.microbatches is None:
        from jax_distributed_tuts_amd.parallel.pipeline import default_microbatches

        args.microbatches = default_microbatches(ws // dp)
    if args.model == "transformer":
        from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch

        tr, lm_cfg = build_lm_pipeline(mesh, dev, num_microbatches=args.microbatches, comm=args.comm,
                                       merge_single_stage=args.merge_microbatches,
                                       layer_major_single_stage=not args.microbatch_passes,
                                       tx=adamw(3e-4, eps=eps) if probe else None)
        batch = shard_batch(lm_batch(lm_cfg, global_batch=args.lm_batch, seed=1), mesh, "data")
        desc = {"model": f"transformer LM {lm_cfg.n_layers}L d{lm_cfg.d_model} h{lm_cfg.n_heads} "
                         f"ff{lm_cfg.d_ff} V{lm_cfg.vocab_size}", "global_batch": args.lm_batch,
                "seq_len": lm_cfg.seq_len, "tokens_per_step": args.lm_batch * lm_cfg.seq_len}
    else:
        tr = build_mlp_pipeline(cfg, mesh, dev, args.hidden_layers, num_microbatches=args.microbatches,
                                comm=args.comm, merge_single_stage=args.merge_microbatches,
                                dropout_rate=0.0 if probe else None,
                                tx=adamw(cfg.optimizer.learning_rate, eps=eps) if probe else None)
        batch = shard_batch(synthetic_batch(cfg, cfg.seed + 1), mesh, "data")
        desc = {"model": f"MLP 784-512x{args.hidden_layers}-10 GPipe", "global_batch": cfg.data.batch_size,
                "seq_len": None}
    desc.update({"num_microbatches": args.microbatches, "parallelism": f"dp{dp}xpp{ws // dp}",
                 "merged_single_stage": bool(args.merge_microbatches and ws // dp == 1)})
    batch = Batch(batch.inputs.to(dev), batch.labels.to(dev))
    return tr, batch, desc


def comm_sweep(tr, dev, iters: int = 20):
    """T5 evidence from the job itself (N > 1, GPU, untimed, after the measured
    region): median per-call device time of this trainer's gradient all-reduce
    transports on the same data -- the xGMI two-shot kernel (comm/xgmi.py) and
    RCCL's all-reduce (nccl process group only) -- at 64 KiB, the DP bucket size
    and (RCCL) 16 MiB.  Every rank runs the same sequence."""
    import torch.distributed as dist

    xg = getattr(tr, "xg", None)
    rccl = D.backend() == "nccl"
    if not (xg is not None or rccl):
        return None
    bucket = int(tr.state.params.grad.numel())
    out = []
    for n in (16_384, bucket, 4 << 20):
        x = torch.ones(n, device=dev)
        row = {"bytes": n * 4}

        def timed(fn):
            fn()
            torch.cuda.synchronize()
            D.barrier()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(iters):
                fn()
            b.record()
            b.synchronize()
            return round(a.elapsed_time(b) * 1e3 / iters, 2)

        if xg is not None and xg.fits(n)["twoshot"]:
            row["xgmi_us"] = timed(lambda: xg.all_reduce_(x))
        if rccl:
            row["rccl_us"] = timed(lambda: dist.all_reduce(x))
        out.append(row)
    if xg is not None and xg.error():
        raise RuntimeError("xgmi all-reduce timed out during the comm sweep")
    return out


def _comm_choice():
    """The per-size transport calibration of this rank's xGMI context (comm/xgmi.py
    ``calibrate``): one-shot threshold, RCCL availability, per-size timings and choice."""
    try:
        from jax_distributed_tuts_amd.comm import xgmi
    except Exception:
        return None
    return xgmi.LAST_CALIBRATION


def comm_check(tr, where: str):
    """Raise (naming the phase of the run) if an in-kernel xGMI wait of this rank timed
    out so far -- the collective, the FSDP context or a pipeline inbox (synchronises)."""
    for xg in (getattr(tr, "xg", None), getattr(getattr(tr, "sp", None), "xg", None)):
        if xg is not None:
            try:
                xg.raise_if_error()
            except RuntimeError as e:
                raise RuntimeError(f"[{where}] {e}") from None
    p2p = getattr(tr, "p2p", None)
    if p2p is not None and p2p.error():
        raise RuntimeError(f"[{where}] xgmi pipeline receive timed out on this rank")


def one_launch_failed(tr, dev) -> bool:
    """True on EVERY rank when the one-launch N > 1 step (parallel/dp.py, fsdp.py
    one_launch: the run-ahead backward's in-kernel tile exchange) reported an error on
    any rank during the eager steps (synchronises; all ranks call it)."""
    eng = getattr(tr, "fused", None)
    tx = getattr(eng, "tx", None)
    bad = 0
    if tx is not None:
        zt = getattr(eng, "ztick", None)
        bad = int(tx.error() != 0 or (zt is not None and int(zt[1].item()) != 0))
        # rehearsal hook (tests/test_bench_fallback_gpu.py): this rank reports a failure
        bad |= int(os.environ.get("JDT_BENCH_FAKE_TX_ERROR", "-1") == str(D.rank()))
    t = torch.tensor([bad], dtype=torch.int32, device=dev if D.backend() == "nccl" else "cpu")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return bool(t.item())


def autotune_candidates(args, ws: int):
    """[stage candidate lists] for this job (utils/autotune.py).  DP / FSDP: the step forms
    that only engage with one rank per GPU (or that the shared-GPU rehearsals could not
    rank) against the plain collective form, validated; PP: GPipe microbatch count, then
    concurrent stage streams, then the overlapped data-axis sync, timed one stage after
    the other (coordinate descent)."""
    from jax_distributed_tuts_amd.utils.autotune import Candidate

    one = lambda tr: bool(getattr(tr, "one_launch", False))   # noqa: E731
    if args.strategy == "dp" and args.accum == "kernel":
        if args.num_layers == 2:
            # persistent: a replay's steps are ONE launch per rank, the tile exchange inside
            # every step (mlp2_pst_kernel TX); one-launch: one run-ahead launch per step
            pst = lambda tr: one(tr) and bool(getattr(getattr(tr, "fused", None), "pst_ok", False))  # noqa: E731
            return [[Candidate("persistent", {"JDT_DP_AHEAD": "1", "JDT_DP_PST": "1"}, replicated=True, engaged=pst),
                     Candidate("one-launch", {"JDT_DP_AHEAD": "1", "JDT_DP_PST": "0"}, replicated=True, engaged=one),
                     Candidate("three-launch", {"JDT_DP_AHEAD": "0"}, reference=True, replicated=True)]]
        if args.optimizer == "adamw":
            return [[Candidate("deep-exchange", {"JDT_DP_DEEP_TX": "1"}, replicated=True, engaged=one),
                     Candidate("collective", {"JDT_DP_DEEP_TX": "0"}, reference=True, replicated=True)]]
        return []
    if args.strategy == "fsdp" and args.accum == "kernel":
        if args.num_layers == 2:
            pst = lambda tr: one(tr) and bool(getattr(getattr(tr, "fused", None), "pst_ok", False))  # noqa: E731
            return [[Candidate("persistent", {"JDT_FSDP_AHEAD": "1", "JDT_FSDP_PST": "1"}, engaged=pst),
                     Candidate("one-launch", {"JDT_FSDP_AHEAD": "1", "JDT_FSDP_PST": "0"}, engaged=one),
                     Candidate("three-launch", {"JDT_FSDP_AHEAD": "0"}, reference=True)]]
        if args.optimizer == "adamw":
            # deep: one backward launch per hidden layer sending its partials to the shard
            # owners (sharded AdamW in-kernel, csrc/mlp_deep.hip md_bwd FX) vs the step
            # collective (xg_fsdp_kernel)
            return [[Candidate("deep-exchange", {"JDT_FSDP_DEEP_FX": "1"}, engaged=one),
                     Candidate("collective", {"JDT_FSDP_DEEP_FX": "0"}, reference=True)]]
        return []
    if args.strategy == "pp":
        S = ws // args.dp
        # data-axis replicas of a stage: bit-identical (hybrid DP x PP)
        rep = dict(replicated=args.dp > 1, group_of=lambda tr: tr.mesh.group("data"))
        stages = []
        if args.microbatches is None and S > 1:
            rows = (args.lm_batch if args.model == "transformer" else 128) // args.dp
            ns = [n for n in (2, 4, 8) if rows % n == 0 and (args.model == "transformer" or rows // n >= 4)]
            stages.append([Candidate(f"microbatches={n}", {}, reference=(n == 2), args={"microbatches": n}, **rep)
                           for n in ns])
        if S > 1 and args.model == "mlp" and args.dp == 1:
            # one persistent launch per stage step (parallel/pp_kernel.py) vs per-tick launches
            stages.append([Candidate("stage-kernel=1", {"JDT_PP_KERNEL": "1"},
                                     engaged=lambda tr: getattr(tr, "pp_kernel", None) is not None),
                           Candidate("stage-kernel=0", {"JDT_PP_KERNEL": "0"}, reference=True)])
        from jax_distributed_tuts_amd.runtime.dist import ranks_per_gpu

        own_gpu = ranks_per_gpu() == 1
        if S > 1 and args.dp > 1 and own_gpu:
            stages.append([Candidate("overlap-sync=0", {"JDT_PP_OVERLAP_SYNC": "0"}, reference=True, **rep),
                           Candidate("overlap-sync=1", {"JDT_PP_OVERLAP_SYNC": "1"}, **rep)])
        # schedules on concurrent streams: only with a GPU per rank, and LAST (stage and
        # candidate): a process that once opened extra hardware queues keeps them, and on a
        # time-shared GPU every later build then ran 20-50x slower (round 5: GPipe-8 1.9 ->
        # 90 ms/step after a stage-streams candidate was built) -- the autotune re-times the
        # reference after it and records "contaminated"
        if S > 1 and own_gpu:
            stages.append([Candidate("stage-streams=0", {"JDT_PP_STREAMS": "0"}, reference=True, **rep),
                           Candidate("stage-streams=1", {"JDT_PP_STREAMS": "1"}, contaminates=True, **rep)])
        return [st for st in stages if len(st) > 1]
    return []


def run_autotune(args, dev, build, prepare):
    """(trainer, batch, desc, report) of the fastest valid step form, or (None, None,
    None, report) when there is nothing to choose (the caller builds as usual)."""
    import copy

    from jax_distributed_tuts_amd.utils import autotune as AT

    stages = autotune_candidates(args, D.world_size())
    if not stages:
        return None, None, None, {"candidates": [], "choice": "default", "reason": "a single step form"}
    spg = args.steps_per_graph
    steps = spg * max(1, -(-100 // spg))   # whole multi-step graphs, >= 100 steps per timing
    log = (lambda m: print(m, file=sys.stderr, flush=True)) if D.rank() == 0 else (lambda m: None)
    chosen_env, chosen_args, tables = {}, {}, []
    tr = batch = None
    for k, cands in enumerate(stages):
        for c in cands:   # earlier stages' choices carry over
            c.env = {**chosen_env, **c.env}
            c.args = {**chosen_args, **c.args}

        def build_one(eps, c):
            a = copy.copy(args)
            a.__dict__.update(c.args)
            a.adam_eps = eps
            t, b, d = build(a, dev)
            t.bench_desc = d
            return t, b

        # every candidate is value-checked against its stage's reference form (PP too: the
        # stage kernel, microbatch counts and stream schedules against per-tick launches)
        rep, t, b = AT.run(cands, build_one, prepare, dev, validate=True, steps=steps, log=log,
                           prepare_probe=lambda tr_, b_: prepare(tr_, b_, spg=AT.VALIDATE_STEPS - 1))
        tables.append(rep)
        chosen_env.update(rep["env"])
        chosen_args.update(rep.get("args", {}))
        if k < len(stages) - 1 and t is not None:
            t.close()
        else:
            tr, batch = t, b
    os.environ.update(chosen_env)
    args.__dict__.update(chosen_args)
    report = {"stages": tables, "env": chosen_env, "args": chosen_args}
    desc = getattr(tr, "bench_desc", None) if tr is not None else None
    if desc is not None:
        bad = [r for t_ in tables for r in t_["candidates"] if r.get("valid") is False]
        if bad and args.strategy in ("dp", "fsdp"):
            desc["one_launch_fallback"] = "; ".join(f"{r['name']}: {r.get('reason')}" for r in bad)
        if bad and args.strategy == "pp":
            desc["pp_rejected"] = "; ".join(f"{r['name']}: {r.get('reason')}" for r in bad)
    return tr, batch, desc, report


def _mlp2_launches(eng, tx_: str, spg: int) -> str:
    """Launches per step of the fused 2-layer engine's captured replay: the persistent
    run-ahead kernel runs a whole replay of ``spg`` steps in one launch (ops/csrc/mlp_fused.hip
    mlp2_pst_kernel; at N > 1 with the tile exchange inside), else one run-ahead launch per step."""
    if getattr(eng, "pst_ok", False) and spg >= 2:
        return f"1/{spg} (persistent run-ahead: {spg} steps per launch, grid barrier between steps{tx_})"
    return f"1 (run-ahead mlp2_bwd{tx_})"


def pick_steps_per_graph(steps: int, cap: int) -> int:
    """Steps per captured graph: all of them when steps <= cap (one replay, one host
    launch for the whole timed region), else the largest divisor of steps <= cap
    (so no single-step remainder replays)."""
    if steps <= cap:
        return max(1, steps)
    for d in range(cap, 0, -1):
        if steps % d == 0:
            return d
    return 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--strategy", choices=["dp", "fsdp", "pp"], default="dp")
    ap.add_argument("--dp", type=int, default=1, help="data-parallel degree for --strategy pp (hybrid)")
    ap.add_argument("--model", choices=["mlp", "transformer"], default="mlp")
    ap.add_argument("--microbatches", type=int, default=None,
                    help="GPipe microbatches (default: pipeline.default_microbatches, measured per stage count)")
    ap.add_argument("--merge-microbatches", action="store_true",
                    help="--strategy pp with a single stage: run the microbatches as one pass (PipeConfig.merge_single_stage)")
    ap.add_argument("--microbatch-passes", action="store_true",
                    help="--strategy pp --model transformer with a single stage: one forward/backward pass per "
                         "microbatch, as a stage of a real multi-stage pipeline runs (on one GPU the LM's "
                         "microbatch passes already run by default, on concurrent streams: JDT_MB_STREAMS; "
                         "this flag only matters with JDT_MB_STREAMS=1, where the default is layer-major)")
    ap.add_argument("--hidden-layers", type=int, default=8)
    ap.add_argument("--lm-batch", type=int, default=16)
    ap.add_argument("--num-layers", type=int, default=2)
    ap.add_argument("--accum", choices=["loop", "scan", "fused", "kernel"], default="kernel")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--capture-collectives", action="store_true")
    ap.add_argument("--comm", choices=["auto", "xgmi", "rccl"], default="auto",
                    help="N>1 DP gradient collective: direct xGMI P2P kernel (fused with AdamW) or RCCL")
    ap.add_argument("--steps-per-graph", type=int, default=None,
                    help="complete training steps recorded per hipGraph (amortises the replay launch); default: "
                         "all timed steps in one graph when --steps <= 200 (DP), else the largest divisor <= the cap")
    ap.add_argument("--no-comm-sweep", action="store_true",
                    help="skip the untimed RCCL-vs-xGMI all-reduce sweep reported for N > 1")
    ap.add_argument("--optimizer", choices=["adamw", "sgd"], default="adamw",
                    help="DP: adamw (the reference's optax.adamw) or sgd (the fused SGD kernel)")
    ap.add_argument("--autotune", choices=["auto", "off"], default="auto",
                    help="N > 1 on GPUs: validate the step forms (one-launch tile exchange, deep exchange, "
                         "pipeline schedules) against the plain collective form and time them before the "
                         "measured region; the timed run uses the fastest valid one (utils/autotune.py)")
    args = ap.parse_args()
    # a native crash (HIP runtime segfault, abort) prints every thread's Python stack
    faulthandler.enable(all_threads=True)

    # N ranks for --gpus N: start them here (this process never touches the GPU) ...
    LCH.maybe_launch(args.gpus, __file__, sys.argv[1:])
    dev = D.init()
    # ... and never report a job of the wrong size
    LCH.check_world(args.gpus)
    ws = D.world_size()
    if args.steps_per_graph is None:
        # the 2-layer DP / FSDP replay is ONE persistent launch whatever its length; the deep and
        # pipeline graphs hold every step's launches, and 50-step ones measured 0.8 % faster than
        # 150-step ones for the 4-layer step (24.10-24.15k vs 23.90-23.95k, session r5s42)
        two_layer = args.strategy in ("dp", "fsdp") and args.num_layers == 2
        args.steps_per_graph = pick_steps_per_graph(args.steps, 200 if two_layer else 50)
    build = {"dp": build_dp, "fsdp": build_fsdp, "pp": build_pp}[args.strategy]
    on_gpu = dev.type == "cuda"
    sync = (lambda: torch.cuda.synchronize()) if on_gpu else (lambda: None)

    def prepare(tr_, batch_, spg=None):
        """Capture the step the way the timed region replays it (DP always; FSDP and PP
        when their collectives / stage hand-offs are xGMI kernels or N = 1); ``spg``: steps
        per graph (default the run's; the autotune's probes capture 2-step replays)."""
        if not (on_gpu and not args.no_graph and (args.strategy == "dp" or tr_.capturable)):
            return False
        spg = args.steps_per_graph if spg is None else spg
        if args.strategy == "dp":
            tr_.capture(batch_, capture_collectives=args.capture_collectives, steps_per_graph=spg)
        else:
            tr_.capture(batch_, steps_per_graph=spg)
        return True

    n_eager = max(1, min(args.warmup, 3))
    tr = autotune = None
    if ws > 1 and on_gpu and args.autotune != "off":
        # validate the N > 1 step forms against the plain collective form and time them
        # (untimed; utils/autotune.py): the timed run uses the fastest valid one
        tr, batch, desc, autotune = run_autotune(args, dev, build, prepare)
    if tr is None:
        tr, batch, desc = build(args, dev)
        # warmup: eager steps (library load, allocator), then capture + replays
        for _ in range(n_eager):
            tr.step(batch)
        sync()
        if ws > 1 and on_gpu and one_launch_failed(tr, dev):
            # the in-kernel tile exchange passed its start-up self-test but a step's wait timed
            # out on some rank: every rank rebuilds (fresh init) on the three-launch step
            tr.close()
            os.environ["JDT_DP_AHEAD"] = os.environ["JDT_FSDP_AHEAD"] = "0"
            tr, batch, desc = build(args, dev)
            desc["one_launch_fallback"] = "tile exchange wait timed out in the eager steps; three-launch step"
            for _ in range(n_eager):
                tr.step(batch)
            sync()
        use_graph = prepare(tr, batch)
    else:
        use_graph = tr.graph is not None
        n_eager = 0

    def run(n):
        if hasattr(tr, "run_steps"):
            tr.run_steps(batch, n)
        else:
            for _ in range(n):
                tr.step(batch)

    run(max(0, args.warmup - n_eager))
    sync()
    if ws > 1 and on_gpu:
        comm_check(tr, "warmup")
    D.barrier()
    sync()
    t0 = time.perf_counter()
    run(args.steps)
    sync()
    D.barrier()
    if D.is_initialized():
        sync()   # an RCCL barrier is device work; without a process group there is none to wait for
    dt = time.perf_counter() - t0
    if D.is_initialized():
        t = torch.tensor([dt], dtype=torch.float64, device=dev if D.backend() == "nccl" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    if ws > 1 and on_gpu:
        comm_check(tr, "timed steps")
    # per-step latency distribution (separate, untimed pass)
    p50 = p90 = None
    if on_gpu:
        ts = []
        for _ in range(min(50, args.steps)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            tr.step(batch)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        p50, p90 = ts[len(ts) // 2], ts[int(0.9 * len(ts))]
    coll_ms = sweep = None
    if hasattr(tr, "time_collective"):
        coll_ms = tr.time_collective(batch, iters=min(20, max(5, args.steps)))
    if on_gpu and ws > 1 and args.strategy == "dp" and not args.no_comm_sweep:
        sweep = comm_sweep(tr, dev)
    if hasattr(tr, "finalize"):
        tr.finalize()
    m = (tr.gather_metrics() if hasattr(tr, "gather_metrics") else tr.metrics).detach().float().cpu()
    sps = args.steps / dt
    if args.strategy == "dp":
        desc["accum"] = tr.cfg.accum  # the path that actually ran (CPU falls back from "kernel")
        if getattr(tr, "_loop_engine", None) is not None:
            desc["loop_streams"] = tr._loop_engine.n_sets   # minibatch loop on concurrent streams
        # 1-GPU fused step: one run-ahead launch per step (step t's backward + AdamW + step
        # t+1's forward) or the two-launch forward / backward pair
        eng = getattr(tr, "fused", None)
        nh = getattr(eng, "nh", None)   # deep engine: hidden layers
        if getattr(tr, "_ahead", None):
            tx_ = ", gradient tiles all-reduced in the launches" if getattr(tr, "one_launch", False) else ""
            desc["step_launches"] = (f"{2 * nh - 1} (layer-0 run-ahead md_bwd{tx_})" if nh
                                     else _mlp2_launches(eng, tx_, args.steps_per_graph))
        elif eng is not None:
            desc["step_launches"] = ((f"{2 * nh} (md_fwd / md_bwd per layer)" if nh else "2 (mlp2_fwd + mlp2_bwd)")
                                     + (" + xGMI all-reduce/AdamW" if ws > 1 else ""))
    if args.strategy == "fsdp" and getattr(tr, "_ahead", None):
        nh = getattr(tr.fused, "nh", None)
        tx_ = (", partials to the shard owners, sharded AdamW in the launches"
               if getattr(tr, "one_launch", False) else "")
        desc["step_launches"] = (f"{2 * nh - 1} (layer-0 run-ahead md_bwd{tx_})" if nh
                                 else _mlp2_launches(tr.fused, tx_, args.steps_per_graph))
    elif args.strategy == "fsdp" and getattr(tr, "fused", None) is not None and ws > 1:
        nh = getattr(tr.fused, "nh", None)
        desc["step_launches"] = ((f"{2 * nh} (md_fwd / md_bwd per layer)" if nh else "2 (mlp2_fwd + mlp2_bwd)")
                                 + " + xGMI FSDP step collective")
    if args.strategy == "pp":
        desc["single_stage_mode"] = tr.single_stage_mode  # how a 1-stage pipeline ran its microbatches
        desc["stage_streams"] = tr.stage_streams          # concurrent microbatch chains per stage
        desc["data_sync"] = tr.data_sync_mode             # data-axis sync: per W-pass group or one call
        if getattr(tr, "pp_kernel", None) is not None:
            desc["step_launches"] = ("2 (one-GPU chain: every layer a stage of one launch + chip-wide AdamW, "
                                     "parallel/pp_kernel.py)" if tr.S == 1 else
                                     "2 per stage (in-kernel GPipe schedule + chip-wide AdamW, parallel/pp_kernel.py)")
    if D.rank() == 0:
        out = {"metric": METRIC, "value": round(sps, 2), "unit": "steps/s", "n_gpus": ws, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 5), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "bf16", "data": "synthetic (N(0,1) inputs, "
               "uniform int labels; random init)", "config": desc,
               "details": {"p50_ms": p50, "p90_ms": p90, "hipgraph": use_graph, "host_sync": D.host_sync_mode(),
                           "steps_per_graph": (tr.multi[0] if getattr(tr, "multi", None) else 1) if use_graph else 0,
                           "samples_per_s":
                           round(sps * desc["global_batch"], 1), "final_loss": float(m[0] / max(m[1], 1)),
                           "comm": getattr(tr, "comm_backend", None) or D.backend() or "none",
                           "process_group": D.backend() or "none",
                           "xgmi_selftest": getattr(tr, "xgmi_status", "n/a"),
                           "collective_ms_p50": coll_ms, "comm_sweep": sweep,
                           "comm_choice": _comm_choice(), "autotune": autotune}}
        print(json.dumps(out), flush=True)
    D.shutdown()


if __name__ == "__main__":
    main()
